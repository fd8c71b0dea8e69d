// multitrack.cpp -- MultiTrack (lib.rs:72-365) on the device: every track's mono wav, dB
// spectrogram and grey image stay resident in HBM; the only host-side arithmetic is the
// scalar global reduction of update_spec_greys (lib.rs:193-263).
#include "multitrack.hpp"

#include <algorithm>
#include <cmath>
#include <limits>

#include "host_tables.hpp"
#include "wav.hpp"

namespace thesia {

MultiTrack::MultiTrack() = default;

MultiTrack::~MultiTrack() {
    for (auto& kv : plans_) delete kv.second;
}

int MultiTrack::set_setting(float win_ms, size_t t_overlap, size_t f_overlap, int freq_scale,
                            float db_range) {
    if (!tracks_.empty())
        return set_error(THESIA_ERR_INVALID_ARG, "settings must be changed before adding tracks");
    if (win_ms <= 0.f || t_overlap == 0 || f_overlap == 0 || (freq_scale != 0 && freq_scale != 1))
        return set_error(THESIA_ERR_INVALID_ARG, "invalid SpecSetting");
    set_ = Setting{win_ms, t_overlap, f_overlap, freq_scale, db_range};
    return THESIA_OK;
}

static std::string file_name_of(const std::string& p) {
    const size_t s = p.find_last_of('/');
    return s == std::string::npos ? p : p.substr(s + 1);
}

int MultiTrack::add_tracks(const std::vector<uint64_t>& ids, const std::vector<PcmIn>& pcm,
                           int* changed) {
    // 1) validate everything first (the reference returns Err mid-loop, lib.rs:174-177,
    //    leaving earlier tracks inserted without specs; here an error changes nothing)
    struct Pending { uint64_t id; Track tr; };
    std::vector<Pending> pend;
    for (size_t i = 0; i < ids.size(); ++i) {
        const PcmIn& in = pcm[i];
        if (in.channels == 0 || in.sr == 0)
            return set_error(THESIA_ERR_INVALID_ARG, "invalid channels / sample rate");
        Track tr;
        tr.path = in.path;
        tr.sr = in.sr;
        tr.n = in.n_samples;
        track_params(in.sr, set_.win_ms, set_.t_overlap, set_.f_overlap, &tr.win, &tr.hop, &tr.n_fft);
        if (tr.n_fft > 4096 || tr.win == 0)
            return set_error(THESIA_ERR_UNSUPPORTED, "derived n_fft outside [2, 4096]");
        if (stft_n_frames(tr.n, tr.win, tr.hop) == 0)
            return set_error(THESIA_ERR_TOO_SHORT, "track '" + in.path + "' is shorter than the window (lib.rs:413)");
        // upload interleaved PCM and downmix on the device (lib.rs:42)
        DevBuf raw;
        int rc = raw.upload(in.samples, (size_t)in.n_samples * in.channels * sizeof(float));
        if (!rc) rc = tr.wav.alloc((size_t)std::max<uint64_t>(tr.n, 1) * sizeof(float));
        if (rc) return rc;
        if (launch_downmix(raw.p, IN_F32, (int)in.channels, tr.n, tr.wav.as<float>(), default_stream()))
            return set_error(THESIA_ERR_DEVICE, "downmix launch failed");
        THESIA_HIP(hipStreamSynchronize(default_stream()));
        pend.push_back({ids[i], std::move(tr)});
    }
    // 2) insert (lib.rs:178-186)
    for (auto& p : pend) {
        const float sec = (float)p.tr.n / (float)p.tr.sr;
        if (sec > max_sec_) {
            max_sec_ = sec;
            id_max_sec_ = p.id;
        }
        tracks_[p.id] = std::move(p.tr);
    }
    // 3) update_specs (lib.rs:142-168): plans per new sr, then one spectrogram per id
    for (auto& p : pend) {
        int rc = compute_spec(p.id);
        if (rc) return rc;
    }
    // 4) update_spec_greys (lib.rs:193-263)
    return update_spec_greys(changed);
}

int MultiTrack::plan_for(uint32_t sr, const Track& tr, Plan** out) {
    auto it = plans_.find(sr);
    if (it != plans_.end()) {
        *out = it->second;
        return THESIA_OK;
    }
    thesia_plan_desc d{};
    d.sr = sr;
    d.win_length = tr.win;
    d.hop_length = tr.hop;
    d.n_fft = tr.n_fft;
    d.window = nullptr;  // calc_window = hann(win)/n_fft, lib.rs:138-140
    d.output = set_.freq_scale == 1 ? THESIA_OUT_MEL_AMP_DB : THESIA_OUT_AMP_DB;
    d.n_mels = 0;        // calc_mel_fb_default, lib.rs:155
    d.fmin = 0.f;
    d.fmax = -1.f;
    Plan* p = nullptr;
    int rc = plan_create(d, &p);
    if (rc) return rc;
    plans_[sr] = p;
    *out = p;
    return THESIA_OK;
}

int MultiTrack::compute_spec(uint64_t id) {
    Track& tr = tracks_.at(id);
    Plan* plan = nullptr;
    int rc = plan_for(tr.sr, tr, &plan);
    if (rc) return rc;
    tr.bins = plan->row_bins();
    tr.T = stft_n_frames(tr.n, tr.win, tr.hop);
    rc = tr.spec.alloc((size_t)tr.T * tr.bins * sizeof(float));
    if (rc) return rc;
    const uint64_t off = 0, len = tr.n;
    thesia_batch_desc bd{};
    bd.input_format = THESIA_IN_F32;
    bd.channels = 1;
    bd.fold_mono = 0;  // the device wav is already the folded channel sum
    bd.d_input = tr.wav.p;
    bd.track_offset = &off;
    bd.track_len = &len;
    bd.n_tracks = 1;
    bd.d_output = tr.spec.p;
    Batch* b = nullptr;
    rc = batch_create(plan, bd, &b);
    if (rc) return rc;
    // the viewer path computes in the reference's operation order (stftx_kernel): its images
    // are the oracle pipeline's bytes
    rc = batch_set_option(b, THESIA_BATCH_OPT_KERNEL, 9);
    if (!rc) rc = batch_run(b, default_stream());
    if (!rc) {
        hipError_t e = hipStreamSynchronize(default_stream());
        if (e != hipSuccess) rc = set_error(THESIA_ERR_DEVICE, hipGetErrorString(e));
    }
    delete b;
    if (rc) return rc;
    // per-track max / min (lib.rs:197-200); a NaN makes ndarray-stats return Err -> +-inf
    float mx, mn;
    bool nan;
    rc = minmax_device(tr.spec.as<float>(), (uint64_t)tr.T * tr.bins, &mx, &mn, &nan, default_stream());
    if (rc) return rc;
    tr.spec_max = nan ? -INFINITY : mx;
    tr.spec_min = nan ? INFINITY : mn;
    tr.has_grey = false;
    return THESIA_OK;
}

// approx 0.4 AbsDiffEq for f32: (if a > b { a - b } else { b - a }) <= eps
static bool abs_diff_ne(float a, float b, float eps) {
    const float d = a > b ? a - b : b - a;
    return !(d <= eps);
}

int MultiTrack::update_spec_greys(int* changed_out) {
    float mx = -INFINITY, mn = INFINITY;
    for (auto& kv : tracks_) {  // lib.rs:194-207 (f32::max / f32::min ignore NaN)
        mx = fmaxf(mx, kv.second.spec_max);
        mn = fminf(mn, kv.second.spec_min);
    }
    mx = fminf(mx, 0.0f);                       // lib.rs:208
    mn = fmaxf(mn, mx - set_.db_range);         // lib.rs:209
    bool changed = false;
    if (abs_diff_ne(max_db_, mx, 1e-3f)) { max_db_ = mx; changed = true; }  // lib.rs:211-214
    if (abs_diff_ne(min_db_, mn, 1e-3f)) { min_db_ = mn; changed = true; }  // lib.rs:215-218
    uint32_t max_sr = 0;
    for (auto& kv : tracks_) max_sr = std::max(max_sr, kv.second.sr);     // lib.rs:220-224
    if (max_sr_ != max_sr) { max_sr_ = max_sr; changed = true; }
    // lib.rs:230-261 rebuilds every grey when changed; tracks that never got a grey are
    // built too (the reference leaves them missing and get_spec_image then panics).
    for (auto& kv : tracks_) {
        Track& tr = kv.second;
        if (!changed && tr.has_grey) continue;
        float up_ratio;
        if (set_.freq_scale == 1)
            up_ratio = hz_to_mel((float)max_sr_ / 2.0f) / hz_to_mel((float)tr.sr / 2.0f);
        else
            up_ratio = (float)max_sr_ / (float)tr.sr;
        float h = roundf((float)tr.bins * up_ratio);  // display.rs:45
        tr.grey_h = h > 0.f ? (uint32_t)h : 0;
        if (tr.grey_h < tr.bins) tr.grey_h = (uint32_t)tr.bins;
        int rc = tr.grey.alloc((size_t)tr.grey_h * tr.T * sizeof(float));
        if (rc) return rc;
        if (launch_spec_to_grey(tr.spec.as<float>(), (uint32_t)tr.T, (uint32_t)tr.bins, tr.grey_h,
                                max_db_, min_db_, tr.grey.as<float>(), default_stream()))
            return set_error(THESIA_ERR_DEVICE, "spec_to_grey launch failed");
        tr.has_grey = true;
    }
    THESIA_HIP(hipStreamSynchronize(default_stream()));
    if (changed_out) *changed_out = changed ? 1 : 0;
    return THESIA_OK;
}

int MultiTrack::remove_track(uint64_t id, int* changed) {
    auto it = tracks_.find(id);
    if (it == tracks_.end()) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    const uint32_t sr = it->second.sr;
    tracks_.erase(it);
    if (id_max_sec_ == id) {  // lib.rs:269-286
        uint64_t best_id = 0;
        float best = 0.f;
        for (auto& kv : tracks_) {
            const float sec = (float)kv.second.n / (float)kv.second.sr;
            if (sec > best) { best = sec; best_id = kv.first; }
        }
        id_max_sec_ = best_id;
        max_sec_ = best;
    }
    bool used = false;  // lib.rs:287-290 evict per-sr caches
    for (auto& kv : tracks_) used |= kv.second.sr == sr;
    if (!used) {
        auto pit = plans_.find(sr);
        if (pit != plans_.end()) { delete pit->second; plans_.erase(pit); }
    }
    return update_spec_greys(changed);
}

const Track* MultiTrack::find(uint64_t id) const {
    auto it = tracks_.find(id);
    return it == tracks_.end() ? nullptr : &it->second;
}

int MultiTrack::spec_image(uint64_t id, float px_per_sec, uint32_t nheight, std::vector<uint8_t>* out) {
    const Track* tr = find(id);
    if (!tr) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    const float wf = px_per_sec * (float)tr->n / (float)tr->sr;  // lib.rs:296
    const uint32_t nwidth = wf >= 4294967295.0f ? 4294967295u : (wf > 0.f ? (uint32_t)wf : 0u);
    out->assign((size_t)nwidth * nheight * 3, 0);
    if (out->empty()) return THESIA_OK;
    DevBuf rgb;
    int rc = rgb.alloc(out->size());
    if (rc) return rc;
    rc = grey_to_rgb_device(tr->grey.as<float>(), (uint32_t)tr->T, tr->grey_h, nwidth, nheight,
                            rgb.as<uint8_t>(), default_stream());
    if (rc) return rc;
    THESIA_HIP(hipMemcpy(out->data(), rgb.p, out->size(), hipMemcpyDeviceToHost));
    return THESIA_OK;
}

int MultiTrack::wav_image(uint64_t id, float px_per_sec, uint32_t nheight, float amp_min,
                          float amp_max, std::vector<uint8_t>* out) {
    const Track* tr = find(id);
    if (!tr) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    const float wf = px_per_sec * (float)tr->n / (float)tr->sr;  // lib.rs:309
    const uint32_t nwidth = wf >= 4294967295.0f ? 4294967295u : (wf > 0.f ? (uint32_t)wf : 0u);
    out->assign((size_t)nwidth * nheight * 4, 0);
    if (out->empty()) return THESIA_OK;
    DevBuf img;
    int rc = img.alloc(out->size());
    if (rc) return rc;
    int panicked = 0;
    rc = wav_to_image_device(tr->wav.as<float>(), tr->n, nwidth, nheight, amp_min, amp_max,
                             img.as<uint8_t>(), &panicked, default_stream());
    if (rc) return rc;
    THESIA_HIP(hipMemcpy(out->data(), img.p, out->size(), hipMemcpyDeviceToHost));
    return THESIA_OK;
}

int MultiTrack::frequency_hz(uint64_t id, float rel, float* hz) const {
    const Track* tr = find(id);
    if (!tr) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    const float half_sr = (float)tr->sr / 2.0f;  // lib.rs:316
    if (set_.freq_scale == 1) *hz = mel_to_hz(hz_to_mel(half_sr) * rel);
    else *hz = half_sr * rel;
    return THESIA_OK;
}

int MultiTrack::spec_host(uint64_t id, std::vector<float>* out, size_t* T, size_t* bins) const {
    const Track* tr = find(id);
    if (!tr) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    out->resize((size_t)tr->T * tr->bins);
    THESIA_HIP(hipMemcpy(out->data(), tr->spec.p, out->size() * 4, hipMemcpyDeviceToHost));
    *T = tr->T;
    *bins = tr->bins;
    return THESIA_OK;
}

int MultiTrack::grey_host(uint64_t id, std::vector<float>* out, uint32_t* w, uint32_t* h) const {
    const Track* tr = find(id);
    if (!tr) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    out->resize((size_t)tr->T * tr->grey_h);
    THESIA_HIP(hipMemcpy(out->data(), tr->grey.p, out->size() * 4, hipMemcpyDeviceToHost));
    *w = (uint32_t)tr->T;
    *h = tr->grey_h;
    return THESIA_OK;
}

std::string MultiTrack::filename_of(const Track& tr) { return file_name_of(tr.path); }

}  // namespace thesia
