// multitrack.cpp -- MultiTrack (lib.rs:72-365) on the device: every track's mono wav, dB
// spectrogram and grey image stay resident in HBM; the only host-side arithmetic is the
// scalar global reduction of update_spec_greys (lib.rs:193-263).
#include "multitrack.hpp"

#include <algorithm>
#include <cmath>
#include <limits>

#include "host_tables.hpp"
#include "kernels.hpp"
#include "wav.hpp"

namespace thesia {

MultiTrack::MultiTrack() = default;

MultiTrack::~MultiTrack() {
    for (auto& kv : plans_) delete kv.second;
    if (stage_) (void)hipHostFree(stage_);
}

PinnedTmp::~PinnedTmp() {
    if (p) {
        (void)hipStreamSynchronize(default_stream());  // the call's uploads may still read it
        (void)hipHostFree(p);
    }
}

uint8_t* MultiTrack::staging(size_t bytes, PinnedTmp* tmp) {
    // an add_tracks that failed after enqueuing its uploads returned before its synchronisation:
    // its copies may still read the staging (the stream is idle otherwise)
    if (hipStreamSynchronize(default_stream()) != hipSuccess) return nullptr;
    if (bytes <= stage_bytes_) return stage_;
    if (stage_) (void)hipHostFree(stage_);
    stage_ = nullptr;
    stage_bytes_ = 0;
    void* p = nullptr;
    if (bytes > kStageKeep) {
        // a call larger than the handle keeps pinned between calls: a buffer of its own, freed
        // (after the stream drains) when the call returns
        if (!tmp || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
        tmp->p = p;
        return static_cast<uint8_t*>(p);
    }
    // headroom: a session adds files of similar sizes
    const size_t want = std::min(bytes + bytes / 4, kStageKeep);
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return nullptr;
    stage_ = static_cast<uint8_t*>(p);
    stage_bytes_ = want;
    return stage_;
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

int MultiTrack::make_plan(const Track& tr, Plan** out) const {
    thesia_plan_desc d{};
    d.sr = tr.sr;
    d.win_length = tr.win;
    d.hop_length = tr.hop;
    d.n_fft = tr.n_fft;
    d.window = nullptr;  // calc_window = hann(win)/n_fft, lib.rs:138-140
    d.output = set_.freq_scale == 1 ? THESIA_OUT_MEL_AMP_DB : THESIA_OUT_AMP_DB;
    d.n_mels = 0;        // calc_mel_fb_default, lib.rs:155
    d.fmin = 0.f;
    d.fmax = -1.f;
    return plan_create(d, out);
}

int MultiTrack::add_tracks(const std::vector<uint64_t>& ids, const std::vector<PcmIn>& pcm,
                           int* changed) {
    const hipStream_t s = default_stream();
    // the call's uploads read the caller's sample buffers: whatever path returns, s has drained
    struct Drain {
        hipStream_t s;
        ~Drain() { (void)hipStreamSynchronize(s); }
    } drain{s};
    // 1) validate every new track before any device work (the reference returns Err mid-loop,
    //    lib.rs:174-177, leaving earlier tracks inserted without specs; here an error at any
    //    step changes nothing)
    std::vector<Track> nt(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
        const PcmIn& in = pcm[i];
        if (in.channels == 0 || in.sr == 0)
            return set_error(THESIA_ERR_INVALID_ARG, "invalid channels / sample rate");
        if (in.kind < PCM_F32 || in.kind > PCM_S32 || (in.n_samples && !in.data))
            return set_error(THESIA_ERR_INVALID_ARG, "invalid sample buffer");
        Track& tr = nt[i];
        tr.path = in.path;
        tr.sr = in.sr;
        tr.n = in.n_samples;
        track_params(in.sr, set_.win_ms, set_.t_overlap, set_.f_overlap, &tr.win, &tr.hop, &tr.n_fft);
        if (tr.n_fft > 4096 || tr.win == 0)
            return set_error(THESIA_ERR_UNSUPPORTED, "derived n_fft outside [2, 4096]");
        if (stft_n_frames(tr.n, tr.win, tr.hop) == 0)
            return set_error(THESIA_ERR_TOO_SHORT, "track '" + in.path + "' is shorter than the window (lib.rs:413)");
    }
    // 2) per sample rate (update_specs, lib.rs:142-168): the new tracks' samples uploaded in
    //    their file encoding (1-4 B per sample), converted + downmixed on the device into one
    //    mono pool, one Batch over all of them (the reference-order kernel) into one
    //    spectrogram pool; a single synchronisation for the whole call
    std::map<uint32_t, std::vector<size_t>> by_sr;
    for (size_t i = 0; i < nt.size(); ++i) by_sr[nt[i].sr].push_back(i);
    std::map<uint32_t, std::unique_ptr<Plan>> new_plans;
    struct Group {
        std::unique_ptr<Batch> batch;
        std::vector<uint64_t> off, len;
        const float* spec = nullptr;
        size_t bins = 0;
        std::vector<size_t> idx;
    };
    std::vector<Group> groups;
    std::vector<std::unique_ptr<DevBuf>> big_raws;  // uploads of calls beyond kStageKeep
    // per-track (max, min, NaN) of the new rows (lib.rs:197-200), left by the spectrogram launches
    // themselves (Batch::range: folded into kernel 7's amp-dB epilogue, one pass over the rows for
    // the other kinds), 3 int32 per track in group order
    DevBuf rng;
    {
        const int rc = rng.alloc(std::max<size_t>(nt.size(), 1) * 3 * sizeof(int));
        if (rc) return rc;
    }
    size_t t_rng = 0;
    for (auto& [sr, idx] : by_sr) {
        Plan* plan = nullptr;
        auto pit = plans_.find(sr);
        if (pit != plans_.end()) {
            plan = pit->second;
        } else {
            int rc = make_plan(nt[idx[0]], &plan);
            if (rc) return rc;
            new_plans[sr].reset(plan);
        }
        Group g;
        g.idx = idx;
        uint64_t rb = 0, wf = 0, T_all = 0;
        std::vector<uint64_t> roff(idx.size());
        for (size_t k = 0; k < idx.size(); ++k) {
            const PcmIn& in = pcm[idx[k]];
            roff[k] = rb;
            rb += (in.n_samples * in.channels * pcm_bytes(in.kind) + 255) & ~uint64_t(255);
            g.off.push_back(wf);
            g.len.push_back(nt[idx[k]].n);
            wf += (nt[idx[k]].n + 63) & ~uint64_t(63);
            T_all += stft_n_frames(nt[idx[k]].n, nt[idx[k]].win, nt[idx[k]].hop);
        }
        // the upload scratch is the handle's, grow-only (a hipFree synchronises and costs
        // ~0.16 ms); a later group's copies are ordered behind this group's decodes on s
        // (a call larger than kStageKeep gets a scratch of its own, freed after the call's sync)
        if (rb > kStageKeep) big_raws.push_back(std::make_unique<DevBuf>());
        DevBuf& raw = rb > kStageKeep ? *big_raws.back() : raw_;
        auto wav = std::make_shared<DevBuf>();
        auto spec = std::make_shared<DevBuf>();
        g.bins = plan->row_bins();
        int rc = raw.bytes >= rb && raw.p ? 0 : raw.alloc(std::max<uint64_t>(rb, 1));
        if (!rc) rc = wav->alloc(std::max<uint64_t>(wf, 1) * sizeof(float));
        if (!rc) rc = spec->alloc(std::max<uint64_t>(T_all * g.bins, 1) * sizeof(float));
        if (rc) return rc;
        // uploads: async copies on the library stream, page-locked sources (the file path's
        // staging) and pageable ones (decoded PCM handed in by the caller) alike -- stream-ordered
        // with the decodes behind them (round 6 probe); every return below runs
        // after `drain` has synchronised s, so no copy outlives the caller's buffers
        for (size_t k = 0; k < idx.size(); ++k) {
            const PcmIn& in = pcm[idx[k]];
            const uint64_t bytes = in.n_samples * in.channels * pcm_bytes(in.kind);
            uint8_t* dst = raw.as<uint8_t>() + roff[k];
            if (!bytes) continue;
            THESIA_HIP(hipMemcpyAsync(dst, in.data, bytes, hipMemcpyHostToDevice, s));
        }
        for (size_t k = 0; k < idx.size(); ++k) {
            const PcmIn& in = pcm[idx[k]];
            uint8_t* dst = raw.as<uint8_t>() + roff[k];
            if (launch_decode_downmix(dst, in.kind, in.scale, (int)in.channels, in.n_samples,
                                      wav->as<float>() + g.off[k], s))
                return set_error(THESIA_ERR_DEVICE, "decode / downmix launch failed");
        }
        thesia_batch_desc bd{};
        bd.input_format = THESIA_IN_F32;
        bd.channels = 1;
        bd.fold_mono = 0;  // the pool holds the folded channel sums already
        bd.d_input = wav->p;
        bd.track_offset = g.off.data();
        bd.track_len = g.len.data();
        bd.n_tracks = idx.size();
        bd.d_output = spec->p;
        Batch* b = nullptr;
        rc = batch_create(plan, bd, &b);
        if (rc) return rc;
        g.batch.reset(b);
        // the viewer path computes in the reference's operation order: kernel 7 (stftq / stftr,
        // round 6: at the viewer's own geometries too, each frame loading its samples) where it
        // runs the plan, else stftx (one wave per frame); its images are the oracle pipeline's
        // bytes. Opt-in (set_fast): the automatic streaming kernel (stft3 at the viewer
        // geometries; stft5 for the 48 kHz rows of batches of >= 400 000 frames), held to the e2e
        // contract relative to the reference's own f32 error (tests/test_gpu_parity.py
        // _check_multitrack)
        rc = batch_set_option(b, THESIA_BATCH_OPT_KERNEL, fast_ ? 0 : b->kr_ok ? 7 : 9);
        if (!rc) rc = batch_set_option(b, THESIA_BATCH_OPT_RANGE, (int64_t)(uintptr_t)(rng.as<int>() + 3 * t_rng));
        t_rng += idx.size();
        if (!rc) rc = batch_run(b, s);
        if (rc) return rc;
        g.spec = spec->as<float>();
        for (size_t k = 0; k < idx.size(); ++k) {
            Track& tr = nt[idx[k]];
            tr.wav_pool = wav;
            tr.wav_off = g.off[k];
            tr.spec_pool = spec;
            tr.bins = g.bins;
            tr.T = b->frame0[k + 1] - b->frame0[k];
            tr.spec_off = b->frame0[k] * g.bins;
        }
        groups.push_back(std::move(g));
    }
    {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return set_error(THESIA_ERR_DEVICE, hipGetErrorString(e));
    }
    // 3) per-track max / min (lib.rs:197-200; a NaN makes ndarray-stats return Err -> +-inf):
    //    the ranges the launches left, one readback
    {
        std::vector<float> mx(nt.size()), mn(nt.size());
        std::vector<int> nan(nt.size());
        int rc = ranges_read(rng.as<int>(), nt.size(), mx.data(), mn.data(), nan.data(), s);
        if (rc) return rc;
        size_t t = 0;
        for (const Group& g : groups)
            for (size_t i : g.idx) {
                nt[i].spec_max = nan[t] ? -INFINITY : mx[t];
                nt[i].spec_min = nan[t] ? INFINITY : mn[t];
                ++t;
            }
    }
    groups.clear();
    // 4) insert (lib.rs:178-186), then update_spec_greys (lib.rs:193-263); if that fails
    //    (device memory for the grey images) the insertion is rolled back
    std::map<uint64_t, std::unique_ptr<Track>> undo;  // id -> replaced track (null: was absent)
    const float max_sec0 = max_sec_;
    const uint64_t id_max_sec0 = id_max_sec_;
    for (size_t i = 0; i < ids.size(); ++i) {
        const uint64_t id = ids[i];
        if (!undo.count(id)) {
            auto it = tracks_.find(id);
            undo[id] = it == tracks_.end() ? nullptr : std::make_unique<Track>(std::move(it->second));
        }
        const float sec = (float)nt[i].n / (float)nt[i].sr;
        if (sec > max_sec_) {
            max_sec_ = sec;
            id_max_sec_ = id;
        }
        tracks_[id] = std::move(nt[i]);
    }
    for (auto& [sr, p] : new_plans) plans_[sr] = p.release();
    int rc = update_spec_greys(changed);
    if (rc) {
        for (auto& [id, old] : undo) {
            if (old) tracks_[id] = std::move(*old);
            else tracks_.erase(id);
        }
        for (auto it = plans_.begin(); it != plans_.end();) {
            bool used = false;
            for (auto& kv : tracks_) used |= kv.second.sr == it->first;
            if (!used) { delete it->second; it = plans_.erase(it); }
            else ++it;
        }
        max_sec_ = max_sec0;
        id_max_sec_ = id_max_sec0;
    }
    return rc;
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
    float max_db = max_db_, min_db = min_db_;
    if (abs_diff_ne(max_db, mx, 1e-3f)) { max_db = mx; changed = true; }  // lib.rs:211-214
    if (abs_diff_ne(min_db, mn, 1e-3f)) { min_db = mn; changed = true; }  // lib.rs:215-218
    uint32_t max_sr = 0;
    for (auto& kv : tracks_) max_sr = std::max(max_sr, kv.second.sr);     // lib.rs:220-224
    if (max_sr_ != max_sr) changed = true;
    // lib.rs:230-261 rebuilds every grey when changed; tracks that never got a grey are
    // built too (the reference leaves them missing and get_spec_image then panics). Every
    // new grey buffer is allocated before any state changes (a failure leaves all as it was).
    struct Job { Track* tr; uint32_t h; DevBuf buf; };
    std::vector<Job> jobs;
    for (auto& kv : tracks_) {
        Track& tr = kv.second;
        if (!changed && tr.has_grey) continue;
        float up_ratio;
        if (set_.freq_scale == 1)
            up_ratio = hz_to_mel((float)max_sr / 2.0f) / hz_to_mel((float)tr.sr / 2.0f);
        else
            up_ratio = (float)max_sr / (float)tr.sr;
        const float h = roundf((float)tr.bins * up_ratio);  // display.rs:45
        uint32_t gh = h > 0.f ? (uint32_t)h : 0;
        if (gh < tr.bins) gh = (uint32_t)tr.bins;
        jobs.push_back(Job{&tr, gh, DevBuf()});
        int rc = jobs.back().buf.alloc(std::max<size_t>((size_t)gh * tr.T, 1) * sizeof(float));
        if (rc) return rc;
    }
    // every grey is formed into its new buffer first; the range, max_sr and the tracks' greys
    // are committed only once all of them succeeded (a failure leaves the old state whole)
    for (Job& j : jobs)
        if (launch_spec_to_grey(j.tr->spec(), (uint32_t)j.tr->T, (uint32_t)j.tr->bins, j.h, max_db,
                                min_db, j.buf.as<float>(), default_stream()))
            return set_error(THESIA_ERR_DEVICE, "spec_to_grey launch failed");
    THESIA_HIP(hipStreamSynchronize(default_stream()));
    max_db_ = max_db;
    min_db_ = min_db;
    max_sr_ = max_sr;
    for (Job& j : jobs) {
        j.tr->grey = std::move(j.buf);
        j.tr->grey_h = j.h;
        j.tr->has_grey = true;
    }
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
    compact_pools();
    bool used = false;  // lib.rs:287-290 evict per-sr caches
    for (auto& kv : tracks_) used |= kv.second.sr == sr;
    if (!used) {
        auto pit = plans_.find(sr);
        if (pit != plans_.end()) { delete pit->second; plans_.erase(pit); }
    }
    return update_spec_greys(changed);
}

// The tracks of one add_tracks call and sample rate share their wav / spectrogram buffers (one
// batched launch wrote them). When removals leave a buffer at most half used, its surviving
// tracks move into buffers of their own (device-to-device copies) and the pool is freed, so a
// long session does not keep removed tracks' samples in HBM (the reference frees per track,
// lib.rs:265-292). Best effort: if an allocation fails the tracks keep sharing.
void MultiTrack::compact_pools() {
    struct Use { size_t live = 0; std::vector<Track*> tracks; };
    std::map<DevBuf*, Use> wav_use, spec_use;
    for (auto& kv : tracks_) {
        Track& tr = kv.second;
        if (tr.wav_pool) {
            Use& u = wav_use[tr.wav_pool.get()];
            u.live += tr.n * sizeof(float);
            u.tracks.push_back(&tr);
        }
        if (tr.spec_pool) {
            Use& u = spec_use[tr.spec_pool.get()];
            u.live += (size_t)tr.T * tr.bins * sizeof(float);
            u.tracks.push_back(&tr);
        }
    }
    hipStream_t s = default_stream();
    bool copied = false;
    auto move_out = [&](std::map<DevBuf*, Use>& use, bool wav) {
        for (auto& [pool, u] : use) {
            if (u.live * 2 > pool->bytes) continue;
            for (Track* tr : u.tracks) {
                auto nb = std::make_shared<DevBuf>();
                const size_t bytes = wav ? tr->n * sizeof(float) : (size_t)tr->T * tr->bins * sizeof(float);
                if (nb->alloc(std::max<size_t>(bytes, 4))) return;
                const float* src = wav ? tr->wav() : tr->spec();
                if (bytes && hipMemcpyAsync(nb->p, src, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return;
                copied = true;
                if (wav) { tr->wav_pool = nb; tr->wav_off = 0; }
                else { tr->spec_pool = nb; tr->spec_off = 0; }
            }
        }
    };
    move_out(wav_use, true);
    move_out(spec_use, false);
    // the old pools are released once the last shared_ptr goes (stream-ordered frees behind the
    // copies); their bytes then leave the library pool's reserve too (trim_pool synchronises)
    if (copied) (void)trim_pool();
}

size_t MultiTrack::device_bytes() const {
    std::map<const DevBuf*, size_t> pools;
    size_t greys = 0;
    for (auto& kv : tracks_) {
        const Track& tr = kv.second;
        if (tr.wav_pool) pools[tr.wav_pool.get()] = tr.wav_pool->bytes;
        if (tr.spec_pool) pools[tr.spec_pool.get()] = tr.spec_pool->bytes;
        greys += tr.grey.bytes;
    }
    size_t b = greys;
    for (auto& kv : pools) b += kv.second;
    return b;
}

const Track* MultiTrack::find(uint64_t id) const {
    auto it = tracks_.find(id);
    return it == tracks_.end() ? nullptr : &it->second;
}

static uint32_t image_width(float px_per_sec, const Track& tr) {  // lib.rs:296, :309
    const float wf = px_per_sec * (float)tr.n / (float)tr.sr;
    return wf >= 4294967295.0f ? 4294967295u : (wf > 0.f ? (uint32_t)wf : 0u);
}

int MultiTrack::spec_image(uint64_t id, float px_per_sec, uint32_t nheight, uint8_t* out,
                           size_t cap, size_t* needed) {
    const Track* tr = find(id);
    if (!tr) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    const size_t bytes = (size_t)image_width(px_per_sec, *tr) * nheight * 3;
    if (needed) *needed = bytes;
    if (bytes == 0) return THESIA_OK;
    if (!out || cap < bytes) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "output buffer too small");
    if (img_.bytes < bytes) {
        img_.release();
        int rc = img_.alloc(bytes);
        if (rc) return rc;
    }
    int rc = grey_to_rgb_device(tr->grey.as<float>(), (uint32_t)tr->T, tr->grey_h,
                                image_width(px_per_sec, *tr), nheight, img_.as<uint8_t>(), default_stream());
    if (rc) return rc;
    THESIA_HIP(copy_ordered(out, img_.p, bytes, hipMemcpyDeviceToHost));
    return THESIA_OK;
}

int MultiTrack::wav_image(uint64_t id, float px_per_sec, uint32_t nheight, float amp_min,
                          float amp_max, uint8_t* out, size_t cap, size_t* needed) {
    const Track* tr = find(id);
    if (!tr) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    const uint32_t nwidth = image_width(px_per_sec, *tr);
    const size_t bytes = (size_t)nwidth * nheight * 4;
    if (needed) *needed = bytes;
    if (bytes == 0) return THESIA_OK;
    if (!out || cap < bytes) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "output buffer too small");
    if (img_.bytes < bytes) {
        img_.release();
        int rc = img_.alloc(bytes);
        if (rc) return rc;
    }
    int panicked = 0;
    int rc = wav_to_image_device(tr->wav(), tr->n, nwidth, nheight, amp_min, amp_max,
                                 img_.as<uint8_t>(), &panicked, default_stream());
    if (rc) return rc;
    THESIA_HIP(copy_ordered(out, img_.p, bytes, hipMemcpyDeviceToHost));
    if (panicked)
        return set_error(THESIA_ERR_PANIC, "the reference panics for these arguments (display.rs:95-108); "
                                           "the image is written with the column clamped");
    return THESIA_OK;
}

int MultiTrack::wav_host(uint64_t id, std::vector<float>* out) const {
    const Track* tr = find(id);
    if (!tr) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    out->resize(tr->n);
    if (tr->n) THESIA_HIP(copy_ordered(out->data(), tr->wav(), tr->n * 4, hipMemcpyDeviceToHost));
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
    THESIA_HIP(copy_ordered(out->data(), tr->spec(), out->size() * 4, hipMemcpyDeviceToHost));
    *T = tr->T;
    *bins = tr->bins;
    return THESIA_OK;
}

int MultiTrack::grey_host(uint64_t id, std::vector<float>* out, uint32_t* w, uint32_t* h) const {
    const Track* tr = find(id);
    if (!tr) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    out->resize((size_t)tr->T * tr->grey_h);
    THESIA_HIP(copy_ordered(out->data(), tr->grey.p, out->size() * 4, hipMemcpyDeviceToHost));
    *w = (uint32_t)tr->T;
    *h = tr->grey_h;
    return THESIA_OK;
}

std::string MultiTrack::filename_of(const Track& tr) { return file_name_of(tr.path); }

}  // namespace thesia
