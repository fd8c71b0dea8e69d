// multitrack.hpp -- the viewer's stateful surface (lib.rs:72-365) over the device engine.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "engine.hpp"

namespace thesia {

struct Track {  // AudioTrack (lib.rs:30-37) + per-track caches (lib.rs:78-79)
    std::string path;
    uint32_t sr = 0;
    uint64_t n = 0;  // samples after downmix
    size_t win = 0, hop = 0, n_fft = 0;
    // the mono wav and the dB spectrogram live in buffers shared by the tracks of one
    // add_tracks call and sample rate (one batched launch), freed with their last track
    std::shared_ptr<DevBuf> wav_pool, spec_pool;
    uint64_t wav_off = 0, spec_off = 0;  // float offsets into the pools
    size_t T = 0, bins = 0;
    float spec_max = -INFINITY, spec_min = INFINITY;
    DevBuf grey;     // [grey_h, T]
    uint32_t grey_h = 0;
    bool has_grey = false;
    const float* wav() const { return wav_pool->as<float>() + wav_off; }
    const float* spec() const { return spec_pool->as<float>() + spec_off; }
};

// One new track for add_tracks: interleaved samples [n_frames][channels] in their file
// encoding (kind: wav.hpp PcmKind; f32 for the in-memory entry point), uploaded as they are
// and converted + downmixed on the device.
struct PcmIn {
    const void* data = nullptr;
    int kind = 0;          // PCM_F32
    float scale = 1.0f;    // integer divisor 2^(bits-1) (audio.rs:15-19)
    uint64_t n_samples = 0;  // per channel
    uint32_t channels = 0, sr = 0;
    std::string path;
};

// a page-locked host buffer for one add_tracks call (hipHostFree after the library stream drains)
struct PinnedTmp {
    void* p = nullptr;
    PinnedTmp() = default;
    PinnedTmp(const PinnedTmp&) = delete;
    PinnedTmp& operator=(const PinnedTmp&) = delete;
    ~PinnedTmp();
};

class MultiTrack {
  public:
    struct Setting {  // SpecSetting, lib.rs:64-70 / defaults lib.rs:93-99
        float win_ms = 40.f;
        size_t t_overlap = 4, f_overlap = 1;
        int freq_scale = 1;  // 0 Linear, 1 Mel
        float db_range = 120.f;
    };
    MultiTrack();
    ~MultiTrack();
    int set_setting(float win_ms, size_t t_overlap, size_t f_overlap, int freq_scale, float db_range);
    // 0 (default): spectrograms from the reference-order kernel (images = the oracle pipeline's
    // bytes); 1: the batch engine's automatic streaming kernel (tolerance contract, SURVEY §8c:
    // end to end <= 1 LSB on <= 1e-4 of the pixels). Applies to the tracks added afterwards.
    void set_fast(bool fast) { fast_ = fast; }
    bool fast() const { return fast_; }
    int add_tracks(const std::vector<uint64_t>& ids, const std::vector<PcmIn>& pcm, int* changed);
    int remove_track(uint64_t id, int* changed);
    // images straight into the caller's buffer: *needed = bytes; THESIA_ERR_BUFFER_TOO_SMALL
    // (nothing computed) when cap is short
    int spec_image(uint64_t id, float px_per_sec, uint32_t nheight, uint8_t* out, size_t cap,
                   size_t* needed);
    int wav_image(uint64_t id, float px_per_sec, uint32_t nheight, float amp_min, float amp_max,
                  uint8_t* out, size_t cap, size_t* needed);
    int wav_host(uint64_t id, std::vector<float>* out) const;
    int frequency_hz(uint64_t id, float rel, float* hz) const;
    int spec_host(uint64_t id, std::vector<float>* out, size_t* T, size_t* bins) const;
    int grey_host(uint64_t id, std::vector<float>* out, uint32_t* w, uint32_t* h) const;
    const Track* find(uint64_t id) const;
    static std::string filename_of(const Track& tr);
    float max_db() const { return max_db_; }
    float min_db() const { return min_db_; }
    float max_sec() const { return max_sec_; }
    size_t size() const { return tracks_.size(); }
    // device bytes the tracks hold: their wav / spectrogram buffers (shared ones once) and greys
    size_t device_bytes() const;
    // page-locked host staging for add_tracks' file reads (this handle's, kept between calls up
    // to kStageKeep bytes; a larger call gets a buffer of its own in *tmp, freed when *tmp goes):
    // nullptr if it cannot be had (the files are then read into pageable memory)
    static constexpr size_t kStageKeep = size_t(256) << 20;
    uint8_t* staging(size_t bytes, PinnedTmp* tmp);

  private:
    int make_plan(const Track& tr, Plan** out) const;
    int update_spec_greys(int* changed);
    void compact_pools();

    Setting set_;
    bool fast_ = false;
    std::map<uint64_t, Track> tracks_;
    std::map<uint32_t, Plan*> plans_;  // windows / mel_fbs per sr (lib.rs:76-77)
    float max_db_ = -INFINITY, min_db_ = INFINITY, max_sec_ = 0.f;
    uint64_t id_max_sec_ = 0;
    uint32_t max_sr_ = 0;
    DevBuf img_;  // image scratch (grow-only)
    DevBuf raw_;  // add_tracks' upload scratch (grow-only: no hipMalloc / hipFree per call)
    uint8_t* stage_ = nullptr;  // hipHostMalloc'd, stage_bytes_
    size_t stage_bytes_ = 0;
};

}  // namespace thesia
