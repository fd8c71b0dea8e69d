// multitrack.hpp -- the viewer's stateful surface (lib.rs:72-365) over the device engine.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "engine.hpp"

namespace thesia {

struct Track {  // AudioTrack (lib.rs:30-37) + per-track caches (lib.rs:78-79)
    std::string path;
    uint32_t sr = 0;
    uint64_t n = 0;  // samples after downmix
    size_t win = 0, hop = 0, n_fft = 0;
    DevBuf wav;      // mono f32 [n]
    DevBuf spec;     // dB [T, bins]
    size_t T = 0, bins = 0;
    float spec_max = -INFINITY, spec_min = INFINITY;
    DevBuf grey;     // [grey_h, T]
    uint32_t grey_h = 0;
    bool has_grey = false;
};

struct PcmIn {
    const float* samples = nullptr;  // interleaved [n][ch]
    uint64_t n_samples = 0;          // per channel
    uint32_t channels = 0, sr = 0;
    std::string path;
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
    int add_tracks(const std::vector<uint64_t>& ids, const std::vector<PcmIn>& pcm, int* changed);
    int remove_track(uint64_t id, int* changed);
    int spec_image(uint64_t id, float px_per_sec, uint32_t nheight, std::vector<uint8_t>* out);
    int wav_image(uint64_t id, float px_per_sec, uint32_t nheight, float amp_min, float amp_max,
                  std::vector<uint8_t>* out);
    int frequency_hz(uint64_t id, float rel, float* hz) const;
    int spec_host(uint64_t id, std::vector<float>* out, size_t* T, size_t* bins) const;
    int grey_host(uint64_t id, std::vector<float>* out, uint32_t* w, uint32_t* h) const;
    const Track* find(uint64_t id) const;
    static std::string filename_of(const Track& tr);
    float max_db() const { return max_db_; }
    float min_db() const { return min_db_; }
    float max_sec() const { return max_sec_; }
    size_t size() const { return tracks_.size(); }

  private:
    int plan_for(uint32_t sr, const Track& tr, Plan** out);
    int compute_spec(uint64_t id);
    int update_spec_greys(int* changed);

    Setting set_;
    std::map<uint64_t, Track> tracks_;
    std::map<uint32_t, Plan*> plans_;  // windows / mel_fbs per sr (lib.rs:76-77)
    float max_db_ = -INFINITY, min_db_ = INFINITY, max_sec_ = 0.f;
    uint64_t id_max_sec_ = 0;
    uint32_t max_sr_ = 0;
};

}  // namespace thesia
