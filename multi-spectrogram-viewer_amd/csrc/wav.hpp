// wav.hpp -- WAV parsing with hound 3.4 semantics (audio.rs:9-37). The sample bytes stay in
// their file encoding: MultiTrack uploads them as they are (1-4 B per sample) and the device
// converts and downmixes (launch_decode_downmix); decode_pcm_f32 is the host restatement of
// that conversion (thesia_open_audio_file).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace thesia {

// sample encodings of a WAV data chunk (bytes per sample 4, 1, 2, 3, 4)
enum PcmKind { PCM_F32 = 0, PCM_U8 = 1, PCM_S16 = 2, PCM_S24 = 3, PCM_S32 = 4 };

inline int pcm_bytes(int kind) {
    return kind == PCM_U8 ? 1 : kind == PCM_S16 ? 2 : kind == PCM_S24 ? 3 : 4;
}

struct WavData {
    uint32_t sr = 0;
    uint32_t channels = 0;
    uint32_t bits = 0;      // bits_per_sample of the fmt chunk
    int kind = PCM_F32;
    uint64_t n_frames = 0;  // samples per channel (whole frames, audio.rs:32-34)
    std::vector<uint8_t> raw;  // channel-interleaved samples, n_frames * channels * pcm_bytes
};

// Returns THESIA_OK or an error code with *err set (message like Rust's io::Error).
int read_wav(const std::string& path, WavData* out, std::string* err);

// audio.rs:15-19: integer x -> (x as f32) / (2^(bits-1) as f32); 8-bit WAV is unsigned
// (x - 128); float samples as they are. Returns the divisor (1 for float).
float pcm_scale(int kind, uint32_t bits);
void decode_pcm_f32(const uint8_t* raw, int kind, float scale, uint64_t n_samples, float* out);

}  // namespace thesia
