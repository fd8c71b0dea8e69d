// wav.hpp -- WAV parsing with hound 3.4 semantics (audio.rs:9-37). The sample bytes stay in
// their file encoding: MultiTrack uploads them as they are (1-4 B per sample) and the device
// converts and downmixes (launch_decode_downmix); decode_pcm_f32 is the host restatement of
// that conversion (thesia_open_audio_file).
#pragma once

#include <cstdint>
#include <string>
#include <memory>
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
    // the whole file, read once (no copy of its data chunk): the channel-interleaved samples,
    // n_frames * channels * pcm_bytes, start at base + data_off; `file` owns base unless the
    // file was read into a caller's buffer (read_wav_into)
    std::unique_ptr<uint8_t[]> file;
    const uint8_t* base = nullptr;
    size_t file_len = 0, data_off = 0;
    const uint8_t* samples() const { return base + data_off; }
};

// Returns THESIA_OK or an error code with *err set (message like Rust's io::Error).
int read_wav(const std::string& path, WavData* out, std::string* err);
// The file's size in bytes (0 when unknown), for sizing a read_wav_into buffer.
int wav_file_size(const std::string& path, size_t* size, std::string* err);
// read_wav into dst[0, cap) (e.g. page-locked staging for the upload): out->samples() then points
// into dst; a file that no longer fits is read as read_wav does (into a buffer out owns).
int read_wav_into(const std::string& path, uint8_t* dst, size_t cap, WavData* out, std::string* err);
// The WAV parse of file[0, len) (out->base = file; nothing is copied).
int parse_wav(const uint8_t* file, size_t len, WavData* out, std::string* err);

// audio.rs:15-19: integer x -> (x as f32) / (2^(bits-1) as f32); 8-bit WAV is unsigned
// (x - 128); float samples as they are. Returns the divisor (1 for float).
float pcm_scale(int kind, uint32_t bits);
void decode_pcm_f32(const uint8_t* raw, int kind, float scale, uint64_t n_samples, float* out);

}  // namespace thesia
