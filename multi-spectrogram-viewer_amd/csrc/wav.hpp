// wav.hpp -- host WAV decoding (hound semantics, audio.rs:9-37).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace thesia {

struct WavData {
    uint32_t sr = 0;
    uint32_t channels = 0;
    std::vector<float> samples;  // interleaved [n][ch]
};

// Returns THESIA_OK or an error code with *err set (message like Rust's io::Error).
int read_wav(const std::string& path, WavData* out, std::string* err);

}  // namespace thesia
