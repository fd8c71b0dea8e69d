// wav.cpp -- WAV parsing with hound 3.4 semantics (audio.rs:9-37): integer PCM converts as
// (x as f32) / 2^(bits-1) (8-bit WAV unsigned, x - 128), float PCM is taken as is, samples stay
// channel-interleaved. Parsing keeps the file's sample bytes (the device converts them);
// decode_pcm_f32 is the host conversion. The reference's rodio fallback (FLAC / Vorbis,
// audio.rs:21-31) is out of scope: such files return THESIA_ERR_UNSUPPORTED.
#include "wav.hpp"

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>

#include "../../include/thesia.h"

namespace thesia {

static uint32_t rd32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

float pcm_scale(int kind, uint32_t bits) {
    return kind == PCM_F32 ? 1.0f : (float)(1ull << (bits - 1));
}

void decode_pcm_f32(const uint8_t* raw, int kind, float scale, uint64_t n, float* out) {
    const int bps = pcm_bytes(kind);
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* p = raw + i * bps;
        if (kind == PCM_F32) {
            std::memcpy(&out[i], p, 4);
            continue;
        }
        int32_t v;
        if (kind == PCM_U8) v = (int32_t)p[0] - 128;
        else if (kind == PCM_S16) v = (int16_t)rd16(p);
        else if (kind == PCM_S24) v = (int32_t)((uint32_t)p[0] << 8 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 24) >> 8;
        else v = (int32_t)rd32(p);
        out[i] = (float)v / scale;
    }
}

static int io_error(std::string* err) {
    const int e = errno;
    *err = std::string(std::strerror(e)) + " (os error " + std::to_string(e) + ")";
    return THESIA_ERR_IO;
}

int wav_file_size(const std::string& path, size_t* size, std::string* err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return io_error(err);
    long sz = -1;
    if (std::fseek(f, 0, SEEK_END) == 0) sz = std::ftell(f);
    std::fclose(f);
    *size = sz > 0 ? (size_t)sz : 0;
    return THESIA_OK;
}

int read_wav_into(const std::string& path, uint8_t* dst, size_t cap, WavData* out, std::string* err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return io_error(err);
    size_t len = 0;
    while (len < cap) {
        const size_t n = std::fread(dst + len, 1, cap - len, f);
        if (n == 0) break;
        len += n;
    }
    uint8_t probe;
    const bool more = len == cap && std::fread(&probe, 1, 1, f) == 1;
    std::fclose(f);
    if (more) return read_wav(path, out, err);  // the file grew since it was sized
    return parse_wav(dst, len, out, err);
}

int read_wav(const std::string& path, WavData* out, std::string* err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return io_error(err);
    // one read into an uninitialised buffer of the file's size (growing only if the file grew)
    size_t cap = 0, len = 0;
    if (std::fseek(f, 0, SEEK_END) == 0) {
        const long sz = std::ftell(f);
        if (sz > 0) cap = (size_t)sz;
        std::fseek(f, 0, SEEK_SET);
    }
    std::unique_ptr<uint8_t[]> file(new uint8_t[std::max<size_t>(cap, 1)]);
    while (true) {
        if (len == cap) {  // full: at the end, or the size was unknown / the file grew
            uint8_t probe;
            if (std::fread(&probe, 1, 1, f) == 0) break;
            const size_t ncap = std::max<size_t>(2 * cap, 1 << 16);
            std::unique_ptr<uint8_t[]> nf(new uint8_t[ncap]);
            if (len) std::memcpy(nf.get(), file.get(), len);
            file = std::move(nf);
            cap = ncap;
            file[len++] = probe;
        }
        const size_t n = std::fread(file.get() + len, 1, cap - len, f);
        len += n;
        if (n == 0) break;
    }
    std::fclose(f);
    const int rc = parse_wav(file.get(), len, out, err);
    if (rc) return rc;
    out->file = std::move(file);
    out->file_len = len;
    return THESIA_OK;
}

int parse_wav(const uint8_t* file, size_t len, WavData* out, std::string* err) {
    struct View {
        const uint8_t* p;
        size_t n;
        size_t size() const { return n; }
        const uint8_t* data() const { return p; }
    } buf{file, len};
    if (buf.size() < 12 || std::memcmp(buf.data(), "RIFF", 4) || std::memcmp(buf.data() + 8, "WAVE", 4)) {
        *err = "not a WAV file: the reference's rodio fallback (FLAC/Vorbis) is not supported";
        return THESIA_ERR_UNSUPPORTED;
    }
    size_t pos = 12;
    bool have_fmt = false;
    uint16_t fmt_tag = 0, channels = 0, block_align = 0, bits = 0;
    uint32_t sr = 0;
    const uint8_t* data = nullptr;
    size_t data_len = 0;
    while (pos + 8 <= buf.size()) {
        const uint8_t* ck = buf.data() + pos;
        const uint32_t len = rd32(ck + 4);
        const size_t body = pos + 8;
        if (!std::memcmp(ck, "fmt ", 4)) {
            if (len < 16 || body + 16 > buf.size()) break;
            fmt_tag = rd16(buf.data() + body);
            channels = rd16(buf.data() + body + 2);
            sr = rd32(buf.data() + body + 4);
            block_align = rd16(buf.data() + body + 12);
            bits = rd16(buf.data() + body + 14);
            if (fmt_tag == 0xFFFE && len >= 40 && body + 40 <= buf.size())
                fmt_tag = rd16(buf.data() + body + 24);  // WAVE_FORMAT_EXTENSIBLE sub-format
            have_fmt = true;
        } else if (!std::memcmp(ck, "data", 4)) {
            data = buf.data() + body;
            data_len = std::min<size_t>(len, buf.size() - body);
            break;
        }
        pos = body + len + (len & 1);
    }
    if (!have_fmt || !data || channels == 0 || block_align == 0) {
        *err = "malformed WAV file (missing fmt or data chunk)";
        return THESIA_ERR_IO;
    }
    const size_t bps = block_align / channels;  // bytes per sample (container)
    int kind;
    if (fmt_tag == 3) {  // IEEE float: hound reads f32 only
        if (bits != 32 || bps != 4) {
            *err = "unsupported float WAV bit depth";
            return THESIA_ERR_UNSUPPORTED;
        }
        kind = PCM_F32;
    } else if (fmt_tag == 1) {
        if (bits == 0 || bits > 32 || bps == 0 || bps > 4 || bps * 8 < bits) {
            *err = "unsupported integer WAV bit depth";
            return THESIA_ERR_UNSUPPORTED;
        }
        kind = bps == 1 ? PCM_U8 : bps == 2 ? PCM_S16 : bps == 3 ? PCM_S24 : PCM_S32;
    } else {
        *err = "unsupported WAV format tag " + std::to_string(fmt_tag);
        return THESIA_ERR_UNSUPPORTED;
    }
    out->sr = sr;
    out->channels = channels;
    out->bits = bits;
    out->kind = kind;
    // audio.rs:32-34: truncate to whole frames
    out->n_frames = (data_len / bps) / channels;
    out->data_off = (size_t)(data - file);
    out->base = file;
    return THESIA_OK;
}

}  // namespace thesia
