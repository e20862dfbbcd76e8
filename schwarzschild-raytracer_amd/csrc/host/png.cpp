// png.cpp — presentation of a rendered frame as a PNG file.
//
// The reference presents its framebuffer in a GLFW window (src/main.cpp:318-319
// draw, :432 glfwSwapBuffers); here a frame copied to host memory can be
// written out instead. RGBA8, 8 bits per channel, rows stored bottom-up as GL
// leaves them (row 0 = the bottom of the image), so the writer flips by
// default. zlib deflate, one filter per row chosen by the usual minimum
// sum-of-absolute-differences heuristic (PNG spec §12.8).
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sr/sr.h"

namespace {

struct CrcTable {
    uint32_t t[256];
    CrcTable() {
        for (uint32_t n = 0; n < 256; n++) {
            uint32_t c = n;
            for (int k = 0; k < 8; k++) c = (c & 1u) ? 0xedb88320u ^ (c >> 1) : c >> 1;
            t[n] = c;
        }
    }
};

uint32_t crc(const uint8_t* p, size_t n, uint32_t c = 0xffffffffu) {
    static const CrcTable tab;  // thread-safe initialisation
    for (size_t i = 0; i < n; i++) c = tab.t[(c ^ p[i]) & 0xffu] ^ (c >> 8);
    return c;
}

void put32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24));
    v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
}

void chunk(std::vector<uint8_t>& out, const char type[4], const uint8_t* data, size_t n) {
    put32(out, (uint32_t)n);
    const size_t at = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data, data + n);
    put32(out, crc(out.data() + at, n + 4) ^ 0xffffffffu);
}

uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return (uint8_t)a;
    return pb <= pc ? (uint8_t)b : (uint8_t)c;
}

// Filtered scanline (filter byte + bytes) of `row` given the previous row (or
// nullptr): the filter of the five with the smallest sum of |signed bytes|.
void filter_row(const uint8_t* row, const uint8_t* prev, size_t n, std::vector<uint8_t>& out) {
    static thread_local std::vector<uint8_t> cand[5];
    long best_sum = -1;
    int best = 0;
    for (int f = 0; f < 5; f++) {
        auto& c = cand[f];
        c.resize(n);
        long sum = 0;
        for (size_t i = 0; i < n; i++) {
            const int a = i >= 4 ? row[i - 4] : 0;
            const int b = prev ? prev[i] : 0;
            const int cc = (i >= 4 && prev) ? prev[i - 4] : 0;
            int pred = 0;
            switch (f) {
            case 1: pred = a; break;
            case 2: pred = b; break;
            case 3: pred = (a + b) >> 1; break;
            case 4: pred = paeth(a, b, cc); break;
            default: break;
            }
            const uint8_t v = (uint8_t)(row[i] - pred);
            c[i] = v;
            sum += v < 128 ? v : 256 - v;
        }
        if (best_sum < 0 || sum < best_sum) {
            best_sum = sum;
            best = f;
        }
    }
    out.push_back((uint8_t)best);
    out.insert(out.end(), cand[best].begin(), cand[best].end());
}

}  // namespace

extern "C" int sr_write_png(const char* path, const uint8_t* rgba8, int width, int height, size_t pitch_bytes,
                            int flip_rows) {
    if (!path || !rgba8 || width <= 0 || height <= 0 || pitch_bytes < (size_t)width * 4) return SR_E_INVALID;
    const size_t n = (size_t)width * 4;
    std::vector<uint8_t> raw;
    raw.reserve((n + 1) * (size_t)height);
    const uint8_t* prev = nullptr;
    for (int y = 0; y < height; y++) {
        const int src = flip_rows ? height - 1 - y : y;
        const uint8_t* row = rgba8 + (size_t)src * pitch_bytes;
        filter_row(row, prev, n, raw);
        prev = row;
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return SR_E_NOMEM;
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)width);
    put32(ihdr, (uint32_t)height);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA, deflate, adaptive filters, no interlace
    chunk(out, "IHDR", ihdr.data(), ihdr.size());
    chunk(out, "IDAT", z.data(), zlen);
    chunk(out, "IEND", nullptr, 0);
    FILE* f = std::fopen(path, "wb");
    if (!f) return SR_E_IO;
    const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    return (std::fclose(f) == 0 && ok) ? SR_OK : SR_E_IO;
}
