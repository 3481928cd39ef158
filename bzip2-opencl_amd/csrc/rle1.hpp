// Host RLE1 front end: run-length pre-pass, block split and block CRC.
//
// Semantics of BlockCompressor::write / writeRun / finishRLE
// (reference include/BlockCompressor.hpp:69-154) driven the way
// OutputStream::write / getNextCompressor drive it (OutputStream.hpp:131-142,
// 179-188): a block refuses the next byte once more than S-6 RLE1 bytes have
// been flushed into it, and its pending run is flushed when it is closed.
// The CRC (CRC32.hpp:75-86) covers the block's input bytes.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <array>

namespace bz2mi {

struct Crc32Table {
    std::array<uint32_t, 256> t{};
    constexpr Crc32Table() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i << 24;
            for (int k = 0; k < 8; ++k) c = (c & 0x80000000u) ? (c << 1) ^ 0x04c11db7u : (c << 1);
            t[i] = c;
        }
    }
};
inline constexpr Crc32Table kCrc{};

// Device CRC tables (layout of kCrcTabWords u32): [0, 1024) slicing-by-4
// tables (T_k[b] = CRC register of byte b followed by k zero bytes), then for
// k = 0..31 the linear map "process 2^k zero bytes" on a raw CRC register as
// four byte-sliced tables (1024 words each): A(x) = T0[x&255] ^ T1[x>>8&255] ^
// T2[x>>16&255] ^ T3[x>>24].  Used to combine CRCs of byte ranges computed in
// parallel: crc(A|B) = A_{|B|}(crc(A)) ^ crc(B) for raw registers.
constexpr int kCrcShiftBase = 1024;
constexpr int kCrcTabWords = 1024 * 33;
inline void crc_device_tables(uint32_t* out) {
    for (int b = 0; b < 256; ++b) {
        uint32_t v = kCrc.t[b];
        out[b] = v;
        for (int k = 1; k < 4; ++k) {
            v = (v << 8) ^ kCrc.t[v >> 24];
            out[256 * k + b] = v;
        }
    }
    uint32_t col[32], sq[32];
    for (int i = 0; i < 32; ++i) {  // A_1: one zero byte
        const uint32_t e = 1u << i;
        col[i] = (e << 8) ^ kCrc.t[e >> 24];
    }
    auto apply = [](const uint32_t* c, uint32_t x) {
        uint32_t r = 0;
        for (int i = 0; i < 32; ++i)
            if (x >> i & 1u) r ^= c[i];
        return r;
    };
    for (int k = 0; k < 32; ++k) {
        uint32_t* T = out + kCrcShiftBase + 1024 * k;
        for (int j = 0; j < 4; ++j)
            for (uint32_t b = 0; b < 256; ++b) T[256 * j + b] = apply(col, b << (8 * j));
        for (int i = 0; i < 32; ++i) sq[i] = apply(col, col[i]);  // A_{2^(k+1)} = A_{2^k} o A_{2^k}
        for (int i = 0; i < 32; ++i) col[i] = sq[i];
    }
}

inline uint32_t crc_update(uint32_t crc, const uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; ++i) crc = (crc << 8) ^ kCrc.t[((crc >> 24) ^ p[i]) & 0xffu];
    return crc;
}

// Incremental RLE1 encoder of one block.
struct Rle1Block {
    uint8_t* out = nullptr;
    int len = 0;        // flushed RLE1 bytes
    int limit = 0;      // S - 6
    int value = -1;     // pending run value
    int run = 0;        // pending run length
    uint32_t crc = 0xffffffffu;

    void begin(uint8_t* dst, int S) {
        out = dst;
        len = 0;
        limit = S - 6;
        value = -1;
        run = 0;
        crc = 0xffffffffu;
    }
    bool empty() const { return len == 0 && run == 0; }
    void flush(int v, int r) {
        crc_run(v, r);
        const uint8_t b = (uint8_t)v;
        out[len++] = b;
        if (r > 1) {
            out[len++] = b;
            if (r > 2) {
                out[len++] = b;
                if (r > 3) {
                    out[len++] = b;
                    out[len++] = (uint8_t)(r - 4);
                }
            }
        }
    }
    void crc_run(int v, int r) {
        for (int i = 0; i < r; ++i) crc = (crc << 8) ^ kCrc.t[((crc >> 24) ^ (uint32_t)v) & 0xffu];
    }
    // false: block full, the byte was not taken
    bool put(int v) {
        if (len > limit) return false;
        if (run == 0) {
            value = v;
            run = 1;
        } else if (value == v) {
            if (++run > 254) {
                flush(value, 255);
                run = 0;
            }
        } else {
            flush(value, run);
            value = v;
            run = 1;
        }
        return true;
    }
    // consume bytes until the block is full; returns bytes taken
    size_t put_many(const uint8_t* p, size_t n) {
        size_t i = 0;
        while (i < n) {
            if (len > limit) break;
            const int v = p[i];
            if (run == 0) {
                value = v;
                run = 1;
                ++i;
                continue;
            }
            if (value == v) {
                // extend the run in one step, capped at the 255 piece
                size_t j = i;
                while (j < n && p[j] == v && run < 255) {
                    ++run;
                    ++j;
                }
                i = j;
                if (run == 255) {
                    flush(value, 255);
                    run = 0;
                }
                continue;
            }
            flush(value, run);
            value = v;
            run = 1;
            ++i;
        }
        return i;
    }
    void finish() {
        if (run > 0) {
            flush(value & 0xff, run);
            run = 0;
        }
    }
    uint32_t block_crc() const { return ~crc; }
};

}  // namespace bz2mi
