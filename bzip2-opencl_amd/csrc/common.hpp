// Shared device helpers and constants for the bz2mi HIP kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Phase stamps for one representative workgroup (make PHASES=1): a kernel
// declares a table with BZ2MI_PHASE_TABLE(name) and stamps wall_clock64()
// (100 MHz) at phase boundaries; bz2mi_debug_phases() reads the tables back.
#ifdef BZ2MI_PHASES
#define BZ2MI_PHASE_TABLE(tab) __device__ unsigned long long tab[16];
#define BZ2MI_PHASE(tab, k, cond)                                   \
    do {                                                            \
        if ((cond) && threadIdx.x == 0) tab[k] = wall_clock64();    \
    } while (0)
#else
#define BZ2MI_PHASE_TABLE(tab)
#define BZ2MI_PHASE(tab, k, cond) \
    do {                          \
    } while (0)
#endif

namespace bz2mi {

// Format constants (reference include/Config.hpp:27-47).
constexpr int kBlockMagicHi = 0x314159;
constexpr int kBlockMagicLo = 0x265359;
constexpr int kEosMagicHi = 0x177245;
constexpr int kEosMagicLo = 0x385090;
constexpr int kGroupRun = 50;      // HUFFMAN_GROUP_RUN_LENGTH
constexpr int kMaxAlpha = 258;     // HUFFMAN_MAXIMUM_ALPHABET_SIZE
constexpr int kMaxTables = 6;      // HUFFMAN_MAXIMUM_TABLES
constexpr int kMaxCodeLen = 20;    // HUFFMAN_ENCODE_MAXIMUM_CODE_LENGTH
constexpr int kHighCost = 15;      // HUFFMAN_HIGH_SYMBOL_COST
constexpr int kHeaderBits = 81;    // 48-bit block magic + 32-bit CRC + randomised bit

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    const uint32_t lo = uniform((uint32_t)x), hi = uniform((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// ---- cross-lane moves without the LDS crossbar (ds_bpermute): DPP row /
// quad permutes and the gfx950 permlane swaps, all plain VALU ops.
namespace dpp {
constexpr int kQuadXor1 = 0xB1;    // quad_perm [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;    // quad_perm [2,3,0,1]
constexpr int kQuadXor3 = 0x1B;    // quad_perm [3,2,1,0]
constexpr int kRowShr1 = 0x111;    // row_shr:n = 0x110 + n
constexpr int kRowRor8 = 0x128;    // row_ror:8 (= xor 8 inside a row of 16)
constexpr int kWaveShr1 = 0x138;   // wave_shr:1
constexpr int kHalfMirror = 0x141; // row_half_mirror (= xor 7 inside 8 lanes)
constexpr int kBcast15 = 0x142;    // row_bcast:15
constexpr int kBcast31 = 0x143;    // row_bcast:31
}  // namespace dpp

template <int Ctrl, int RowMask = 0xf>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v, uint32_t old = 0) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, Ctrl, RowMask, 0xf, false);
}

// value of lane (lane ^ J), J a power of two < 64
template <int J>
__device__ __forceinline__ uint32_t xor_lanes(uint32_t v) {
    if constexpr (J == 1) {
        return dpp_mov<dpp::kQuadXor1>(v);
    } else if constexpr (J == 2) {
        return dpp_mov<dpp::kQuadXor2>(v);
    } else if constexpr (J == 4) {
        return dpp_mov<dpp::kQuadXor3>(dpp_mov<dpp::kHalfMirror>(v));
    } else if constexpr (J == 8) {
        return dpp_mov<dpp::kRowRor8>(v);
    } else if constexpr (J == 16) {
        // swaps the odd rows of the first operand with the even rows of the second
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & 16) ? r[0] : r[1];
    } else {
        static_assert(J == 32, "xor_lanes: J in {1,2,4,8,16,32}");
        // swaps the upper half of the first operand with the lower half of the second
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    }
}

__device__ __forceinline__ uint32_t xor_lanes_rt(uint32_t v, int j) {
    switch (j) {
        case 1: return xor_lanes<1>(v);
        case 2: return xor_lanes<2>(v);
        case 4: return xor_lanes<4>(v);
        case 8: return xor_lanes<8>(v);
        case 16: return xor_lanes<16>(v);
        default: return xor_lanes<32>(v);
    }
}

__device__ __forceinline__ uint64_t xor_lanes_rt64(uint64_t v, int j) {
    const uint32_t lo = xor_lanes_rt((uint32_t)v, j), hi = xor_lanes_rt((uint32_t)(v >> 32), j);
    return ((uint64_t)hi << 32) | lo;
}

// value of lane - 1 (lane 0 gets `first`)
__device__ __forceinline__ uint32_t lane_prev(uint32_t v, uint32_t first = 0) {
    const uint32_t p = dpp_mov<dpp::kWaveShr1>(v);
    return lane_id() ? p : first;
}

// Inclusive scans over one 64-lane wave: row_shr 1,2,4,8 inside rows of 16,
// then row_bcast15 / row_bcast31 carry across rows.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += dpp_mov<dpp::kRowShr1>(x);
    x += dpp_mov<dpp::kRowShr1 + 1>(x);
    x += dpp_mov<dpp::kRowShr1 + 3>(x);
    x += dpp_mov<dpp::kRowShr1 + 7>(x);
    x += dpp_mov<dpp::kBcast15, 0xa>(x);
    x += dpp_mov<dpp::kBcast31, 0xc>(x);
    return x;
}

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = max(x, dpp_mov<dpp::kRowShr1>(x));
    x = max(x, dpp_mov<dpp::kRowShr1 + 1>(x));
    x = max(x, dpp_mov<dpp::kRowShr1 + 3>(x));
    x = max(x, dpp_mov<dpp::kRowShr1 + 7>(x));
    x = max(x, dpp_mov<dpp::kBcast15, 0xa>(x));
    x = max(x, dpp_mov<dpp::kBcast31, 0xc>(x));
    return x;
}

__device__ __forceinline__ uint64_t wave_incl_sum64(uint64_t x) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    return x;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(x), 63);
}

// Exclusive sum over a workgroup of NT threads.  `tmp` needs NT/64 words of
// LDS.  Returns the exclusive prefix; *total receives the workgroup sum.
template <int NT>
__device__ __forceinline__ uint32_t wg_excl_sum(uint32_t v, uint32_t* tmp, uint32_t* total) {
    constexpr int NW = NT / 64;
    const uint32_t inc = wave_incl_sum(v);
    if (lane_id() == 63) tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        uint32_t t = tmp[w];
        base += (w < wave_id()) ? t : 0u;
        all += t;
    }
    __syncthreads();
    *total = uniform(all);
    return base + inc - v;
}

template <int NT>
__device__ __forceinline__ uint64_t wg_excl_sum64(uint64_t v, uint64_t* tmp, uint64_t* total) {
    constexpr int NW = NT / 64;
    const uint64_t inc = wave_incl_sum64(v);
    if (lane_id() == 63) tmp[wave_id()] = inc;
    __syncthreads();
    uint64_t base = 0, all = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        uint64_t t = tmp[w];
        base += (w < wave_id()) ? t : 0ull;
        all += t;
    }
    __syncthreads();
    *total = uniform64(all);
    return base + inc - v;
}

// Inclusive max over a workgroup (values are indices, so 0 is neutral).
template <int NT>
__device__ __forceinline__ uint32_t wg_incl_max(uint32_t v, uint32_t* tmp, uint32_t* total) {
    constexpr int NW = NT / 64;
    const uint32_t inc = wave_incl_max(v);
    if (lane_id() == 63) tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        uint32_t t = tmp[w];
        if (w < wave_id()) base = base > t ? base : t;
        all = all > t ? all : t;
    }
    __syncthreads();
    *total = uniform(all);
    return inc > base ? inc : base;
}

// Mask of the lanes of this wave whose `key` (8 bits) equals this lane's,
// restricted to `valid` lanes.
__device__ __forceinline__ uint64_t wave_match8(uint32_t key, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const bool bit = (key >> b) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
    }
    return peers;
}

// Write `count` (1..32) bits of `value`, MSB-first, at absolute bit `pos` of
// a big-endian bit stream held in 32-bit words (byte-swapped on store so the
// memory image is the byte stream).  Used for words shared between writers.
__device__ __forceinline__ void put_bits_or(uint32_t* out, uint64_t pos, int count, uint32_t value) {
    const uint64_t w = pos >> 5;
    const int off = (int)(pos & 31);
    const uint64_t v = ((uint64_t)(value & (count == 32 ? 0xffffffffu : ((1u << count) - 1u))))
                       << (64 - count - off);
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    if (hi) atomicOr(&out[w], bswap32(hi));
    if (lo) atomicOr(&out[w + 1], bswap32(lo));
}

// Sequential bit writer owned by one thread over [start, end): interior words
// are plain stores, the first and last (possibly shared) words use atomicOr.
// The destination words must be zero beforehand.
struct BitSink {
    uint32_t* out;
    uint64_t start;   // first bit this writer owns
    uint64_t pos;     // next bit position
    uint64_t acc;     // pending bits, MSB-aligned
    int nacc;

    __device__ void init(uint32_t* o, uint64_t p) {
        out = o;
        start = p;
        pos = p;
        acc = 0;
        nacc = (int)(p & 31);  // leading bits of the first word are someone else's
    }
    __device__ __forceinline__ void flush_word(bool last) {
        const uint64_t w = (pos - (uint64_t)nacc) >> 5;
        const uint32_t word = (uint32_t)(acc >> 32);
        const bool shared = (w << 5) < start || last;
        if (shared) {
            if (word) atomicOr(&out[w], bswap32(word));
        } else {
            out[w] = bswap32(word);
        }
    }
    __device__ __forceinline__ void put(int count, uint32_t value) {
        // count <= 32
        const uint64_t v = (uint64_t)(value & (count == 32 ? 0xffffffffu : ((1u << count) - 1u)));
        acc |= (v << (64 - count)) >> nacc;
        nacc += count;
        pos += count;
        if (nacc >= 32) {
            flush_word(false);
            acc <<= 32;
            nacc -= 32;
        }
    }
    __device__ __forceinline__ void finish() {
        if (nacc > 0) {
            // partially filled last word: shared with the next writer
            const uint64_t w = (pos - (uint64_t)nacc) >> 5;
            const uint32_t word = (uint32_t)(acc >> 32);
            if (word) atomicOr(&out[w], bswap32(word));
        }
    }
};

}  // namespace bz2mi
