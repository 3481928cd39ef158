// Move-to-front + RLE2 (zero-run RUNA/RUNB coding) on the device.
//
// Restates MTFAndRLE2StageEncoder / valueToFront (reference
// kernel.cpp:2514-2533, 2561-2649) with exact sequential semantics.  One
// 64-lane wave per block walks the block in tiles of 64 symbols, lane j
// holding symbol j of the tile, with the MTF list state of the tile start
// kept in LDS as pos[] (symbol -> list position R0) and lst[] (the list).
// The rank of tile symbol j follows from set arithmetic over the tile:
//   * if the symbol occurred earlier in the tile (last at j'), its rank is the
//     number of distinct symbols in (j', j): positions d in (j', j) that are
//     not the previous occurrence of any e < j (an OR-scan of 1 << prev(e));
//   * otherwise it is |T_j| + R0 - #{c in T_j : R0(c) < R0}, T_j the distinct
//     symbols before j (an OR-scan of one-hot 256-bit R0 masks);
// and the list of the next tile is the tile's distinct symbols by last
// occurrence followed by the others in R0 order.  The initial list is the
// block's symbols in use, ascending (the reference's symbol map,
// :2565-2572).  Zero ranks are coded as bijective base-2 RUNA/RUNB digits
// (:2585-2606); the per-block histogram of the emitted symbols (258 bins) is
// what the reference adds into its frequency array (:2613, :2641-2643).
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"

namespace bz2mi {

namespace {

constexpr int kSuper = 1024;  // symbols staged in LDS at a time (16 tiles)

struct MtfShared {
    uint64_t occ[256];  // lanes of the current tile holding each symbol (zero between tiles)
    uint32_t hist[kMaxAlpha];
    uint8_t pos[256];   // symbol -> MTF list position at the tile start
    uint8_t lst[256];   // MTF list at the tile start
    uint8_t sym[kSuper];
};

__device__ __forceinline__ uint32_t wave_incl_or(uint32_t x) {
    x |= dpp_mov<dpp::kRowShr1>(x);
    x |= dpp_mov<dpp::kRowShr1 + 1>(x);
    x |= dpp_mov<dpp::kRowShr1 + 3>(x);
    x |= dpp_mov<dpp::kRowShr1 + 7>(x);
    x |= dpp_mov<dpp::kBcast15, 0xa>(x);
    x |= dpp_mov<dpp::kBcast31, 0xc>(x);
    return x;
}

__device__ __forceinline__ uint64_t wave_incl_or64(uint64_t x) {
    return ((uint64_t)wave_incl_or((uint32_t)(x >> 32)) << 32) | wave_incl_or((uint32_t)x);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ int msb64(uint64_t v) { return 63 - __clzll((long long)v); }  // v != 0

// RUNA/RUNB digits of a zero run of length r >= 1: floor(log2(r + 1))
__device__ __forceinline__ uint32_t run_ndigits(uint32_t r) { return 31u - (uint32_t)__clz(r + 1); }

// bijective base-2 digits of a zero run, least significant first
__device__ __forceinline__ uint32_t emit_run(uint32_t r, uint16_t* out, uint32_t o, uint32_t& na, uint32_t& nb) {
    uint32_t rep = r - 1;
    for (;;) {
        const uint32_t d = rep & 1u;  // RUNA = 0, RUNB = 1
        out[o++] = (uint16_t)d;
        na += d ^ 1u;
        nb += d;
        if (rep <= 1) break;
        rep = (rep - 2) >> 1;
    }
    return o;
}

}  // namespace

BZ2MI_PHASE_TABLE(g_mtf_phase)

int mtf_phases(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mtf_phase), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

__global__ __launch_bounds__(64) void mtf_kernel(const uint8_t* __restrict__ bwt, size_t stride,
                                                 const uint32_t* __restrict__ lens, int nblocks,
                                                 const uint32_t* __restrict__ present, uint16_t* __restrict__ mtf_out,
                                                 size_t mtf_stride, uint32_t* __restrict__ mtf_len,
                                                 uint32_t* __restrict__ alpha_out, uint32_t* __restrict__ hist_out) {
    __shared__ MtfShared sh;
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    const int j = threadIdx.x;  // lane == tile position
    const int n = (int)uniform(lens[b]);
    const uint8_t* X = bwt + (size_t)b * stride;
    uint16_t* out = mtf_out + (size_t)b * mtf_stride;
    [[maybe_unused]] const bool stamp = b == nblocks / 2;
    BZ2MI_PHASE(g_mtf_phase, 0, stamp);

    for (int s = j; s < 256; s += 64) sh.occ[s] = 0;
    for (int s = j; s < kMaxAlpha; s += 64) sh.hist[s] = 0;
    // initial list: the symbols in use, ascending; lane j places symbols 4j..4j+3
    const uint32_t nib = (present[(size_t)b * 8 + (j >> 3)] >> ((j & 7) * 4)) & 15u;
    const uint32_t pinc = wave_incl_sum((uint32_t)__popc(nib));
    const int k = (int)uniform((uint32_t)__builtin_amdgcn_readlane((int)pinc, 63));
    {
        uint32_t r = pinc - (uint32_t)__popc(nib);
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (nib >> e & 1u) {
                sh.pos[4 * j + e] = (uint8_t)r;
                sh.lst[r] = (uint8_t)(4 * j + e);
                r++;
            }
    }
    const uint64_t below = (1ull << j) - 1;  // lanes before j
    uint32_t o = 0;      // output symbols so far
    uint32_t carry = 0;  // zero run open at the tile start
    uint32_t na = 0, nb = 0;
    auto load16 = [&](int at) -> uint4 {
        return at < n ? *reinterpret_cast<const uint4*>(X + at) : make_uint4(0, 0, 0, 0);
    };
    uint4 cur = load16(16 * j);
    // the tile loop, instantiated for the words of the 256-bit symbol sets
    // the block's k symbols occupy (2, 4 or 8): fewer OR-scans per tile
    auto tiles = [&](auto kw) {
    constexpr int KW = decltype(kw)::value;
    for (int sb = 0; sb < n; sb += kSuper) {
        __syncthreads();  // the previous superblock is consumed
        *reinterpret_cast<uint4*>(sh.sym + 16 * j) = cur;
        if (sb + kSuper < n) cur = load16(sb + kSuper + 16 * j);
        __syncthreads();
        const int ntile = min(kSuper / 64, (n - sb + 63) >> 6);
        for (int q = 0; q < ntile; ++q) {
            const int nlive = min(64, n - sb - q * 64);
            const bool live = j < nlive;
            const uint64_t lmask = nlive == 64 ? ~0ull : ((1ull << nlive) - 1);
            const uint32_t s = sh.sym[q * 64 + j];
            // ---- lanes holding the same symbol; previous occurrence in the tile
            if (live) atomicOr(reinterpret_cast<unsigned long long*>(&sh.occ[s]), 1ull << j);
            const uint64_t M = live ? sh.occ[s] : 0ull;
            const uint32_t R0 = sh.pos[s];
            if (live) sh.occ[s] = 0;
            const uint64_t pb = M & below;
            const bool hasprv = pb != 0;
            const int prv = hasprv ? msb64(pb) : 0;
            const bool fo = live && !hasprv;
            // ---- seen earlier in the tile: distinct symbols in (prv, j)
            const uint64_t pbit = hasprv ? (1ull << prv) : 0ull;
            const uint64_t Pinc = wave_incl_or64(pbit);
            const uint64_t rng = below & ~((2ull << prv) - 1);
            const uint32_t rC = (uint32_t)__popcll(rng & ~(Pinc & ~pbit));
            // ---- first in the tile: |T_j| + R0 - #{c in T_j : R0(c) < R0}
            const uint64_t FO = __ballot(fo);
            const uint32_t w = R0 >> 5, bit = 1u << (R0 & 31);
            // the scans of the 256-bit first-occurrence sets: only the KW words
            // the block's k symbols can occupy (list positions < k)
            uint32_t qi[8], qall[8];
            uint32_t less = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                qi[e] = 0u;
                if (e < KW) {
                    qi[e] = wave_incl_or((fo && w == (uint32_t)e) ? bit : 0u);
                    const uint32_t m = (uint32_t)e < w ? ~0u : ((uint32_t)e == w ? bit - 1 : 0u);
                    less += (uint32_t)__popc(qi[e] & m);
                }
            }
            const uint32_t rB = (uint32_t)__popcll(FO & below) + R0 - less;
            const uint32_t rank = hasprv ? rC : rB;
            // ---- list of the next tile
            const uint64_t LO = ~readlane64(Pinc, 63) & lmask;  // last occurrences
            const uint32_t D = (uint32_t)__popcll(LO);
#pragma unroll
            for (int e = 0; e < 8; ++e) qall[e] = e < KW ? (uint32_t)__builtin_amdgcn_readlane((int)qi[e], 63) : 0u;
            {
                const uint32_t lw = reinterpret_cast<const uint32_t*>(sh.lst)[j];  // positions 4j..4j+3
                uint32_t qa = 0, cb = 0;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    qa = (j >> 3) == e ? qall[e] : qa;
                    cb += (j >> 3) > e ? (uint32_t)__popc(qall[e]) : 0u;
                }
                const uint32_t sh4 = (uint32_t)(j & 7) * 4;
                cb += (uint32_t)__popc(qa & ((1u << sh4) - 1u));
                const uint32_t nq = (qa >> sh4) & 15u;
                if (live && (LO >> j & 1ull)) {
                    const uint32_t np = (uint32_t)__popcll(LO & ~((2ull << j) - 1));
                    sh.lst[np] = (uint8_t)s;
                    sh.pos[s] = (uint8_t)np;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t rpos = 4u * (uint32_t)j + e;
                    if (rpos < (uint32_t)k && !(nq >> e & 1u)) {
                        const uint32_t c = (lw >> (8 * e)) & 0xffu;
                        const uint32_t np = D + rpos - (cb + (uint32_t)__popc(nq & ((1u << e) - 1u)));
                        sh.lst[np] = (uint8_t)c;
                        sh.pos[c] = (uint8_t)np;
                    }
                }
            }
            // ---- zero runs, output offsets, emission
            const bool nz = live && rank != 0;
            const uint64_t NZ = __ballot(nz);
            uint32_t cnt = 0, run = 0;
            if (nz) {
                const uint64_t nzb = NZ & below;
                run = nzb ? (uint32_t)(j - msb64(nzb) - 1) : (uint32_t)j + carry;
                cnt = (run ? run_ndigits(run) : 0u) + 1u;
                atomicAdd(&sh.hist[rank + 1], 1u);
            }
            const uint32_t ci = wave_incl_sum(cnt);
            if (nz) {
                uint32_t e = o + ci - cnt;
                if (run) e = emit_run(run, out, e, na, nb);
                out[e] = (uint16_t)(rank + 1);
            }
            o += (uint32_t)__builtin_amdgcn_readlane((int)ci, 63);
            carry = NZ ? (uint32_t)(nlive - 1 - msb64(NZ)) : carry + (uint32_t)nlive;
        }
    }
    };
    if (k <= 64) tiles(std::integral_constant<int, 2>{});
    else if (k <= 128) tiles(std::integral_constant<int, 4>{});
    else tiles(std::integral_constant<int, 8>{});
    if (carry) {  // the block ends in a zero run
        if (j == 0) emit_run(carry, out, o, na, nb);
        o += run_ndigits(carry);
    }
    __syncthreads();
    BZ2MI_PHASE(g_mtf_phase, 1, stamp);
    const uint32_t runA = wave_sum(na), runB = wave_sum(nb);
    const uint32_t eob = (uint32_t)k + 1;
    if (j == 0) {
        out[o] = (uint16_t)eob;
        mtf_len[b] = o + 1;
        alpha_out[b] = eob + 1;
    }
    uint32_t* H = hist_out + (size_t)b * kMaxAlpha;
    for (int s = j; s < kMaxAlpha; s += 64) {
        uint32_t h = sh.hist[s];
        if (s == 0) h += runA;
        if (s == 1) h += runB;
        if ((uint32_t)s == eob) h += 1;
        H[s] = h;
    }
}

}  // namespace bz2mi
