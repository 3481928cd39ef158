// Move-to-front + RLE2 (zero-run RUNA/RUNB coding) on the device.
//
// Restates MTFAndRLE2StageEncoder / valueToFront (reference
// kernel.cpp:2514-2533, 2561-2649) with exact sequential semantics.
//
// A wave walks a range of the block in tiles of 64 symbols, lane j holding
// symbol j of the tile, with the MTF list state of the tile start in LDS as
// pos[] (symbol -> list position R0) and lst[] (the list).  The rank of tile
// symbol j follows from set arithmetic over the tile:
//   * if the symbol occurred earlier in the tile (last at j'), its rank is the
//     number of distinct symbols in (j', j): positions d in (j', j) that are
//     not the previous occurrence of any e < j (an OR-scan of 1 << prev(e));
//   * otherwise (a first occurrence) it is |T_j| + R0 - #{c in T_j : R0(c) <
//     R0}, T_j the distinct symbols before j.  The first occurrences' R0 form
//     a set F (one LDS atomicOr per lane into a 256-bit set); an R0 is replaced
//     by its rank q among F (word prefix counts of the set, read across lanes
//     with ds_bpermute), so the count is one 64-bit OR-scan of 1 << q;
// and the list of the next tile is the tile's distinct symbols by last
// occurrence followed by the others in R0 order (old positions not in F keep
// their order, shifted by the set's prefix counts).  The initial list is the
// block's symbols in use, ascending (the reference's symbol map, :2565-2572).
// Zero runs are coded as bijective base-2 RUNA/RUNB digits (:2585-2606); the
// per-block histogram of the emitted symbols (258 bins) is what the reference
// adds into its frequency array (:2613, :2641-2643).
//
// Segments (G waves per block, for batches with few blocks -- the 900 KB
// mode): the block is cut at G symbol changes (a cut where bwt[p] != bwt[p-1]
// never splits a zero run, and the symbol at p has a nonzero rank whatever
// the list), each wave finds its segment's distinct symbols ordered by last
// occurrence D_g, and composes its start list L_g = D_{g-1} ++ (L_{g-1} \
// D_{g-1}) from the block's initial list -- the list the sequential encoder
// holds at p_g.  Segments are coded concurrently into scratch and then
// concatenated.
#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"

namespace bz2mi {

namespace {

constexpr int kSuper = 1024;  // symbols staged in LDS at a time (16 tiles)

struct MtfWave {
    uint64_t occ[256];  // lanes of the current tile holding each symbol (zero between tiles);
                        // the segment phase keeps last occurrences here first
    uint32_t fset[8];   // R0 of the tile's first occurrences (zero between tiles)
    uint8_t pos[256];   // symbol -> MTF list position at the tile start
    uint8_t lst[256];   // MTF list at the tile start
    uint8_t sym[kSuper];
};

// list composition state of the segments (G > 1 only)
template <int G>
struct MtfSegs {
    uint8_t init[256];       // the initial list
    uint8_t dl[G][256];      // each segment's distinct symbols, most recent first
    uint8_t mark[G][256];    // composition scratch (per wave)
    uint32_t dcnt[G];        // distinct symbols of each segment
};
template <>
struct MtfSegs<1> {};

template <int G>
struct MtfBlock {
    MtfWave w[G];
    uint32_t hist[kMaxAlpha];
    uint32_t seg[G + 1];     // segment starts (seg[G] = n)
    uint32_t cnt[G];         // output symbols of each segment
    uint32_t runs[2];        // RUNA / RUNB digits
    MtfSegs<G> sg;
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

// value of `v` in lane `src` (0..63), through the LDS crossbar (no memory)
__device__ __forceinline__ uint32_t lane_get(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}

__device__ __forceinline__ int msb64(uint64_t v) { return 63 - __clzll((long long)v); }  // v != 0

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

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

// ascending register bitonic sort of 256 keys over one wave, striped
// (element e of lane l is item e*64 + l)
__device__ __forceinline__ void wave_bitonic256(uint32_t (&key)[4]) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= 256; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j >= 1; j >>= 1) {
            if (j >= 64) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int pe = e ^ (j / 64);
                    if (pe > e) {
                        const bool asc = ((e * 64) & k) == 0;
                        const uint32_t lo = min(key[e], key[pe]), hi = max(key[e], key[pe]);
                        key[e] = asc ? lo : hi;
                        key[pe] = asc ? hi : lo;
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t o = xor_lanes_rt(key[e], j);
                    const bool asc = ((e * 64 + lane) & k) == 0;
                    const bool lower = (lane & j) == 0;
                    key[e] = (lower == asc) ? min(key[e], o) : max(key[e], o);
                }
            }
        }
    }
}

// MTF/RLE2 of X[p0, p1) from the list in W.lst / W.pos (k symbols in use),
// symbols to out[0..); returns the output count.  X[p0] (p0 > 0) differs
// from X[p0-1], so no zero run is open at p0.
__device__ uint32_t mtf_range(const uint8_t* __restrict__ X, int p0, int p1, int k, MtfWave& W, uint32_t* hist,
                              uint16_t* __restrict__ out, uint32_t& na, uint32_t& nb) {
    const int j = lane_id();
    const uint64_t below = (1ull << j) - 1;  // lanes before j
    uint32_t o = 0;      // output symbols so far
    uint32_t carry = 0;  // zero run open at the tile start
    const int a0 = p0 & ~63;  // tiles are 64-aligned block positions
    auto load16 = [&](int at) -> uint4 {
        return at < p1 ? *reinterpret_cast<const uint4*>(X + at) : make_uint4(0, 0, 0, 0);
    };
    uint4 cur = load16(a0 + 16 * j);
    for (int sb = a0; sb < p1; sb += kSuper) {
        wave_sync_lds();  // the previous superblock is consumed
        *reinterpret_cast<uint4*>(W.sym + 16 * j) = cur;
        if (sb + kSuper < p1) cur = load16(sb + kSuper + 16 * j);
        wave_sync_lds();
        const int ntile = min(kSuper / 64, (p1 - sb + 63) >> 6);
        for (int q = 0; q < ntile; ++q) {
            const int at = sb + q * 64 + j;
            const bool live = at >= p0 && at < p1;
            const uint64_t L = __ballot(live);
            const uint32_t s = W.sym[q * 64 + j];
            // ---- lanes holding the same symbol; previous occurrence in the tile
            if (live) atomicOr(reinterpret_cast<unsigned long long*>(&W.occ[s]), 1ull << j);
            const uint64_t M = live ? W.occ[s] : 0ull;
            const uint32_t R0 = W.pos[s];
            if (live) W.occ[s] = 0;
            const uint64_t pb = M & below;
            const bool hasprv = pb != 0;
            const int prv = hasprv ? msb64(pb) : 0;
            const bool fo = live && !hasprv;
            // ---- first occurrences: their R0 into the 256-bit set F
            if (fo) atomicOr(&W.fset[R0 >> 5], 1u << (R0 & 31));
            // ---- seen earlier in the tile: distinct symbols in (prv, j)
            const uint64_t pbit = hasprv ? (1ull << prv) : 0ull;
            const uint64_t Pinc = wave_incl_or64(pbit);
            const uint64_t rng = below & ~((2ull << prv) - 1);
            const uint32_t rC = (uint32_t)__popcll(rng & ~(Pinc & ~pbit));
            const uint64_t FO = __ballot(fo);
            wave_sync_lds();
            // lane w < 8: word w of F and the F members below it
            const uint32_t fw = W.fset[j & 7];
            const uint32_t fc = j < 8 ? (uint32_t)__popc(fw) : 0u;
            uint32_t fpre = fc;
            fpre += dpp_mov<dpp::kRowShr1>(fpre);
            fpre += dpp_mov<dpp::kRowShr1 + 1>(fpre);
            fpre += dpp_mov<dpp::kRowShr1 + 3>(fpre);
            fpre -= fc;  // exclusive, lanes 0..7
            if (j < 8) W.fset[j] = 0u;
            // ---- first in the tile: |T_j| + R0 - #{c in T_j : R0(c) < R0},
            // with R0 replaced by its rank q among F
            const uint32_t bit = 1u << (R0 & 31);
            const uint32_t qr = lane_get(fpre, R0 >> 5) + (uint32_t)__popc(lane_get(fw, R0 >> 5) & (bit - 1u));
            const uint64_t qbit = fo ? (1ull << (qr & 63)) : 0ull;
            const uint64_t Qinc = wave_incl_or64(qbit);
            const uint32_t less = (uint32_t)__popcll(Qinc & (qbit - 1ull));
            const uint32_t rB = (uint32_t)__popcll(FO & below) + R0 - less;
            const uint32_t rank = hasprv ? rC : rB;
            // ---- list of the next tile
            const uint64_t LO = ~readlane64(Pinc, 63) & L;  // last occurrences
            const uint32_t D = (uint32_t)__popcll(LO);
            {
                const uint32_t lw = reinterpret_cast<const uint32_t*>(W.lst)[j];  // positions 4j..4j+3
                const uint32_t sh4 = (uint32_t)(j & 7) * 4;
                const uint32_t fj = lane_get(fw, (uint32_t)j >> 3);
                const uint32_t cb = lane_get(fpre, (uint32_t)j >> 3) + (uint32_t)__popc(fj & ((1u << sh4) - 1u));
                const uint32_t nq = (fj >> sh4) & 15u;
                if (LO >> j & 1ull) {
                    const uint32_t np = (uint32_t)__popcll(LO & ~((2ull << j) - 1));
                    W.lst[np] = (uint8_t)s;
                    W.pos[s] = (uint8_t)np;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t rpos = 4u * (uint32_t)j + e;
                    if (rpos < (uint32_t)k && !(nq >> e & 1u)) {
                        const uint32_t c = (lw >> (8 * e)) & 0xffu;
                        const uint32_t np = D + rpos - (cb + (uint32_t)__popc(nq & ((1u << e) - 1u)));
                        W.lst[np] = (uint8_t)c;
                        W.pos[c] = (uint8_t)np;
                    }
                }
            }
            // ---- zero runs, output offsets, emission
            const bool nz = live && rank != 0;
            const uint64_t NZ = __ballot(nz);
            uint32_t cnt = 0, run = 0;
            if (nz) {
                const uint64_t nzb = NZ & below;
                run = nzb ? (uint32_t)(j - msb64(nzb) - 1) : (uint32_t)(j - __builtin_ctzll(L)) + carry;
                cnt = (run ? run_ndigits(run) : 0u) + 1u;
                atomicAdd(&hist[rank + 1], 1u);
            }
            const uint32_t ci = wave_incl_sum(cnt);
            if (nz) {
                uint32_t e = o + ci - cnt;
                if (run) e = emit_run(run, out, e, na, nb);
                out[e] = (uint16_t)(rank + 1);
            }
            o += (uint32_t)__builtin_amdgcn_readlane((int)ci, 63);
            carry = NZ ? (uint32_t)(msb64(L) - msb64(NZ)) : carry + (uint32_t)__popcll(L);
        }
    }
    if (carry) {  // the range ends in a zero run
        if (j == 0) emit_run(carry, out, o, na, nb);
        o += run_ndigits(carry);
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

// One workgroup of G waves per block.  G = 1: the wave codes the whole block
// straight into mtf_out.  G > 1: segments (see the top of the file) coded
// into `scratch` (scratch_stride u16 per block) and concatenated.
template <int G>
__global__ __launch_bounds__(64 * G) void mtf_kernel(const uint8_t* __restrict__ bwt, size_t stride,
                                                     const uint32_t* __restrict__ lens, int nblocks,
                                                     const uint32_t* __restrict__ present,
                                                     uint16_t* __restrict__ mtf_out, size_t mtf_stride,
                                                     uint32_t* __restrict__ mtf_len, uint32_t* __restrict__ alpha_out,
                                                     uint32_t* __restrict__ hist_out, uint16_t* __restrict__ scratch,
                                                     size_t scratch_stride) {
    __shared__ MtfBlock<G> sh;
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    const int t = threadIdx.x, j = lane_id(), w = wave_id();
    const int n = (int)uniform(lens[b]);
    const uint8_t* X = bwt + (size_t)b * stride;
    uint16_t* out = mtf_out + (size_t)b * mtf_stride;
    MtfWave& W = sh.w[w];
    [[maybe_unused]] const bool stamp = b == nblocks / 2;
    BZ2MI_PHASE(g_mtf_phase, 0, stamp);

    for (int s = t; s < kMaxAlpha; s += 64 * G) sh.hist[s] = 0;
    for (int s = j; s < 256; s += 64) W.occ[s] = 0;
    if (j < 8) W.fset[j] = 0;
    if (t < 2) sh.runs[t] = 0;
    // initial list: the symbols in use, ascending; lane j places symbols 4j..4j+3
    const uint32_t nib = (present[(size_t)b * 8 + (j >> 3)] >> ((j & 7) * 4)) & 15u;
    const uint32_t pinc = wave_incl_sum((uint32_t)__popc(nib));
    const int k = (int)uniform((uint32_t)__builtin_amdgcn_readlane((int)pinc, 63));
    if (G == 1 || w == 0) {
        uint32_t r = pinc - (uint32_t)__popc(nib);
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (nib >> e & 1u) {
                if constexpr (G == 1) {
                    W.pos[4 * j + e] = (uint8_t)r;
                    W.lst[r] = (uint8_t)(4 * j + e);
                } else {
                    sh.sg.init[r] = (uint8_t)(4 * j + e);
                }
                r++;
            }
    }
    uint32_t na = 0, nb = 0;
    if constexpr (G == 1) {
        wave_sync_lds();
        const uint32_t o = mtf_range(X, 0, n, k, W, sh.hist, out, na, nb);
        sh.cnt[0] = o;
    } else {
        // ---- segment starts: the first symbol change at or after w * n / G
        if (j == 0) sh.seg[G] = (uint32_t)n;
        {
            int p = w == 0 ? 0 : max(1, (int)(((long long)w * n) / G));
            if (w > 0) {
                int found = n;
                for (int at = p; at < n; at += 64) {
                    const int i = at + j;
                    const bool chg = i < n && X[i] != X[i - 1];
                    const uint64_t m = __ballot(chg);
                    if (m) {
                        found = at + __builtin_ctzll(m);
                        break;
                    }
                }
                p = found;
            }
            if (j == 0) sh.seg[w] = (uint32_t)p;
        }
        __syncthreads();
        const int p0 = (int)sh.seg[w], p1 = max(p0, (int)sh.seg[w + 1]);
        // ---- the segment's distinct symbols by last occurrence (most recent
        // first); the occurrence masks hold the last occurrences meanwhile
        if (w < G - 1) {
            uint32_t* last = reinterpret_cast<uint32_t*>(W.occ);
            for (int s = j; s < 256; s += 64) last[s] = 0;
            wave_sync_lds();
            for (int at = p0 + j; at < p1; at += 64) atomicMax(&last[X[at]], (uint32_t)(at + 1));
            wave_sync_lds();
            uint32_t key[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t c = (uint32_t)(e * 64 + j), l = last[c];
                key[e] = l ? ~((l << 8) | c) : 0xffffffffu;  // ascending = most recent first
            }
            wave_bitonic256(key);
            uint32_t d = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (key[e] != 0xffffffffu) {
                    sh.sg.dl[w][e * 64 + j] = (uint8_t)(~key[e] & 255u);
                    d++;
                }
            }
            d = wave_sum(d);
            if (j == 0) sh.sg.dcnt[w] = d;
            for (int s = j; s < 256; s += 64) W.occ[s] = 0;
        }
        __syncthreads();
        // ---- start list: L_w = D_{w-1} ++ (L_{w-1} \ D_{w-1}), from the initial list
        {
            uint8_t* mk = sh.sg.mark[w];
            for (int r = j; r < k; r += 64) W.lst[r] = sh.sg.init[r];
            for (int h = 0; h < w; ++h) {
                const uint32_t dh = sh.sg.dcnt[h];
                for (int s = j; s < 256; s += 64) mk[s] = 0;
                wave_sync_lds();
                for (uint32_t r = j; r < dh; r += 64) mk[sh.sg.dl[h][r]] = 1;
                wave_sync_lds();
                // the kept entries of L, in order, after D_h (4 list positions per lane)
                const uint32_t lw = reinterpret_cast<const uint32_t*>(W.lst)[j];
                uint32_t keep = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t rpos = 4u * (uint32_t)j + e;
                    keep |= (rpos < (uint32_t)k && !mk[(lw >> (8 * e)) & 255u]) ? 1u << e : 0u;
                }
                const uint32_t kc = (uint32_t)__popc(keep);
                uint32_t np = dh + wave_incl_sum(kc) - kc;
                wave_sync_lds();  // every lane has read its list word
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (keep >> e & 1u) W.lst[np++] = (uint8_t)((lw >> (8 * e)) & 255u);
                for (uint32_t r = j; r < dh; r += 64) W.lst[r] = sh.sg.dl[h][r];
                wave_sync_lds();
            }
            for (int r = j; r < k; r += 64) W.pos[W.lst[r]] = (uint8_t)r;
            wave_sync_lds();
        }
        uint16_t* so = scratch + (size_t)b * scratch_stride + p0;
        const uint32_t o = p1 > p0 ? mtf_range(X, p0, p1, k, W, sh.hist, so, na, nb) : 0u;
        if (j == 0) sh.cnt[w] = o;
        __syncthreads();
        // ---- concatenate the segments
        uint32_t off = 0;
        for (int h = 0; h < w; ++h) off += sh.cnt[h];
        for (uint32_t i = j; i < o; i += 64) out[off + i] = so[i];
    }
    const uint32_t runA = wave_sum(na), runB = wave_sum(nb);
    if (j == 0) {
        atomicAdd(&sh.runs[0], runA);
        atomicAdd(&sh.runs[1], runB);
    }
    __syncthreads();
    BZ2MI_PHASE(g_mtf_phase, 1, stamp);
    uint32_t total = 0;
    for (int h = 0; h < G; ++h) total += sh.cnt[h];
    const uint32_t eob = (uint32_t)k + 1;
    if (t == 0) {
        out[total] = (uint16_t)eob;
        mtf_len[b] = total + 1;
        alpha_out[b] = eob + 1;
    }
    uint32_t* H = hist_out + (size_t)b * kMaxAlpha;
    for (int s = t; s < kMaxAlpha; s += 64 * G) {
        uint32_t h = sh.hist[s];
        if (s == 0) h += sh.runs[0];
        if (s == 1) h += sh.runs[1];
        if ((uint32_t)s == eob) h += 1;
        H[s] = h;
    }
}

void launch_mtf(int nb, const uint8_t* bwt, size_t stride, const uint32_t* lens, const uint32_t* present,
                uint16_t* mtf_out, size_t mtf_stride, uint32_t* mtf_len, uint32_t* alpha_out, uint32_t* hist_out,
                uint16_t* scratch, size_t scratch_stride, hipStream_t s) {
    // waves per block: one while the blocks alone fill the chip's SIMDs
    // several times over (each wave's tile chain is latency-bound below ~6
    // waves per SIMD), else segments
    // (1 GiB batches take G = 1, the 900 KB mode (1,193 blocks per GiB) 16 --
    // measured 5.95 vs 6.43 ms for G = 8 --, small batches 4 / 16; G = 8 only
    // in A/B builds: -DBZ2MI_AB_MTF_WAVES=G)
#ifdef BZ2MI_AB_MTF_WAVES
    const int g = BZ2MI_AB_MTF_WAVES;
#else
    static const int g_env = [] {
        const char* e = getenv("BZ2MI_MTF_WAVES");  // A/B knob: 1, 2, 4, 8 or 16
        return e && *e ? atoi(e) : 0;
    }();
    const int g = g_env ? g_env : nb >= 6144 ? 1 : nb >= 3072 ? 2 : nb >= 1536 ? 4 : 16;
#endif
#define BZ2MI_MTF_LAUNCH(G)                                                                                     \
    hipLaunchKernelGGL(mtf_kernel<G>, dim3(nb), dim3(64 * G), 0, s, bwt, stride, lens, nb, present, mtf_out,      \
                       mtf_stride, mtf_len, alpha_out, hist_out, scratch, scratch_stride)
    switch (g) {
        case 1: BZ2MI_MTF_LAUNCH(1); break;
        case 2: BZ2MI_MTF_LAUNCH(2); break;
        case 4: BZ2MI_MTF_LAUNCH(4); break;
        case 8: BZ2MI_MTF_LAUNCH(8); break;
        default: BZ2MI_MTF_LAUNCH(16); break;
    }
#undef BZ2MI_MTF_LAUNCH
}

}  // namespace bz2mi
