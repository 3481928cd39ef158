// Device RLE1 front end: run-length pre-pass, block split and block CRCs of a
// raw byte stream resident in HBM.
//
// Semantics: BlockCompressor::write / writeRun / finishRLE
// (reference include/BlockCompressor.hpp:69-154) as driven by
// OutputStream::write / getNextCompressor (OutputStream.hpp:131-142,
// 179-188).  A byte is refused by a block once more than S-6 RLE1 bytes have
// been flushed into it; a flush happens when a run changes value (flushing
// the previous run's last piece) or when a run piece reaches 255 bytes.
//
// Parallel formulation (all per-byte work is data parallel; only the block
// chain is sequential and it touches one byte per block):
//   cost(i)  output bytes flushed by the write of byte i in an unsplit stream
//            (0, or the size 1/2/3/5 of the piece it completes)
//   Fg(i)    sum of cost(j), j < i      (chunk-level prefix Fc + in-chunk scan)
//   Ginv(y)  min { i : Fg(i) > y }
// A block that starts at a run start p ends at E(p) = Ginv(Fg(p+1) + S - 6).
// D[y] (one byte per output position y) holds Fg(Ginv(y)+1) - y and whether
// Ginv(y) starts a run, so the chain advances a block per D lookup:
// y_{k+1} = y_k + D[y_k] + S - 6.  Blocks that start inside a run (rare:
// the byte after the crossing flush repeats its predecessor) take a slow path
// that re-phases the run's 255-byte pieces from the block start.
#include "common.hpp"
#include "kernels.hpp"
#include "rle1.hpp"

namespace bz2mi {

BZ2MI_PHASE_TABLE(g_fe_phase)

// chain kernel: stamps at the first 16 window starts
int fe_phases(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fe_phase), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

namespace {

constexpr int CH = 4096;  // chunk bytes (one wave: 64 lanes x 64 bytes)

__device__ __forceinline__ uint32_t piece_cost(uint32_t len) {  // output bytes of a piece
    return len >= 4 ? 5u : len;
}

// the 64 bytes of lane `l` of a chunk as 16 dwords (zero beyond n)
__device__ __forceinline__ void load16w(const uint8_t* x, uint64_t n, uint64_t at, uint32_t (&w)[16]) {
    if (at + 64 <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(x + at);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 a = p[q];
            w[4 * q] = a.x, w[4 * q + 1] = a.y, w[4 * q + 2] = a.z, w[4 * q + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            uint32_t d = 0;
            for (int r = 0; r < 4; ++r)
                if (at + 4 * q + r < n) d |= (uint32_t)x[at + 4 * q + r] << (8 * r);
            w[q] = d;
        }
    }
}

// bit q: byte q of the lane's 64 differs from the byte before it (byte 0:
// from `prev_last`), by SWAR on the dwords
__device__ __forceinline__ uint64_t rs_mask(const uint32_t (&w)[16], uint32_t prev_last) {
    uint64_t m = 0;
    uint32_t top = prev_last & 255u;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t d = w[k];
        const uint32_t t = d ^ ((d << 8) | top);
        const uint32_t nz = (((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
        const uint32_t bits = ((nz >> 7) & 1u) | ((nz >> 14) & 2u) | ((nz >> 21) & 4u) | ((nz >> 28) & 8u);
        m |= (uint64_t)bits << (4 * k);
        top = d >> 24;
    }
    return m;
}

// whether chunk c starts a run (its first byte differs from the byte before it)
__device__ __forceinline__ bool chunk_starts_run(const uint4* summ, uint64_t c) {
    return c == 0 || (summ[c].x & 0xffu) != ((summ[c - 1].x >> 8) & 0xffu);
}

// Per-byte trigger costs (cost(i) of the header comment) of lane `lane`'s 64
// bytes of chunk c, packed four to a dword; returns the lane's sum.  Called by
// the whole wave (run starts are scanned across the lanes).  rsbc = rsb[c]
// (the start of the run that holds the byte before the chunk).
__device__ __forceinline__ uint64_t lane_rs(const uint32_t (&w)[16], uint64_t c, uint32_t len, bool chunk_rs) {
    const int lane = lane_id();
    const uint32_t prev_last = (uint32_t)__shfl_up((int)(w[15] >> 24), 1);
    uint64_t m = rs_mask(w, prev_last);
    if (lane == 0) m = (m & ~1ull) | (chunk_rs ? 1ull : 0ull);
    const int valid = (int)min(64u, len > (uint32_t)lane * 64u ? len - (uint32_t)lane * 64u : 0u);
    (void)c;
    return valid >= 64 ? m : (m & ((1ull << valid) - 1ull));
}

// 1 + the last run start (chunk-relative) in the lanes before this one, 0 if none
__device__ __forceinline__ uint32_t lane_before(uint64_t m) {
    const int lane = lane_id();
    const uint32_t lrs = m ? (uint32_t)lane * 64u + 64u - (uint32_t)__clzll((long long)m) : 0u;  // last start + 1
    uint32_t xs = lrs;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)xs, d);
        if (lane >= d) xs = xs > y ? xs : y;
    }
    uint32_t before = (uint32_t)__shfl_up((int)xs, 1);
    if (lane == 0) before = 0;
    return before;
}

// run start in effect before the lane's first byte (absolute)
__device__ __forceinline__ uint64_t lane_run_start(uint64_t m, uint64_t c, uint64_t rsbc) {
    const uint32_t before = lane_before(m);
    return before ? c * CH + before - 1 : (c == 0 ? 0 : rsbc);
}

// the costs of the lane's bytes q < qend from its run-start mask; packed
// four to a dword when PACK
template <bool PACK>
__device__ __forceinline__ uint32_t lane_cost_walk(uint64_t m, uint64_t at, uint64_t cur, uint32_t qend,
                                                   uint32_t (&packed)[16]) {
    uint32_t ph = (uint32_t)((at - cur) % 255u);
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < 64; ++q) {
        uint32_t cst = 0;
        if ((m >> q) & 1u) {
            if (at + q > 0) cst = piece_cost(ph);
            ph = 0;
        } else if (ph == 254u) {
            cst = 5;
        }
        ph = ph == 254u ? 0u : ph + 1u;
        cst = (uint32_t)q < qend ? cst : 0u;
        sum += cst;
        if constexpr (PACK) {
            if ((q & 3) == 0) packed[q >> 2] = cst;
            else packed[q >> 2] |= cst << ((q & 3) * 8);
        }
    }
    return sum;
}

__device__ __forceinline__ uint32_t lane_costs(const uint32_t (&w)[16], uint64_t c, uint32_t len, bool chunk_rs,
                                               uint64_t rsbc, uint32_t (&packed)[16], uint32_t* ph0) {
    const uint64_t at = c * CH + (uint64_t)lane_id() * 64;
    const uint64_t m = lane_rs(w, c, len, chunk_rs);
    const uint64_t cur = lane_run_start(m, c, rsbc);
    *ph0 = (uint32_t)((at - cur) % 255u);
    const uint32_t qend = len > (uint32_t)lane_id() * 64u ? min(64u, len - (uint32_t)lane_id() * 64u) : 0u;
    return lane_cost_walk<true>(m, at, cur, qend, packed);
}

// cost of the first byte of chunk c (c < nc) from the scans alone
__device__ __forceinline__ uint32_t chunk_first_cost(const uint4* summ, const uint64_t* rsb, uint64_t c) {
    if (c == 0) return 0;
    const uint32_t ph = (uint32_t)((c * CH - rsb[c]) % 255u);
    return chunk_starts_run(summ, c) ? piece_cost(ph) : (ph == 254u ? 5u : 0u);
}

}  // namespace

// ---- K1: per-chunk run summary
__global__ __launch_bounds__(256) void fe_summary_kernel(const uint8_t* __restrict__ x, uint64_t n, uint64_t nc,
                                                         uint4* __restrict__ summ, uint32_t* __restrict__ cfree) {
    const uint64_t c = (uint64_t)blockIdx.x * 4 + wave_id();
    if (c >= nc) return;
    const int lane = lane_id();
    const uint64_t c0 = c * CH;
    const uint32_t len = (uint32_t)min((uint64_t)CH, n - c0);
    const uint64_t at = c0 + (uint64_t)lane * 64;
    uint32_t w[16];
    load16w(x, n, at, w);
    // run starts inside the chunk (pos >= 1)
    const uint64_t m = lane_rs(w, c, len, false);
    const uint32_t lfirst = m ? (uint32_t)lane * 64u + (uint32_t)__builtin_ctzll(m) : 0xffffffffu;
    const uint32_t llast = m ? (uint32_t)lane * 64u + 63u - (uint32_t)__clzll((long long)m) : 0u;
    uint32_t first_rs = lfirst, last_rs = llast;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        first_rs = min(first_rs, (uint32_t)__shfl_xor((int)first_rs, d));
        last_rs = max(last_rs, (uint32_t)__shfl_xor((int)last_rs, d));
    }
    const uint32_t lead = first_rs == 0xffffffffu ? len : first_rs;
    // the context-free part of the chunk's cost: the bytes after the first run
    // start inside the chunk (lead), whose runs all start in the chunk; the
    // bytes up to lead depend on the run that comes in (fe_costscan_kernel).
    // Walked as if the chunk's first run started at lead; bytes <= lead dropped.
    const uint32_t lo = (uint32_t)lane * 64u, before = lane_before(m);
    uint64_t keep = lead + 1 > lo ? (lead + 1 - lo >= 64 ? 0ull : ~0ull << (lead + 1 - lo)) : ~0ull;  // pos > lead
    const uint32_t qend = len > lo ? min(64u, len - lo) : 0u;                                         // pos < len
    keep &= qend >= 64 ? ~0ull : ((1ull << qend) - 1ull);
    // (a lane after lead has a run start before it; a lane holding lead
    // restarts its phase there)
    uint32_t ph = (lo - (before ? before - 1 : 0u)) % 255u;
    uint32_t fsum = 0;
#pragma unroll
    for (int q = 0; q < 64; ++q) {
        uint32_t cst = 0;
        if ((m >> q) & 1u) {
            cst = piece_cost(ph);
            ph = 0;
        } else if (ph == 254u) {
            cst = 5;
        }
        ph = ph == 254u ? 0u : ph + 1u;
        fsum += ((keep >> q) & 1u) ? cst : 0u;
    }
    fsum = wave_sum(fsum);
    if (lane == 0) {
        const uint32_t trail = len - last_rs;
        const uint32_t fb = x[c0], lb = x[c0 + len - 1];
        summ[c] = make_uint4(fb | (lb << 8), lead, trail, len);
        cfree[c] = fsum;
    }
}

// ---- K2/K4: scans over chunks, one tile of kScanTile chunks per workgroup,
// in two launches: pass 0 leaves every tile's aggregate in agg[], pass 1
// folds the aggregates of the earlier tiles into a carry and scans its tile
// with it (the tiles' loads are all in flight at once instead of one tile
// after another on one workgroup: 0.49 + 0.18 ms per GiB before).
constexpr int kScanE = 8, kScanTile = kFeScanThreads * kScanE;
static_assert(kScanTile == kFeScanTile, "scan tile");

// inclusive scan over the workgroup of per-thread values (op: max or sum);
// returns the thread's exclusive prefix (from `carry`) and the new carry
template <bool kMax>
__device__ __forceinline__ uint64_t wg_scan_1024(uint64_t v, uint64_t carry, uint64_t* wt, uint64_t* total) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    uint64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(incl, d);
        if (lane >= d) incl = kMax ? (incl > o ? incl : o) : incl + o;
    }
    if (lane == 63) wt[w] = incl;
    __syncthreads();
    uint64_t pre = carry, all = carry;
#pragma unroll
    for (int q = 0; q < kFeScanThreads / 64; ++q) {
        const uint64_t t = wt[q];
        if (q < w) pre = kMax ? (pre > t ? pre : t) : pre + t;
        all = kMax ? (all > t ? all : t) : all + t;
    }
    __syncthreads();
    *total = all;
    // exclusive (for sums) / inclusive-of-earlier-threads (for max) prefix
    const uint64_t before = __shfl_up(incl, 1);
    if (lane == 0) return pre;
    return kMax ? (pre > before ? pre : before) : pre + before;
}

// rsb[c] = start of the run that holds byte c*CH-1 (c >= 1): an inclusive
// max-scan of the trailing-run start of every chunk that starts a new run.
// carry into tile g: op over agg[0..g-1]
template <bool kMax>
__device__ __forceinline__ uint64_t tile_carry(const uint64_t* __restrict__ agg, uint64_t g, uint64_t* wt) {
    uint64_t v = 0;
    for (uint64_t q = threadIdx.x; q < g; q += kFeScanThreads) {
        const uint64_t a = agg[q];
        v = kMax ? (v > a ? v : a) : v + a;
    }
    uint64_t all;
    (void)wg_scan_1024<kMax>(v, 0, wt, &all);
    return all;
}

__global__ __launch_bounds__(kFeScanThreads) void fe_runscan_kernel(const uint4* __restrict__ summ, uint64_t nc,
                                                                    uint64_t* __restrict__ rsb,
                                                                    uint64_t* __restrict__ agg, int pass) {
    __shared__ uint64_t wt[kFeScanThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
    const uint64_t c = base + (uint64_t)threadIdx.x * kScanE;
    uint4 cur[kScanE + 1];
#pragma unroll
    for (int e = 0; e <= kScanE; ++e) {  // cur[0] = chunk c-1
        const uint64_t cc = c + (uint64_t)e - 1;
        cur[e] = (c + e >= 1 && cc < nc) ? summ[cc] : make_uint4(0, 0, 0, 0);
    }
    const uint64_t carry = pass ? tile_carry<true>(agg, blockIdx.x, wt) : 0ull;
    uint64_t own[kScanE], run = 0;
#pragma unroll
    for (int e = 0; e < kScanE; ++e) {
        const uint64_t ce = c + e;
        const uint4 sm = cur[e + 1];
        uint64_t o = 0;
        if (ce < nc) {
            if (sm.z != sm.w) {
                o = ce * CH + sm.w - sm.z;  // trailing run starts inside the chunk
            } else if (ce == 0 || (sm.x & 0xff) != ((cur[e].x >> 8) & 0xff)) {
                o = ce * CH;                // a one-run chunk that starts a new run
            }                               // else: the run continues
        }
        run = run > o ? run : o;
        own[e] = run;
    }
    uint64_t all;
    const uint64_t pre = wg_scan_1024<true>(run, carry, wt, &all);
    if (pass == 0) {
        if (threadIdx.x == 0) agg[blockIdx.x] = all;
        return;
    }
#pragma unroll
    for (int e = 0; e < kScanE; ++e)
        if (c + e < nc) rsb[c + e + 1] = pre > own[e] ? pre : own[e];
    if (blockIdx.x == 0 && threadIdx.x == 0) rsb[0] = 0;
}

// A chunk's cost = its context-free part (fe_summary_kernel) + the part of the
// run that comes in: with ph0 = (c*CH - rsb[c]) % 255 (the piece position of
// that run at the chunk start) and L = the chunk's lead, a chunk that starts a
// run pays the previous run's last piece first and its own first run starts
// at phase 0; either way the first run completes (p + L) / 255 pieces of 255
// bytes in the chunk (5 bytes each) and, when it ends inside the chunk, pays
// its last piece at byte L.
__global__ __launch_bounds__(kFeScanThreads) void fe_costscan_kernel(const uint32_t* __restrict__ cfree,
                                                                     const uint4* __restrict__ summ,
                                                                     const uint64_t* __restrict__ rsb, uint64_t nc,
                                                                     uint64_t* __restrict__ fc,
                                                                     uint64_t* __restrict__ agg, int pass) {
    __shared__ uint64_t wt[kFeScanThreads / 64];
    static_assert(kScanE == 8, "two uint4 loads per thread");
    const uint64_t c = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanE;
    uint32_t cur[kScanE];
    if (c + kScanE <= nc) {
        const uint4 a = *reinterpret_cast<const uint4*>(cfree + c);
        const uint4 b = *reinterpret_cast<const uint4*>(cfree + c + 4);
        cur[0] = a.x, cur[1] = a.y, cur[2] = a.z, cur[3] = a.w, cur[4] = b.x, cur[5] = b.y, cur[6] = b.z, cur[7] = b.w;
    } else {
#pragma unroll
        for (int e = 0; e < kScanE; ++e) cur[e] = c + e < nc ? cfree[c + e] : 0u;
    }
#pragma unroll
    for (int e = 0; e < kScanE; ++e) {
        const uint64_t ce = c + e;
        if (ce >= nc) continue;
        const uint4 sm = summ[ce];
        const uint32_t L = sm.y, len = sm.w;
        const uint32_t ph0 = ce ? (uint32_t)((ce * CH - rsb[ce]) % 255u) : 0u;
        uint32_t p = ph0, add = 0;
        if (chunk_starts_run(summ, ce)) {
            if (ce) add = piece_cost(ph0);
            p = 0;
        }
        add += 5u * ((p + L) / 255u);
        if (L < len) add += piece_cost((p + L) % 255u);
        cur[e] += add;
    }
    const uint64_t carry = pass ? tile_carry<false>(agg, blockIdx.x, wt) : 0ull;
    uint64_t ex[kScanE], run = 0;
#pragma unroll
    for (int e = 0; e < kScanE; ++e) {
        ex[e] = run;
        run += cur[e];
    }
    uint64_t all;
    const uint64_t pre = wg_scan_1024<false>(run, carry, wt, &all);
    if (pass == 0) {
        if (threadIdx.x == 0) agg[blockIdx.x] = all;
        return;
    }
#pragma unroll
    for (int e = 0; e < kScanE; ++e)
        if (c + e < nc) fc[c + e] = pre + ex[e];
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) fc[nc] = all;
}

// ---- K5: D map over output positions.  A chunk's entries cover the output
// range [fc[c], fc[c+1]) exactly once: they are built in LDS by the lanes
// (64 input bytes each) and written out as one coalesced run.
constexpr int kDmapMax = CH + CH / 4 + 64;  // RLE1 output of one chunk, at most 5/4 of its bytes

__global__ __launch_bounds__(256) void fe_dmap_kernel(const uint8_t* __restrict__ x, const uint4* __restrict__ summ,
                                                      const uint64_t* __restrict__ rsb, uint64_t n, uint64_t nc,
                                                      const uint64_t* __restrict__ fc, uint8_t* __restrict__ dmap,
                                                      uint32_t* __restrict__ laneinfo) {
    // (a padded layout -- 4 bytes every 64, lanes' stores on distinct banks --
    // removed the bank conflicts but measured 6 % slower: 1.216 vs 1.148 ms)
    __shared__ uint8_t stage[4][kDmapMax + 64];  // + one sink byte per lane
    const uint64_t c = (uint64_t)blockIdx.x * 4 + wave_id();
    if (c >= nc) return;
    uint8_t* st = stage[wave_id()];
    const int lane = lane_id();
    const uint64_t c0 = c * CH;
    const uint64_t at = c0 + (uint64_t)lane * 64;
    // 64 input bytes as 16 dwords (plus the next 4), their costs recomputed
    // (the per-byte cost array is not materialised)
    uint32_t xv[17], kv[17], ph0 = 0;
    {
        uint32_t w[16];
        load16w(x, n, at, w);
#pragma unroll
        for (int q = 0; q < 16; ++q) xv[q] = w[q];
        uint32_t nx = 0;
        if (at + 68 <= n) {
            nx = *reinterpret_cast<const uint32_t*>(x + at + 64);
        } else {
            for (int r = 0; r < 4; ++r)
                if (at + 64 + r < n) nx |= (uint32_t)x[at + 64 + r] << (8 * r);
        }
        xv[16] = nx;
        const uint32_t len = (uint32_t)min((uint64_t)CH, n - c0);
        uint32_t pk[16];
        (void)lane_costs(w, c, len, chunk_starts_run(summ, c), c ? rsb[c] : 0ull, pk, &ph0);
#pragma unroll
        for (int q = 0; q < 16; ++q) kv[q] = pk[q];
        // cost of the byte after the lane: the next lane's first, or the next chunk's
        uint32_t kn = (uint32_t)__shfl_down((int)(pk[0] & 255u), 1);
        if (lane == 63) kn = (c + 1 < nc && at + 64 < n) ? chunk_first_cost(summ, rsb, c + 1) : 0u;
        kv[16] = kn;
    }
    uint32_t lsum = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const uint32_t kw = kv[q];
        lsum += (kw & 255u) + ((kw >> 8) & 255u) + ((kw >> 16) & 255u) + (kw >> 24);
    }
    const uint32_t incl = wave_incl_sum(lsum);
    uint32_t fl = incl - lsum;  // chunk-local output position
    // for the chain's in-chunk lookups: the lane's cost prefix and its phase
    laneinfo[c * 64 + (uint64_t)lane] = fl | (ph0 << 16);
    const uint32_t ctot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    // (entries of the last byte or two of the input stay unwritten: no target
    // reaches them)
    const uint64_t lim_i = n >= 2 ? n - 2 : 0;  // bytes i <= n-2 have entries
    // entry r of byte q's piece: Fg(i+2) - y = ci + kn - r, run-start flag.
    // The first entry is one unconditional store (to the lane's sink byte when
    // the byte flushes nothing); pieces of 2+ bytes (run ends) add the rest.
    const uint64_t span = at <= lim_i ? lim_i - at : 0;
    const uint32_t lim_q = at <= lim_i ? (uint32_t)(span < 63u ? span : 63u) + 1u : 0u;  // bytes q < lim_q have entries
    const uint32_t sink = (uint32_t)kDmapMax + (uint32_t)lane;
    // the byte before the lane's first (previous lane, previous chunk)
    uint32_t vprev = (uint32_t)__shfl_up((int)(xv[15] >> 24), 1);
    if (lane == 0) vprev = at > 0 ? (uint32_t)x[at - 1] : 0x100u;
#pragma unroll
    for (int q = 0; q < 64; ++q) {
        const uint32_t ci = (kv[q >> 2] >> ((q & 3) * 8)) & 255u;
        const uint32_t vq = (xv[q >> 2] >> ((q & 3) * 8)) & 255u;
        const uint32_t vn = (xv[(q + 1) >> 2] >> (((q + 1) & 3) * 8)) & 255u;
        const uint32_t kn = (kv[(q + 1) >> 2] >> (((q + 1) & 3) * 8)) & 255u;
        uint32_t hi = (vn != vq) ? 16u : 0u;
        // A block that would start at i+1 inside a run of 2 or 3 bytes that
        // begins at i (x[i-1] != x[i] == x[i+1]) is written here as a fast
        // step: the block's own run is the L-1 bytes [i+1, e), whose RLE1
        // output is L-1 bytes, while the unsplit costs flush all L of them at
        // e -- so its target is Fg(i+2) + 1 + S-6 (D one larger), what the
        // chain's mid-run path (slow_from) computes with e and Fg(e+1).
        // Longer runs (4+: count bytes, pieces) keep that path.
        uint32_t dadj = 0;
        if (hi == 0u && q + 3 <= 66) {
            const uint32_t v2 = (xv[(q + 2) >> 2] >> (((q + 2) & 3) * 8)) & 255u;
            const uint32_t v3 = (xv[(q + 3) >> 2] >> (((q + 3) & 3) * 8)) & 255u;
            const uint32_t vp = q == 0 ? vprev : (xv[(q - 1) >> 2] >> (((q - 1) & 3) * 8)) & 255u;
            const bool short_run = vp != vq && (v2 != vn || v3 != v2) && at + (uint64_t)q + 3 < n;
            if (short_run) {
                hi = 16u;
                dadj = 1u;
            }
        }
        const bool has = ci != 0 && (uint32_t)q < lim_q;
        st[has ? fl : sink] = (uint8_t)(((ci + kn + dadj) & 15u) | hi);
        if (has && ci > 1) {
#pragma unroll
            for (uint32_t r = 1; r < 5; ++r) st[r < ci ? fl + r : sink] = (uint8_t)(((ci + kn + dadj - r) & 15u) | hi);
        }
        fl += ci;
    }
    uint8_t* dst = dmap + fc[c];
    for (uint32_t j = lane; j < ctot; j += 64) dst[j] = st[j];
}

namespace {

struct FeView {
    const uint8_t* x;
    const uint32_t* lane;  // per 64-byte lane of a chunk: cost prefix | phase << 16 (fe_dmap_kernel)
    const uint64_t* fc;
    const uint4* summ;
    uint64_t n, nc;
    uint64_t fc_end;  // fc[nc], loaded once
};

// cost of byte at + lane of the 64-byte lane window at `at` (whole wave, one
// byte per lane); ph0 = the piece phase before the window's first byte
__device__ __forceinline__ uint32_t window_byte_cost(const FeView& f, uint64_t at, uint32_t ph0) {
    const int lane = lane_id();
    const uint64_t p = at + (uint64_t)lane;
    const bool in = p < f.n;
    const uint32_t b = in ? f.x[p] : 0u, pb = (in && p > 0) ? f.x[p - 1] : 0u;
    const bool rs = in && (p == 0 || b != pb);
    uint32_t xs = rs ? (uint32_t)lane + 1u : 0u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)xs, d);
        if (lane >= d) xs = xs > y ? xs : y;
    }
    uint32_t e = (uint32_t)__shfl_up((int)xs, 1);
    if (lane == 0) e = 0;
    const uint32_t ph = e ? ((uint32_t)lane - (e - 1)) % 255u : (ph0 + (uint32_t)lane) % 255u;  // before byte p
    if (!in) return 0u;
    return rs ? (p > 0 ? piece_cost(ph) : 0u) : (ph == 254u ? 5u : 0u);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return (uint64_t)hi << 32 | lo;
}

// Fg(i) by one wave: chunk prefix + lane prefix + the window's bytes below i
// (all lanes return it)
__device__ __forceinline__ uint64_t fg_at(const FeView& f, uint64_t i) {
    if (i >= f.n) return f.fc_end;
    const uint64_t c = i / CH, c0 = c * CH;
    const uint32_t L = (uint32_t)((i - c0) >> 6);
    const uint64_t at = c0 + 64u * L;
    const uint32_t info = f.lane[c * 64 + L];
    const uint32_t v = window_byte_cost(f, at, info >> 16);
    const uint32_t s = wave_sum(at + (uint64_t)lane_id() < i ? v : 0u);
    return f.fc[c] + (info & 0xffffu) + s;
}

// cost of byte i (whole wave)
__device__ __forceinline__ uint32_t byte_cost(const FeView& f, uint64_t i) {
    const uint64_t c = i / CH, c0 = c * CH;
    const uint32_t L = (uint32_t)((i - c0) >> 6);
    const uint64_t at = c0 + 64u * L;
    const uint32_t v = window_byte_cost(f, at, f.lane[c * 64 + L] >> 16);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(i - at));
}

// Ginv(y) = min { i : Fg(i) > y } by one wave: a 65-ary search over the
// chunk prefixes (each lane probes one point per level), the lane prefixes
// of the chunk, then a scan of the 64 bytes that hold the crossing; n if none.
__device__ __forceinline__ uint64_t ginv(const FeView& f, uint64_t y) {
    if (f.fc_end <= y) return f.n;
    const int lane = lane_id();
    uint64_t lo = 0, hi = f.nc;  // fc[lo] <= y < fc[hi]
    while (hi - lo > 1) {
        const uint64_t q = lo + ((hi - lo) * (uint64_t)(lane + 1)) / 65u;
        const int cnt = __popcll(__ballot(f.fc[q] <= y));  // fc is monotone: a prefix of lanes
        const uint64_t nlo = cnt ? readlane64(q, cnt - 1) : lo;
        const uint64_t nhi = cnt < 64 ? readlane64(q, cnt) : hi;
        lo = nlo;
        hi = nhi;
    }
    const uint64_t c0 = lo * CH;
    const uint32_t nl = (uint32_t)((min(f.n, c0 + CH) - c0 + 63) >> 6);  // lanes holding bytes
    const uint32_t info = (uint32_t)lane < nl ? f.lane[lo * 64 + (uint64_t)lane] : 0xffffffffu;
    // the crossing lane: the last one whose prefix is <= y (lane 0's is 0)
    const uint64_t le = __ballot((uint32_t)lane < nl && f.fc[lo] + (info & 0xffffu) <= y);
    const int L = 63 - __clzll((long long)le);
    const uint32_t infoL = (uint32_t)__builtin_amdgcn_readlane((int)info, L);
    const uint64_t baseL = f.fc[lo] + (infoL & 0xffffu);
    const uint64_t atL = c0 + 64u * (uint64_t)L;
    const uint32_t cb = window_byte_cost(f, atL, infoL >> 16);
    const uint64_t hit = __ballot(baseL + wave_incl_sum(cb) > y);
    return hit ? atL + (uint64_t)__ffsll((long long)hit) : f.n;
}

// first index > p whose byte differs from x[p] (or n): whole chunks that are
// one run are skipped by their summaries, otherwise each lane compares 16
// bytes (four aligned dwords) per pass
__device__ uint64_t run_end(const FeView& f, uint64_t p) {
    const uint32_t v = f.x[p];
    const uint32_t vv = v * 0x01010101u;
    uint64_t at = p + 1;
    const int lane = lane_id();
    const uint64_t mis = (uint64_t)(reinterpret_cast<uintptr_t>(f.x) & 3u);
    for (;;) {
        if (at >= f.n) return f.n;
        const uint64_t c = at / CH;
        if (at == c * CH && c < f.nc) {
            const uint4 s = f.summ[c];
            if (s.z == s.w && (s.x & 0xff) == v) {
                at += s.w;
                continue;
            }
        }
        // dword-aligned base (as an index relative to x, may be up to 3 below at)
        const uint64_t base = ((at + mis) & ~3ull) - mis;
        uint32_t off = 64;
#pragma unroll
        for (int j = 3; j >= 0; --j) {
            const uint64_t b = base + 4u * (uint64_t)(lane * 4 + j);
            uint32_t d = 0xffffffffu;
            if (b + 4 <= at) {
                d = 0;  // wholly before at
            } else if (b < f.n) {
                d = *reinterpret_cast<const uint32_t*>(f.x + b) ^ vv;
                if (b < at) d &= ~0u << (8 * (uint32_t)(at - b));
            }
            if (d) off = 4u * j + (__builtin_ctz(d) >> 3);
        }
        const uint64_t m = __ballot(off < 64);
        if (m) {
            const int L = __ffsll((long long)m) - 1;
            const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)off, L);
            const uint64_t e = base + 16u * (uint64_t)L + o;
            return e < f.n ? e : f.n;
        }
        at = base + 1024;
    }
}

}  // namespace

// ---- K6: the block chain (one workgroup) of one unit of the stream: the
// buffer holds the unit's own bytes [0, n_own) and a tail halo [n_own, n) of
// the bytes that follow it (n_own == n: the unit ends the stream).  The
// unit's first block starts at entry (bit 63: mid-run, i.e. x[p] == x[p-1] in
// the whole stream); blocks follow until the next start is >= n_own.
// bnd[j] is the end (= start of the next block) of block j, either as a target
// y (bit 63 clear: position Ginv(y)) or as an explicit position (bit 63 set);
// bnd[nb-1] is the unit's exit (n when the stream ends).  out[0] = nb,
// out[1] = status (0 ok, 1 the last block runs past a halo that does not
// reach the stream end, 2 overflow).
// The chain depends only on the bytes from the entry on (RLE1 state restarts
// at every block start), so a unit's front end treats its buffer as a stream
// of its own and the entry comes from the previous unit (bz2mi_shard_chain).
__global__ __launch_bounds__(kFeChainThreads) void fe_chain_kernel(const uint8_t* __restrict__ x, const uint32_t* __restrict__ laneinfo,
                                                      const uint64_t* __restrict__ fc, const uint4* __restrict__ summ,
                                                      const uint8_t* __restrict__ dmap, uint64_t n, uint64_t nc, int S,
                                                      uint64_t n_own, uint64_t entry, int ends,
                                                      uint64_t* __restrict__ bnd, uint64_t max_bnd,
                                                      uint64_t* __restrict__ nb_out,
                                                      const uint64_t* __restrict__ spec, uint64_t spec_nb) {
    FeView f{x, laneinfo, fc, summ, n, nc, uniform64(fc[nc])};
    constexpr uint64_t kExpl = 1ull << 63;
    if (n == 0 || n_own == 0) {
        if (threadIdx.x == 0) {
            nb_out[0] = 0;
            nb_out[1] = 0;
            nb_out[3] = 0;
        }
        return;
    }
    // ytot = Fg(n-1): targets y >= ytot have no start inside the buffer;
    // ystop = Fg(n_own-1): targets y >= ystop start at or after n_own
    const uint64_t ytot = fc[nc] - byte_cost(f, n - 1);
    const uint64_t ystop = n_own >= n ? ytot : uniform64(fg_at(f, n_own - 1));
    const uint64_t lim = (uint64_t)(S - 6);
    const uint32_t jstar = (uint32_t)((S - 6) / 5 + 1);
    // Case-A steps advance y by D + S-6 (D < 16).  A round covers the next
    // kStepsR steps: step m gets a 256-byte window of the D map around its
    // predicted position (running mean of D) and all waves turn every window
    // byte into a transition (offset of the next start in step m+1's window,
    // or a terminal code), then compose them into 8-step jumps.  Wave 0 then
    // chases the chain through the jumps (one LDS read per 8 blocks), takes
    // single steps near terminals, runs the mid-run slow path itself and
    // resumes the chase when the chain comes back into the windows.  The
    // offsets of jumped-over steps are replayed in parallel afterwards and
    // the block starts written out by all threads.
#ifndef BZ2MI_CHAIN_STEPS
#define BZ2MI_CHAIN_STEPS 256
#endif
    constexpr int kStepsR = BZ2MI_CHAIN_STEPS, kWin = 256, kJ = 16, kGroups = kStepsR / kJ;
    constexpr uint32_t kOut = 0x100, kMidRun = 0x200, kEnd = 0x300;  // kOut | D&15
    constexpr uint16_t kStop = 0xffff, kDirect = 0xffff;
    __shared__ uint16_t trans[kStepsR * kWin];
    __shared__ uint16_t jmp[kGroups * kWin];
    __shared__ uint16_t walk[kStepsR];  // offset of step m, or kDirect (bnd written by the slow path)
    __shared__ uint32_t jumped[kGroups];
    __shared__ uint64_t ctl[6];  // next round's y, k after the round, steps, mean D, done, exit
    const int tid = threadIdx.x;
    // chain state (wave 0; uniform)
    uint64_t k = 0;
    uint64_t y = 0;
    uint64_t status = 0;
    bool done = false;
    uint64_t exit_b = n | kExpl;
    uint64_t dsum = 0, dcnt = 0;  // (wave 0)
    uint64_t dfp = 8ull << 16;    // mean D, 16.16, for the window predictions
    uint64_t scur = 1, merged = 0;  // speculation: search cursor, spec index of the merge (0: none)
    [[maybe_unused]] int nwin = 0, nslow = 0;
#ifdef BZ2MI_PHASES
#define FE_NOW() wall_clock64()
#else
#define FE_NOW() 0ull
#endif
    unsigned long long t_tab = 0, t_ch = 0, t_bnd = 0, t_slow = 0, n_out = 0, n_mid = 0;
    // The slow path (wave 0): blocks that start inside a run (p, mid-run),
    // block by block, until the chain is back on a run start (returns true, y
    // set) or the unit's chain ends (returns false, exit_b set).  `direct`
    // records a block start found here.
    auto slow_from = [&](uint64_t p, auto&& direct) -> bool {
        for (;;) {
            if (k + 1 >= max_bnd) {
                status = 2;
                exit_b = n | kExpl;
                return false;
            }
            nslow++;
            // block starting at p, mid-run: its first run is [p, e)
            const uint64_t e = run_end(f, p);
            const uint64_t Lr = e - p;
            if ((uint64_t)jstar * 255u <= Lr) {
                const uint64_t E = p + (uint64_t)jstar * 255u;
                if (E >= n_own) {
                    exit_b = (E >= n ? n : E) | kExpl;
                    if (E >= n && !ends) status = 1;
                    return false;
                }
                direct(E | kExpl);
                if (E < e) {
                    p = E;  // still inside the run
                    continue;
                }
                // E == e: a run start
                y = fg_at(f, E + 1) + lim;
                return true;
            }
            if (e >= n) {  // the run reaches the end of the buffer: last block
                exit_b = n | kExpl;
                if (!ends) status = 1;
                return false;
            }
            const uint64_t tot = 5ull * (Lr / 255) + piece_cost((uint32_t)(Lr % 255));
            if (tot > lim) {
                const uint64_t E = e + 1;
                if (E >= n_own) {
                    exit_b = (E >= n ? n : E) | kExpl;
                    if (E >= n && !ends) status = 1;
                    return false;
                }
                direct(E | kExpl);
                if (f.x[E] != f.x[E - 1]) {
                    y = fg_at(f, E + 1) + lim;
                    return true;
                }
                p = E;
                continue;
            }
            // continue in unsplit coordinates after the run
            y = fg_at(f, e + 1) - tot + lim;
            return true;
        }
    };
    // entry: a run start (the target of the next block follows from Fg), or
    // mid-run (the slow path, wave 0, before the rounds)
    {
        const uint64_t p0 = entry & ~kExpl;
        if (!(entry >> 63)) {
            y = uniform64(fg_at(f, p0 + 1)) + lim;
        } else {
            if (tid < 64) {
                const bool have = slow_from(p0, [&](uint64_t v) {
                    if (tid == 0) bnd[k] = v;
                    k++;
                });
                if (tid == 0) {
                    ctl[0] = y;
                    ctl[1] = k;
                    ctl[4] = have ? 0 : 1;
                    ctl[5] = exit_b;
                    ctl[2] = status;
                }
            }
            __syncthreads();
            y = ctl[0];
            k = ctl[1];
            done = ctl[4] != 0;
            exit_b = ctl[5];
            status = ctl[2];
            __syncthreads();
        }
    }
    for (;;) {
        if (done) break;
        if (k + 1 >= max_bnd) {
            status = 2;
            exit_b = n | kExpl;
            break;
        }
        if (y >= ystop) {  // the next start is outside the unit: the exit
            exit_b = y >= ytot ? (n | kExpl) : y;
            if (y >= ytot && !ends) status = 1;
            break;
        }
        const unsigned long long tr = FE_NOW();
        BZ2MI_PHASE(g_fe_phase, nwin < 6 ? nwin : 5, nwin < 6);
        nwin++;
        const uint64_t ybase = y, k0 = k;
        // window of step m: 16-aligned, from 128 below the prediction but
        // not below step m's minimum position ybase + m (S-6)
        auto wstart_of = [&](uint64_t m) -> uint64_t {
            const uint64_t lo_m = ybase + m * lim;
            const uint64_t pm = lo_m + ((m * dfp) >> 16);
            return (pm >= lo_m + 128 ? pm - 128 : lo_m) & ~15ull;
        };
        static_assert(kStepsR * (kWin / 16) % kFeChainThreads == 0, "table items per thread");
#pragma unroll
        for (int it = tid; it < kStepsR * (kWin / 16); it += kFeChainThreads) {
            const int m = it >> 4, c = it & 15;
            const uint64_t ws = wstart_of((uint64_t)m), wsn = wstart_of((uint64_t)m + 1);
            const uint64_t y0 = ws + 16u * (uint64_t)c;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (y0 < ytot) v = *reinterpret_cast<const uint4*>(dmap + y0);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            uint32_t packed[8];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint64_t yy = y0 + (uint64_t)q;
                const uint32_t d = (w[q >> 2] >> (8 * (q & 3))) & 0xffu;
                uint32_t t;
                if (yy >= ystop) {
                    t = kEnd;
                } else if (!(d & 16u)) {
                    t = kMidRun;
                } else {
                    const uint64_t yn = yy + (d & 15u) + lim;
                    t = (m + 1 < kStepsR && yn >= wsn && yn < wsn + kWin) ? (uint32_t)(yn - wsn) : (kOut | (d & 15u));
                }
                if (q & 1) packed[q >> 1] |= t << 16;
                else packed[q >> 1] = t;
            }
            uint4* dst = reinterpret_cast<uint4*>(trans + m * kWin + 16 * c);
            dst[0] = make_uint4(packed[0], packed[1], packed[2], packed[3]);
            dst[1] = make_uint4(packed[4], packed[5], packed[6], packed[7]);
        }
        if (tid < kGroups) jumped[tid] = 0;
        __syncthreads();
        // jumps: group g covers the kJ steps from step kJ g (the last group
        // kJ - 1: step kStepsR - 1 always leaves the windows); kStop if a
        // terminal lies inside
        static_assert(kGroups * kWin % kFeChainThreads == 0, "jump items per thread");
        {
            constexpr int kPer = kGroups * kWin / kFeChainThreads;
            uint32_t o[kPer];
#pragma unroll
            for (int e = 0; e < kPer; ++e) o[e] = (uint32_t)((tid + e * kFeChainThreads) & (kWin - 1));
#pragma unroll
            for (int i = 0; i < kJ; ++i) {
#pragma unroll
                for (int e = 0; e < kPer; ++e) {
                    const int g = (tid + e * kFeChainThreads) / kWin;
                    if (o[e] < (uint32_t)kWin && g * kJ + i < kStepsR - 1) o[e] = trans[(g * kJ + i) * kWin + (int)o[e]];
                }
            }
#pragma unroll
            for (int e = 0; e < kPer; ++e) jmp[tid + e * kFeChainThreads] = o[e] < (uint32_t)kWin ? (uint16_t)o[e] : kStop;
        }
        __syncthreads();
        const unsigned long long t1 = FE_NOW();
        t_tab += t1 - tr;
        if (tid < 64) {
            int m = 0;
            uint32_t o = (uint32_t)(y - wstart_of(0));
            bool clean = true;
            auto direct = [&](uint64_t v) {  // a block start found by the slow path
                if (tid == 0) {
                    bnd[k] = v;
                    if (m < kStepsR) walk[m] = kDirect;
                }
                m++;
                k++;
            };
            for (;;) {
                if ((m & (kJ - 1)) == 0) {
                    const int len = m + kJ < kStepsR ? kJ : kJ - 1;
                    if (k + (uint64_t)len < max_bnd) {
                        const uint32_t j = (uint32_t)__builtin_amdgcn_readfirstlane((int)jmp[(m / kJ) * kWin + (int)o]);
                        if (j != kStop) {
                            if (tid == 0) {
                                walk[m] = (uint16_t)o;
                                jumped[m / kJ] = 1;
                            }
                            o = j;
                            m += len;
                            k += (uint64_t)len;
                            continue;
                        }
                    }
                }
                if (k + 1 >= max_bnd) {
                    y = wstart_of((uint64_t)m) + o;  // (the top of the next round reports the overflow)
                    break;
                }
                const uint32_t t = (uint32_t)__builtin_amdgcn_readfirstlane((int)trans[m * kWin + (int)o]);
                if (t < (uint32_t)kWin) {
                    if (tid == 0) walk[m] = (uint16_t)o;
                    o = t;
                    m++;
                    k++;
                    continue;
                }
                // a terminal at step m
                y = uniform64(wstart_of((uint64_t)m) + o);
                if (t == kEnd) break;  // y >= ystop: the exit (reported at the top of the next round)
                if (tid == 0) walk[m] = (uint16_t)o;  // the block at y itself
                m++;
                k++;
                if ((t & ~15u) == kOut) {  // next start outside the windows: new round from it
                    if (clean) {
                        dsum += y - ybase - (uint64_t)(m - 1) * lim;
                        dcnt += (uint64_t)(m - 1);
                    }
                    y = uniform64(y + (uint64_t)(t & 15u) + lim);
                    n_out++;
                    break;
                }
                // the next block starts inside a run: the slow path, block by
                // block, until the chain is back on a run start (have y)
                n_mid++;
                const unsigned long long ts = FE_NOW();
                if (clean) {
                    dsum += y - ybase - (uint64_t)(m - 1) * lim;
                    dcnt += (uint64_t)(m - 1);
                }
                clean = false;
                const uint64_t p = ginv(f, y);
                const bool have_y = slow_from(p, direct);
                t_slow += FE_NOW() - ts;
                if (!have_y) {
                    done = true;
                    break;
                }
                // back in the windows?  then the chase goes on
                if (m < kStepsR && y < ystop) {
                    const uint64_t ws = wstart_of((uint64_t)m);
                    if (y >= ws && y < ws + kWin) {
                        o = (uint32_t)(y - ws);
                        continue;
                    }
                }
                break;
            }
            if (tid == 0) {
                ctl[0] = y;
                ctl[1] = k;
                ctl[2] = (uint64_t)m;
                ctl[3] = dcnt ? (uint64_t)((float)dsum / (float)dcnt * 65536.0f) : dfp;
                ctl[4] = done ? 1 : 0;
                ctl[5] = exit_b | (status << 61);
            }
        }
        __syncthreads();
        const unsigned long long t2 = FE_NOW();
        t_ch += t2 - t1;
        y = ctl[0];
        k = ctl[1];
        const int msteps = min((int)ctl[2], kStepsR);
        const uint64_t dfp_next = ctl[3];
        done = ctl[4] != 0;
        if (done) {
            exit_b = ctl[5] & ~(3ull << 61);
            status = (ctl[5] >> 61) & 3u;
        }
        // replay the jumped-over steps (one thread per group)
        if (tid < kGroups && jumped[tid]) {
            uint32_t o = walk[tid * kJ];
            const int len = tid * kJ + kJ < kStepsR ? kJ : kJ - 1;
            for (int i = 1; i < len; ++i) {
                o = trans[(tid * kJ + i - 1) * kWin + (int)o];
                walk[tid * kJ + i] = (uint16_t)o;
            }
        }
        __syncthreads();
        for (int j = tid; j < msteps; j += kFeChainThreads) {
            const uint16_t o = walk[j];
            if (o != kDirect) bnd[k0 + j] = wstart_of((uint64_t)j) + o;
        }
        __syncthreads();  // trans/walk are rewritten by the next round
        dfp = dfp_next;
        t_bnd += FE_NOW() - t2;
        // speculation (bz2mi_unit_speculate): spec[0, spec_nb) are the block
        // starts of the chain from the unit's first byte.  A block's end
        // depends only on the bytes from its start on, so once a block of this
        // chain starts where a speculative block starts, the chains agree from
        // there: stop, the host splices the speculative tail.  One check per
        // round, on its last block end, with a cursor that only moves forward
        // (both start lists ascend).
        if (spec_nb > 1 && !done && k > k0) {
            if (tid < 64) {
                const uint64_t b = bnd[k - 1];
                const uint64_t P = (b >> 63) ? (b & ~kExpl) : ginv(f, b);
                uint64_t j = scur;
                bool hit = false;
                for (;;) {
                    const uint64_t i = j + (uint64_t)lane_id();
                    const uint64_t v = i < spec_nb ? spec[i] : ~0ull;
                    const uint64_t m = __ballot(v >= P);
                    if (m) {
                        const int L = __ffsll((long long)m) - 1;
                        j += (uint64_t)L;
                        hit = uniform64(__shfl(v, L)) == P;
                        break;
                    }
                    j += 64;
                }
                if (tid == 0) {
                    ctl[0] = j;
                    ctl[1] = hit ? 1 : 0;
                }
            }
            __syncthreads();
            scur = ctl[0];
            if (ctl[1]) {
                merged = scur;
                done = true;
            }
            __syncthreads();
        }
    }
#ifdef BZ2MI_PHASES
    if (threadIdx.x == 0) {
        g_fe_phase[6] = t_tab;
        g_fe_phase[7] = t_ch;
        g_fe_phase[8] = t_bnd;
        g_fe_phase[9] = t_slow;
        g_fe_phase[10] = n_out;
        g_fe_phase[11] = n_mid;
        g_fe_phase[12] = (unsigned long long)nwin;
        g_fe_phase[13] = k;
        g_fe_phase[14] = (unsigned long long)nslow;
        g_fe_phase[15] = wall_clock64();
    }
#else
    (void)nslow;
    (void)t_tab, (void)t_ch, (void)t_bnd, (void)t_slow, (void)n_out, (void)n_mid;
#endif
    if (threadIdx.x == 0) {
        if (merged) {  // blocks [0, k) chained, then the speculative blocks from spec[merged]
            nb_out[0] = k;
            nb_out[3] = merged;
        } else {
            bnd[k] = exit_b;
            nb_out[0] = k + 1;
            nb_out[3] = 0;
        }
        nb_out[1] = status;
    }
}

// ---- K7: block ends -> positions: starts[0] = entry, starts[j+1] = the end
// of block j (bnd[j]); nb_io[2] = the exit token of the next unit
// (starts[nb] - n_own, bit 63: mid-run), when the unit does not end the stream
__global__ __launch_bounds__(256) void fe_resolve_kernel(const uint8_t* __restrict__ x, const uint32_t* __restrict__ laneinfo,
                                                         const uint64_t* __restrict__ fc, const uint4* __restrict__ summ,
                                                         uint64_t n, uint64_t nc, uint64_t n_own, uint64_t entry,
                                                         const uint64_t* __restrict__ bnd, uint64_t* __restrict__ nb_io,
                                                         uint64_t* __restrict__ starts) {
    FeView f{x, laneinfo, fc, summ, n, nc, uniform64(fc[nc])};
    const uint64_t nb = nb_io[0];
    const uint64_t k = (uint64_t)blockIdx.x * 4 + wave_id();
    if (k == 0 && lane_id() == 0) starts[0] = entry & ~(1ull << 63);
    if (k >= nb) return;
    const uint64_t b = bnd[k];
    uint64_t pos;
    if (b >> 63) pos = b & ~(1ull << 63);
    else pos = ginv(f, b);
    if (lane_id() == 0) {
        starts[k + 1] = pos;
        if (k + 1 == nb) {
            const bool mid = pos > 0 && pos < n && x[pos] == x[pos - 1];
            nb_io[2] = (pos >= n_own ? pos - n_own : 0) | (mid ? 1ull << 63 : 0);
        }
    }
}


// ---- K8: RLE1 emission and block CRC, one workgroup per block, tiles of
// 4096 input bytes: the tile (and the bytes before it the CRC needs) is staged
// in LDS with 16-byte loads, each thread emits its 16 bytes into an LDS copy
// of the tile's output, which is then written out contiguously.  A count byte
// that belongs to a piece begun in an earlier tile is written straight to the
// block.
// Block CRC (CRC32.hpp:75-86 over the input bytes [p0, p1)): the block is
// viewed front-padded with zero bytes to whole 4096-byte tiles (leading zeros
// leave a raw CRC register at 0), so thread t always owns bytes [16t, 16t+16)
// of every padded tile: it folds their raw CRC into its accumulator
// acc = A_4096(acc) ^ crc16 (Horner over the tiles); the block's raw CRC is the
// ordered combination of the 256 accumulators (a tree with the maps
// A_{16*2^l}), and crc = ~(A_len(0xffffffff) ^ raw).
constexpr int kTile = 4096;
constexpr int kTileOut = kTile + kTile / 4 + 16;

__device__ __forceinline__ uint32_t crc_map(const uint32_t* __restrict__ T, uint32_t x) {
    return T[x & 255u] ^ T[256 + ((x >> 8) & 255u)] ^ T[512 + ((x >> 16) & 255u)] ^ T[768 + (x >> 24)];
}

// Long raw blocks (run-heavy input: a block can cover 4.6 MB) are cut into
// segments of about kFeSegLen bytes, each emitted by a workgroup of its own.
// A cut is clean -- a run start, or a 255-byte piece boundary inside a run
// (the block-local run phase there is 0) -- so every segment is an RLE1
// encoding of its own: the emission restarts the piece phase at the cut
// exactly as the sequential encoder does there.  Segment output offsets are
// the emission counts of the earlier segments (a counting pass), and segment
// CRCs combine as crc(A|B) = A_{|B|}(crc(A)) ^ crc(B) on raw registers.
struct FeSeg {
    uint64_t lo, hi;  // input bytes [lo, hi)
    uint32_t lb, s;   // batch-local block, segment index within the block
};
static_assert(sizeof(FeSeg) == kFeSegBytes, "segment table entry");

// Emission (mode 1) or only its byte count (mode 0) of input bytes [lo, hi)
// that start a piece, into out[o0, ...): returns the count.  CRC (mode 1):
// the raw register (from 0) of [lo, hi) in *raw.
template <int MODE>
__device__ uint32_t rle1_range(const uint8_t* __restrict__ x, uint64_t n, uint64_t lo_, uint64_t hi_,
                               uint8_t* __restrict__ out, uint32_t o0, uint32_t* raw,
                               const uint32_t* __restrict__ tslice, const uint32_t* __restrict__ t4096,
                               const uint32_t* __restrict__ crc_tabs, uint4* tin4, uint8_t* tout, uint32_t* tmp,
                               uint32_t* lastv) {
    const int t = threadIdx.x;
    const uint64_t p0 = lo_, p1 = hi_;
    const uint64_t pad = (kTile - (p1 - p0) % kTile) % kTile;
    uint32_t acc = 0;
    const uint8_t* tin = reinterpret_cast<const uint8_t*>(tin4);
    uint32_t o_carry = o0;
    uint64_t rs_carry = p0;  // run start in effect before the tile
    for (uint64_t base = p0; base < p1; base += kTile) {
        // stage [abase, abase + 16*nvec) covering base-1 .. base+kTile and the
        // CRC bytes from base - pad on
        const uint64_t lo = base == p0 ? p0 : base - pad;
        const uint64_t lo1 = base < lo + 1 ? base : lo + 1;
        const uint64_t abase = lo1 ? ((lo1 - 1) & ~15ull) : 0;
        const uint64_t aend = min(n, base + kTile + 1);
        const int nvec = (int)((aend - abase + 15) >> 4);
        for (int v = t; v < nvec; v += 256) {
            const uint64_t ad = abase + 16ull * (uint64_t)v;
            if (ad + 16 <= n) {
                tin4[v] = *reinterpret_cast<const uint4*>(x + ad);
            } else {
                uint32_t w[4] = {0, 0, 0, 0};
                for (int q = 0; q < 16; ++q)
                    if (ad + q < n) w[q >> 2] |= (uint32_t)x[ad + q] << ((q & 3) * 8);
                tin4[v] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
        __syncthreads();
        const uint32_t off0 = (uint32_t)(base - abase);
        if (MODE == 1) {  // CRC of padded-tile bytes [16t, 16t+16): real positions base - pad + 16t + k
            const int64_t r0 = (int64_t)base - (int64_t)pad + 16 * t;
            uint32_t r = 0;
#pragma unroll
            for (int w4 = 0; w4 < 4; ++w4) {
                uint32_t wd = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int64_t rp = r0 + 4 * w4 + k;
                    const uint32_t by = rp >= (int64_t)p0 ? (uint32_t)tin[(uint64_t)rp - abase] : 0u;
                    wd = (wd << 8) | by;
                }
                const uint32_t xw = r ^ wd;
                r = tslice[768 + (xw >> 24)] ^ tslice[512 + ((xw >> 16) & 255u)] ^ tslice[256 + ((xw >> 8) & 255u)] ^
                    tslice[xw & 255u];
            }
            acc = (base == p0) ? r : crc_map(t4096, acc) ^ r;
        }
        const uint64_t a = base + (uint64_t)t * 16;
        uint8_t v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = (a + q < p1) ? tin[off0 + t * 16 + q] : 0;
        const uint32_t prev = a > 0 ? tin[off0 + t * 16 - 1] : 0;
        const uint32_t nextb = (a + 16 < p1) ? tin[off0 + t * 16 + 16] : 0;
        // last run start (local: i == p0 or x[i] != x[i-1]) inside this thread's bytes
        uint32_t lrs = 0;  // as offset+1 from p0 (0 = none)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint64_t i = a + q;
            if (i < p1) {
                const uint32_t pv = q ? v[q - 1] : prev;
                if (i == p0 || v[q] != pv) lrs = (uint32_t)(i - p0) + 1;
            }
        }
        uint32_t tot;
        const uint32_t mx = wg_incl_max<256>(lrs, tmp, &tot);
        lastv[t] = mx;
        __syncthreads();
        const uint32_t ex = t ? lastv[t - 1] : 0u;  // exclusive max over earlier threads
        // u = (i - run start) % 255 of byte i, kept incrementally from the
        // thread's first byte (one 64-bit modulo per thread and tile)
        const uint64_t cur = ex ? p0 + ex - 1 : rs_carry;
        const uint32_t u0 = a < p1 ? (uint32_t)((a - cur) % 255u) : 0u;
        // emission counts
        uint32_t e = 0;
        bool ones = true;  // every byte of the thread's emits itself (u < 3)
        uint32_t u = u0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint64_t i = a + q;
            if (i < p1) {
                const uint32_t pv = q ? v[q - 1] : prev;
                if (i == p0 || v[q] != pv) u = 0;
                e += u < 3 ? 1u : (u == 3 ? 2u : 0u);
                ones = ones && u < 3;
            }
            u = u == 254u ? 0u : u + 1u;
        }
        uint32_t etot;
        const uint32_t eoff = wg_excl_sum<256>(e, tmp, &etot);
        // A tile without a run of 4 (random-like data: nearly every tile) is
        // its own encoding: each thread stores its 16 bytes at o_carry + 16 t
        // straight from registers -- dword stores when the output offset is
        // 4-aligned (it is while every earlier tile was verbatim) -- with no
        // LDS output copy and no byte-wise copy-out.
        if (MODE == 1 && __syncthreads_and(ones)) {
            const uint32_t o = o_carry + 16u * (uint32_t)t;
            const uint32_t cnt = a < p1 ? (uint32_t)min<uint64_t>(16, p1 - a) : 0u;
            if (cnt == 16 && (o & 3u) == 0) {
                uint32_t w[4];
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    w[k] = v[4 * k] | ((uint32_t)v[4 * k + 1] << 8) | ((uint32_t)v[4 * k + 2] << 16) |
                           ((uint32_t)v[4 * k + 3] << 24);
                if ((o & 15u) == 0) {
                    *reinterpret_cast<uint4*>(out + o) = make_uint4(w[0], w[1], w[2], w[3]);
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k) *reinterpret_cast<uint32_t*>(out + o + 4 * k) = w[k];
                }
            } else {
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    if ((uint32_t)q < cnt) out[o + q] = v[q];
            }
            o_carry += etot;
            if (tot) rs_carry = p0 + tot - 1;
            __syncthreads();
            continue;
        }
        if (MODE == 1) {
            // emit into the LDS copy (o: block-relative output position)
            uint32_t o = o_carry + eoff;
            uint32_t un = u0;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint64_t i = a + q;
                uint32_t u = un;
                un = u == 254u ? 0u : u + 1u;
                if (i < p1) {
                    const uint32_t pv = q ? v[q - 1] : prev;
                    if (i == p0 || v[q] != pv) {
                        u = 0;
                        un = 1;
                    }
                    const uint32_t nx = q < 15 ? v[q + 1] : nextb;
                    const bool last = (i + 1 == p1) || nx != v[q] || u == 254;
                    if (u < 3) {
                        tout[o - o_carry] = v[q];
                        o++;
                    } else if (u == 3) {
                        tout[o - o_carry] = v[q];
                        if (last) tout[o + 1 - o_carry] = 0;  // else the piece's last byte fills the slot
                        o += 2;
                    } else if (last) {
                        if (o - 1 >= o_carry) tout[o - 1 - o_carry] = (uint8_t)(u - 3);
                        else out[o - 1] = (uint8_t)(u - 3);  // piece begun in an earlier tile
                    }
                }
            }
            __syncthreads();
            for (uint32_t j = t; j < etot; j += 256) out[o_carry + j] = tout[j];
        }
        o_carry += etot;
        if (tot) rs_carry = p0 + tot - 1;
        __syncthreads();
    }
    if (MODE == 1) {
        // ordered combination of the accumulators: level l joins neighbours of
        // 16 * 2^l padded bytes each (in-wave levels by shuffles, then LDS)
        uint32_t v = acc;
#pragma unroll
        for (int l = 0; l < 6; ++l) {
            const uint32_t right = (uint32_t)__shfl_down((int)v, 1 << l);
            if ((t & ((2 << l) - 1)) == 0) v = crc_map(crc_tabs + kCrcShiftBase + 1024 * (l + 4), v) ^ right;
        }
        if ((t & 63) == 0) lastv[t >> 6] = v;
        __syncthreads();
        if (t == 0) {
            const uint32_t* A1024 = crc_tabs + kCrcShiftBase + 1024 * 10;
            const uint32_t* A2048 = crc_tabs + kCrcShiftBase + 1024 * 11;
            const uint32_t left = crc_map(A1024, lastv[0]) ^ lastv[1];
            const uint32_t right = crc_map(A1024, lastv[2]) ^ lastv[3];
            *raw = crc_map(A2048, left) ^ right;
        }
    }
    return o_carry - o0;
}

// the raw register x processed over `len` zero bytes (A_len, binary powers)
__device__ __forceinline__ uint32_t crc_shift(const uint32_t* __restrict__ crc_tabs, uint32_t x, uint64_t len) {
    for (int k = 0; k < 32 && (len >> k); ++k)
        if ((len >> k) & 1u) x = crc_map(crc_tabs + kCrcShiftBase + 1024 * k, x);
    return x;
}

// Segments of the batch's blocks (one workgroup): a block of at least
// 2 kFeSegLen raw bytes is cut near every kFeSegLen bytes at a clean cut (see
// FeSeg); segs[] in block order, segfirst[lb] its first segment,
// segfirst[count] = *nseg the total.  rsb[c]: start of the run holding the
// byte before chunk c (fe_runscan_kernel).
__global__ __launch_bounds__(1024) void fe_segplan_kernel(const uint8_t* __restrict__ x, uint64_t n,
                                                          const uint64_t* __restrict__ starts, uint64_t first,
                                                          uint64_t count, const uint64_t* __restrict__ rsb,
                                                          const uint4* __restrict__ summ, FeSeg* __restrict__ segs,
                                                          uint32_t* __restrict__ segfirst, uint64_t seg_cap,
                                                          uint32_t* __restrict__ nseg) {
    __shared__ uint32_t tmp[16];
    const int t = threadIdx.x;
    // cut j >= 1 of block [p0, p1) is near the chunk boundary q at or after
    // p0 + j kFeSegLen (only while q + 256 < p1); the cut is q itself when a
    // run starts there, else the next piece boundary of the run that goes on
    // through q -- or the run's end, if that comes first (the chunk
    // summary's first run start): O(1) from the summaries, no byte scans
    auto cut_at = [&](uint64_t p0, uint64_t j) -> uint64_t {
        const uint64_t want = p0 + j * kFeSegLen;
        return (want + kFeChunk - 1) / kFeChunk * kFeChunk;
    };
    auto clean = [&](uint64_t p0, uint64_t q) -> uint64_t {
        const uint64_t c = q / kFeChunk;
        if (chunk_starts_run(summ, c)) return q;
        const uint64_t r = max(p0, rsb[c]);
        const uint32_t ph = (uint32_t)((q - r) % 255u);
        const uint64_t pb = q + (ph ? 255u - ph : 0u);
        const uint32_t lead = summ[c].y;  // the chunk's first run start (its length if none)
        return q + lead < pb ? q + lead : pb;
    };
    uint32_t carry = 0;
    for (uint64_t b0 = 0; b0 < count; b0 += 1024) {
        const uint64_t lb = b0 + (uint64_t)t;
        uint32_t k = 0;
        uint64_t p0 = 0, p1 = 0;
        if (lb < count) {
            p0 = starts[first + lb];
            p1 = starts[first + lb + 1];
            k = 1;
            if (p1 - p0 >= 2ull * kFeSegLen)
                while (cut_at(p0, k) + 256 < p1) ++k;
        }
        uint32_t tot;
        const uint32_t off = carry + wg_excl_sum<1024>(k, tmp, &tot);
        if (lb < count) {
            segfirst[lb] = off;
            uint64_t lo = p0;
            for (uint32_t j = 1; j <= k; ++j) {
                const uint64_t hi = j < k ? clean(p0, cut_at(p0, j)) : p1;
                if (off + j - 1 < seg_cap) segs[off + j - 1] = FeSeg{lo, hi, (uint32_t)lb, j - 1};
                lo = hi;
            }
        }
        carry += tot;
        __syncthreads();
    }
    if (t == 0) {
        segfirst[count] = carry;
        *nseg = carry <= seg_cap ? carry : (uint32_t)seg_cap;
        // a table overflow (the capacity bounds every batch by arithmetic)
        // leaves blocks unemitted: a sticky flag the host checks
        if (carry > seg_cap) nseg[1] = 1u;
    }
    (void)x;
    (void)n;
}

// mode 0: emission counts of the segments that have a successor; mode 1:
// emission into the block (at the earlier segments' counts), lens, and the CRC
// (whole blocks) or the segment's raw CRC (cut blocks).  One workgroup per
// segment; workgroups past *nseg return.
__global__ __launch_bounds__(256) void fe_rle1_kernel(const uint8_t* __restrict__ x, uint64_t n,
                                                      const FeSeg* __restrict__ segs,
                                                      const uint32_t* __restrict__ segfirst,
                                                      const uint32_t* __restrict__ nseg, uint32_t* __restrict__ segcnt,
                                                      uint32_t* __restrict__ segcrc, int mode,
                                                      uint8_t* __restrict__ blocks, size_t stride,
                                                      uint32_t* __restrict__ lens, uint32_t* __restrict__ crcs,
                                                      const uint32_t* __restrict__ crc_tabs) {
    __shared__ uint4 tin4[2 * kTile / 16 + 4];
    __shared__ uint8_t tout[kTileOut];
    __shared__ uint32_t tmp[8];
    __shared__ uint32_t lastv[256];
    __shared__ uint32_t tslice[1024], t4096[1024];
    __shared__ uint32_t rawv;
    const int t = threadIdx.x;
    const uint32_t ns = uniform(*nseg);
    if (mode == 0) {
        // counts of the segments that have a successor in their block (none
        // without cut blocks): a small grid striding over the table, so the
        // pass costs nothing when there is nothing to count (one workgroup per
        // segment here measured 0.95 ms behind a concurrent MTF kernel)
        for (uint32_t w = blockIdx.x; w < ns; w += gridDim.x) {
            const FeSeg sg = segs[w];
            const uint32_t lb = uniform(sg.lb), si = uniform(sg.s);
            if (si + 1 >= uniform(segfirst[lb + 1]) - uniform(segfirst[lb])) continue;  // last segment: not needed
            const uint32_t e = rle1_range<0>(x, n, uniform64(sg.lo), uniform64(sg.hi), nullptr, 0, nullptr, nullptr,
                                             nullptr, crc_tabs, tin4, tout, tmp, lastv);
            if (t == 0) segcnt[w] = e;
            __syncthreads();  // (LDS tiles reused by the next segment)
        }
        return;
    }
    if (blockIdx.x >= ns) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        tslice[t + 256 * q] = crc_tabs[t + 256 * q];
        t4096[t + 256 * q] = crc_tabs[kCrcShiftBase + 1024 * 12 + t + 256 * q];
    }
    // segment w, w + grid, ...: the grid is one workgroup per block plus a
    // bounded number for the cut blocks' extra segments, so nearly every
    // workgroup takes one segment and none is launched only to return
    for (uint32_t w = blockIdx.x; w < ns; w += gridDim.x) {
        const FeSeg sg = segs[w];
        const uint32_t lb = uniform(sg.lb), si = uniform(sg.s);
        const uint32_t f0 = uniform(segfirst[lb]), k = uniform(segfirst[lb + 1]) - f0;
        const uint64_t lo = uniform64(sg.lo), hi = uniform64(sg.hi);
        uint32_t o0 = 0;
        for (uint32_t j = 0; j < si; ++j) o0 += segcnt[f0 + j];
        o0 = uniform(o0);
        __syncthreads();  // (the CRC tables; the previous segment's LDS tiles)
        const uint32_t e = rle1_range<1>(x, n, lo, hi, blocks + (size_t)lb * stride, o0, &rawv, tslice, t4096,
                                         crc_tabs, tin4, tout, tmp, lastv);
        if (t == 0) {
            if (si + 1 == k) lens[lb] = o0 + e;
            if (k == 1) {
                // the initial register 0xffffffff processed over the block's length
                crcs[lb] = ~(crc_shift(crc_tabs, 0xffffffffu, hi - lo) ^ rawv);
            } else {
                segcrc[w] = rawv;
            }
        }
        __syncthreads();
    }
}

// CRCs of the cut blocks from their segments' raw registers (a thread per block)
__global__ __launch_bounds__(256) void fe_crccomb_kernel(const FeSeg* __restrict__ segs,
                                                         const uint32_t* __restrict__ segfirst, uint64_t count,
                                                         const uint32_t* __restrict__ segcrc,
                                                         uint32_t* __restrict__ crcs,
                                                         const uint32_t* __restrict__ crc_tabs) {
    const uint64_t lb = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lb >= count) return;
    const uint32_t f0 = segfirst[lb], k = segfirst[lb + 1] - f0;
    if (k < 2) return;
    uint32_t raw = 0;
    for (uint32_t j = 0; j < k; ++j) {
        const FeSeg sg = segs[f0 + j];
        raw = crc_shift(crc_tabs, raw, sg.hi - sg.lo) ^ segcrc[f0 + j];
    }
    const uint64_t p0 = segs[f0].lo, p1 = segs[f0 + k - 1].hi;
    crcs[lb] = ~(crc_shift(crc_tabs, 0xffffffffu, p1 - p0) ^ raw);
}

}  // namespace bz2mi
