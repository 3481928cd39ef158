// Per-block cyclic BWT on the device: one 256-thread workgroup per block.
//
// Replaces DivSufSortBWT (reference kernel.cpp:2429-2456, with the wrap byte
// of close_block kernel.cpp:3113).  The rotation order of an aperiodic block
// is unique, so any correct rotation sort reproduces the reference; equal
// rotations of a periodic block end in index order (SURVEY H2/H8 decision):
// every sort below breaks ties by the rotation index.
//
// Phase 1 (characters, MSD): counting sort of the rotations by their first
// byte, then every bucket is either
//   * small (<= 512): sorted by ONE wave with a register bitonic network on
//     (next 8 bytes, index) -- for random data this resolves everything, and
//     equal 8-byte keys form groups for phase 2;
//   * large: partitioned by the next byte by the whole workgroup (one level
//     deeper), up to kMaxDepth bytes.
// Every element gets a group label = the SA index of its group's first
// element (Larsson-Sadakane style; labels are order-consistent refinements).
// Phase 2 (prefix doubling on the unresolved groups only): with h <= every
// group's common prefix, sort each group by (label[i+h], index) -- snapshot
// keys first, then per-group sorts (waves for small groups, a workgroup LSD
// radix on (key, index) for large ones), relabel, h *= 2, until no group is
// left or h >= n (periodic blocks).
//
// HBM layout per workgroup slot (bwt_slot_bytes): SA, labels, 64-bit keys,
// radix ping-pong buffers and the segment lists; blocks are pulled from a
// device work counter so the grid is sized to the chip.
#include "common.hpp"
#include "kernels.hpp"

namespace bz2mi {

BZ2MI_PHASE_TABLE(g_bwt_phase)

int bwt_phases(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwt_phase), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

namespace {

constexpr int NT = 256;
constexpr int NW = NT / 64;
constexpr int kSmall = 512;    // largest segment one wave sorts
constexpr int kMaxDepth = 48;  // character partition depth limit before doubling
constexpr int kIdxBits = 20;   // S <= 2^20

struct BwtShared {
    uint32_t hist[256];
    uint32_t base[256];
    uint32_t wcnt[NW][256];
    uint32_t tmp[NW * 2];
    uint64_t tmp64[NW];
    uint64_t tmp64b[NW];
    uint32_t cnt[8];     // list counters
    uint32_t bcast[4];
};

struct Seg {
    uint32_t start, len;
};

struct Scratch {
    uint32_t* sa;
    uint32_t* rank;
    uint64_t* ka;
    uint64_t* kb;
    uint32_t* va;
    uint32_t* vb;
    Seg* small;   // phase-1 small buckets
    Seg* large;   // phase-1 large buckets (current level)
    Seg* large2;  // phase-1 large buckets (next level)
    Seg* grp;     // phase-2 groups (current round)
    Seg* grp2;    // phase-2 groups (next round)
};

__device__ Scratch carve(uint8_t* base, int S) {
    Scratch s;
    uint8_t* p = base;
    const size_t n = (size_t)S;
    s.ka = (uint64_t*)p; p += 8 * n;
    s.kb = (uint64_t*)p; p += 8 * n;
    s.sa = (uint32_t*)p; p += 4 * n;
    s.rank = (uint32_t*)p; p += 4 * n;
    s.va = (uint32_t*)p; p += 4 * n;
    s.vb = (uint32_t*)p; p += 4 * n;
    s.small = (Seg*)p; p += 8 * (n / 2 + 2);
    s.grp = (Seg*)p; p += 8 * (n / 2 + 2);
    s.grp2 = (Seg*)p; p += 8 * (n / 2 + 2);
    s.large = (Seg*)p; p += 8 * (n / kSmall + 8);
    s.large2 = (Seg*)p; p += 8 * (n / kSmall + 8);
    return s;
}

// 8 bytes of the rotation starting at `pos` (< n), most significant first.
__device__ __forceinline__ uint64_t load8(const uint8_t* __restrict__ T, int n, uint32_t pos) {
    if (pos + 8 <= (uint32_t)n) {
        const uint32_t a = pos & ~3u;
        const uint32_t* T32 = (const uint32_t*)T;
        const uint32_t w0 = T32[a >> 2], w1 = T32[(a >> 2) + 1], w2 = T32[(a >> 2) + 2];
        const uint32_t sh = (pos & 3u) * 8u;
        // little-endian words: bytes pos.. are w0 >> sh, then w1, w2
        const uint32_t lo32 = sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
        const uint32_t hi32 = sh ? (w1 >> sh) | (w2 << (32 - sh)) : w1;
        return ((uint64_t)__builtin_bswap32(lo32) << 32) | __builtin_bswap32(hi32);
    }
    uint64_t k = 0;
    uint32_t j = pos;
    for (int q = 0; q < 8; ++q) {
        k = (k << 8) | T[j];
        j = (j + 1 == (uint32_t)n) ? 0 : j + 1;
    }
    return k;
}

__device__ __forceinline__ uint8_t byte_at(const uint8_t* __restrict__ T, int n, uint32_t pos) {
    return T[pos >= (uint32_t)n ? pos % (uint32_t)n : pos];
}

// ---- wave-level register bitonic sort of 64*E (key, index) pairs, striped
// (element e of lane l is item e*64 + l); ascending by (hi, lo).
template <int E>
__device__ __forceinline__ void wave_bitonic(uint64_t (&hi)[E], uint32_t (&lo)[E]) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= 64 * E; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j >= 1; j >>= 1) {
            if (j >= 64) {
                const int je = j / 64;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int pe = e ^ je;
                    if (pe > e) {
                        const bool asc = (((e * 64) & k) == 0);  // k >= 128 here: lane bits do not matter
                        const bool gt = hi[e] > hi[pe] || (hi[e] == hi[pe] && lo[e] > lo[pe]);
                        if (gt == asc) {
                            const uint64_t th = hi[e];
                            hi[e] = hi[pe];
                            hi[pe] = th;
                            const uint32_t tl = lo[e];
                            lo[e] = lo[pe];
                            lo[pe] = tl;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const uint64_t oh = __shfl_xor(hi[e], j);
                    const uint32_t ol = __shfl_xor(lo[e], j);
                    const int g = e * 64 + lane;
                    const bool asc = (g & k) == 0;
                    const bool lower = (lane & j) == 0;
                    const bool mine_gt = hi[e] > oh || (hi[e] == oh && lo[e] > ol);
                    // lower slot keeps the min when ascending, the max when descending
                    const bool take = (lower == asc) ? mine_gt : !mine_gt;
                    if (take) {
                        hi[e] = oh;
                        lo[e] = ol;
                    }
                }
            }
        }
    }
}

// Sort one small segment with one wave, relabel its members and emit its
// groups of size > 1 to `out` (slot from *counter).
// mode 0: keys are the 8 bytes at depth d (phase 1); mode 1: keys from ka[] (phase 2).
template <int E>
__device__ void wave_sort_segment(const uint8_t* __restrict__ T, int n, Scratch& s, Seg seg, uint32_t d, int mode,
                                  Seg* out, uint32_t* counter) {
    const int lane = lane_id();
    uint64_t hi[E];
    uint32_t lo[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(e * 64 + lane);
        if (g < seg.len) {
            const uint32_t i = s.sa[seg.start + g];
            lo[e] = i;
            if (mode == 0) {
                uint32_t p = i + d;
                if (p >= (uint32_t)n) p %= (uint32_t)n;
                hi[e] = load8(T, n, p);
            } else {
                hi[e] = s.ka[seg.start + g];
            }
        } else {
            hi[e] = ~0ull;
            lo[e] = ~0u;
        }
    }
    wave_bitonic<E>(hi, lo);
    // group boundaries (by key only) and group-start labels
    bool flag[E];
    uint32_t gs[E];
    uint32_t carry = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(e * 64 + lane);
        uint64_t ph = __shfl_up(hi[e], 1);
        if (e > 0) {
            const uint64_t last_prev = __shfl(hi[e > 0 ? e - 1 : 0], 63);
            if (lane == 0) ph = last_prev;
        }
        flag[e] = (g == 0) || (hi[e] != ph);
        uint32_t v = flag[e] ? g : 0u;
        v = wave_incl_max(v);
        v = v > carry ? v : carry;
        gs[e] = v;
        carry = __shfl(v, 63);
        if (g < seg.len) s.sa[seg.start + g] = lo[e];
    }
    // end of each group = the next flag position (suffix min), or len
    uint32_t ncarry = seg.len;
#pragma unroll
    for (int e = E - 1; e >= 0; --e) {
        const uint32_t g = (uint32_t)(e * 64 + lane);
        uint32_t v = (flag[e] && g < seg.len) ? g : seg.len;
        for (int dd = 1; dd < 64; dd <<= 1) {  // inclusive suffix min
            const uint32_t y = __shfl_down(v, dd);
            if (lane + dd < 64) v = v < y ? v : y;
        }
        uint32_t after = __shfl_down(v, 1);
        if (lane == 63) after = ncarry;
        after = after < ncarry ? after : ncarry;
        const uint32_t first_here = __shfl(v, 0);
        if (g < seg.len) {
            s.rank[lo[e]] = seg.start + gs[e];
            if (flag[e]) {
                const uint32_t glen = after - g;
                if (glen > 1) {
                    const uint32_t slot = atomicAdd(counter, 1u);
                    out[slot] = Seg{seg.start + g, glen};
                }
            }
        }
        ncarry = first_here < ncarry ? first_here : ncarry;
    }
}

// dispatch a small segment to the right register width
__device__ void wave_sort_any(const uint8_t* T, int n, Scratch& s, Seg seg, uint32_t d, int mode, Seg* out,
                              uint32_t* counter) {
    seg.start = uniform(seg.start);
    seg.len = uniform(seg.len);
    if (seg.len <= 64) wave_sort_segment<1>(T, n, s, seg, d, mode, out, counter);
    else if (seg.len <= 128) wave_sort_segment<2>(T, n, s, seg, d, mode, out, counter);
    else if (seg.len <= 256) wave_sort_segment<4>(T, n, s, seg, d, mode, out, counter);
    else wave_sort_segment<8>(T, n, s, seg, d, mode, out, counter);
}

// ---- workgroup LSD radix (large phase-2 groups)
__device__ void key_span(const uint64_t* k, int m, BwtShared& sh, uint64_t* vary) {
    uint64_t o = 0, a = ~0ull;
    for (int i = threadIdx.x; i < m; i += NT) {
        const uint64_t x = k[i];
        o |= x;
        a &= x;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        o |= __shfl_xor(o, d);
        a &= __shfl_xor(a, d);
    }
    if (lane_id() == 0) {
        sh.tmp64[wave_id()] = o;
        sh.tmp64b[wave_id()] = a;
    }
    __syncthreads();
    uint64_t oall = 0, aall = ~0ull;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        oall |= sh.tmp64[w];
        aall &= sh.tmp64b[w];
    }
    __syncthreads();
    *vary = uniform64(oall ^ aall);
}

__device__ void radix_pass(const uint64_t* kin, const uint32_t* vin, uint64_t* kout, uint32_t* vout, int m, int shift,
                           BwtShared& sh) {
    const int t = threadIdx.x;
    sh.hist[t] = 0;
    for (int w = 0; w < NW; ++w) sh.wcnt[w][t] = 0;
    __syncthreads();
    for (int i = t; i < m; i += NT) atomicAdd(&sh.hist[(kin[i] >> shift) & 255u], 1u);
    __syncthreads();
    uint32_t total;
    const uint32_t ex = wg_excl_sum<NT>(sh.hist[t], sh.tmp, &total);
    sh.base[t] = ex;
    __syncthreads();
    const int w = wave_id();
    for (int tile = 0; tile < m; tile += NT) {
        const int i = tile + t;
        const bool valid = i < m;
        uint64_t key = 0;
        uint32_t val = 0, d = 0;
        if (valid) {
            key = kin[i];
            val = vin[i];
            d = (uint32_t)(key >> shift) & 255u;
        }
        const uint64_t peers = wave_match8(d, valid);
        const uint64_t lt = peers & __lanemask_lt();
        const uint32_t lrank = (uint32_t)__popcll(lt);
        if (valid && lt == 0) sh.wcnt[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        uint32_t pos = 0;
        if (valid) {
            pos = sh.base[d] + lrank;
            for (int q = 0; q < w; ++q) pos += sh.wcnt[q][d];
        }
        __syncthreads();
        {
            uint32_t add = 0;
            for (int q = 0; q < NW; ++q) {
                add += sh.wcnt[q][t];
                sh.wcnt[q][t] = 0;
            }
            sh.base[t] += add;
        }
        if (valid) {
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
    }
}

// Sort a large phase-2 group [start, start+len) by (snapshot key, index) with
// the whole workgroup, then relabel and emit subgroups.
__device__ void wg_sort_group(Scratch& s, Seg seg, BwtShared& sh, Seg* out, uint32_t* counter) {
    seg.start = uniform(seg.start);
    seg.len = uniform(seg.len);
    const int t = threadIdx.x;
    const int m = (int)seg.len;
    uint64_t* k0 = s.ka + seg.start;  // keys were snapshotted here (pass A)
    uint64_t* k1 = s.kb + seg.start;
    uint32_t* v0 = s.va + seg.start;
    uint32_t* v1 = s.vb + seg.start;
    for (int k = t; k < m; k += NT) {
        const uint32_t i = s.sa[seg.start + k];
        k0[k] = (k0[k] << kIdxBits) | i;  // composite (key, index)
        v0[k] = i;
    }
    __syncthreads();
    uint64_t vary;
    key_span(k0, m, sh, &vary);
    bool flip = false;
    for (int shift = 0; shift < 64; shift += 8) {
        if (((vary >> shift) & 255u) == 0) continue;
        if (!flip) radix_pass(k0, v0, k1, v1, m, shift, sh);
        else radix_pass(k1, v1, k0, v0, m, shift, sh);
        flip = !flip;
    }
    const uint64_t* K = flip ? k1 : k0;
    const uint32_t* V = flip ? v1 : v0;
    // relabel by the key part, emit subgroups
    uint32_t carry = 0;
    for (int tile = 0; tile < m; tile += NT) {
        const int k = tile + t;
        const bool valid = k < m;
        bool start = false, next_start = true;
        uint64_t me = 0;
        if (valid) {
            me = K[k] >> kIdxBits;
            start = (k == 0) || (K[k - 1] >> kIdxBits) != me;
            next_start = (k + 1 == m) || (K[k + 1] >> kIdxBits) != me;
            s.sa[seg.start + k] = V[k];
        }
        uint32_t tot;
        uint32_t gst = wg_incl_max<NT>(start ? (uint32_t)k : 0u, sh.tmp, &tot);
        gst = gst > carry ? gst : carry;
        if (valid) {
            s.rank[V[k]] = seg.start + gst;
            if (start && !next_start) {
                // group length: walk to the next start (groups are contiguous)
                uint32_t e = (uint32_t)k + 1;
                while (e < (uint32_t)m && (K[e] >> kIdxBits) == me) e++;
                const uint32_t slot = atomicAdd(counter, 1u);
                out[slot] = Seg{seg.start + (uint32_t)k, e - (uint32_t)k};
            }
        }
        carry = carry > tot ? carry : tot;
        __syncthreads();
    }
}

// Phase 1 large bucket at depth d: partition by byte d; children go to the
// small list, the next large list, or are finished (size 1 / depth limit).
__device__ void wg_partition(const uint8_t* __restrict__ T, int n, Scratch& s, Seg seg, uint32_t d, BwtShared& sh,
                             Seg* large_next) {
    seg.start = uniform(seg.start);
    seg.len = uniform(seg.len);
    const int t = threadIdx.x;
    sh.hist[t] = 0;
    __syncthreads();
    for (uint32_t k = t; k < seg.len; k += NT) {
        const uint32_t i = s.sa[seg.start + k];
        s.vb[seg.start + k] = i;
        atomicAdd(&sh.hist[byte_at(T, n, i + d)], 1u);
    }
    __syncthreads();
    const uint32_t c = sh.hist[t];
    uint32_t total;
    const uint32_t ex = wg_excl_sum<NT>(c, sh.tmp, &total);
    sh.base[t] = ex;
    __syncthreads();
    // stable placement is not needed: later sorts break ties by index
    for (uint32_t k = t; k < seg.len; k += NT) {
        const uint32_t i = s.vb[seg.start + k];
        const uint32_t slot = atomicAdd(&sh.base[byte_at(T, n, i + d)], 1u);
        s.sa[seg.start + slot] = i;
    }
    __syncthreads();
    // children: bucket t spans [ex, ex + c)
    if (c == 1) {
        s.rank[s.sa[seg.start + ex]] = seg.start + ex;
    } else if (c > 1) {
        const Seg ch{seg.start + ex, c};
        if (c <= (uint32_t)kSmall) {
            s.small[atomicAdd(&sh.cnt[0], 1u)] = ch;
        } else if (d + 1 >= (uint32_t)kMaxDepth) {
            for (uint32_t k = 0; k < c; ++k) s.rank[s.sa[ch.start + k]] = ch.start;
            s.grp[atomicAdd(&sh.cnt[2], 1u)] = ch;
        } else {
            large_next[atomicAdd(&sh.cnt[3], 1u)] = ch;
        }
    }
    __syncthreads();
}

__device__ void bwt_block(const uint8_t* __restrict__ T, int n, uint8_t* __restrict__ out, uint32_t* __restrict__ orig,
                          Scratch& s, BwtShared& sh, bool stamp) {
    const int t = threadIdx.x;
    BZ2MI_PHASE(g_bwt_phase, 0, stamp);
    // ---- phase 1a: counting sort by the first byte
    sh.hist[t] = 0;
    if (t < 8) sh.cnt[t] = 0;
    __syncthreads();
    for (int i = t; i < n; i += NT) atomicAdd(&sh.hist[T[i]], 1u);
    __syncthreads();
    {
        const uint32_t c = sh.hist[t];
        uint32_t total;
        const uint32_t ex = wg_excl_sum<NT>(c, sh.tmp, &total);
        sh.base[t] = ex;
        __syncthreads();
        for (int i = t; i < n; i += NT) s.sa[atomicAdd(&sh.base[T[i]], 1u)] = (uint32_t)i;
        __syncthreads();
        if (c == 1) s.rank[s.sa[ex]] = ex;
        else if (c > 1) {
            if (c <= (uint32_t)kSmall) s.small[atomicAdd(&sh.cnt[0], 1u)] = Seg{ex, c};
            else s.large[atomicAdd(&sh.cnt[1], 1u)] = Seg{ex, c};
        }
        __syncthreads();
    }
    BZ2MI_PHASE(g_bwt_phase, 1, stamp);
    // ---- phase 1b: levels of (small sorts, large partitions)
    uint32_t depth = 1;
    Seg* large = s.large;
    Seg* large_next = s.large2;
    for (;;) {
        // small buckets: one wave each, keys = the 8 bytes at `depth`
        const uint32_t nsmall = uniform(sh.cnt[0]);
        if (t == 0) sh.cnt[4] = 0;
        __syncthreads();
        for (;;) {
            uint32_t idx = 0;
            if (lane_id() == 0) idx = atomicAdd(&sh.cnt[4], 1u);
            idx = uniform(__shfl(idx, 0));
            if (idx >= nsmall) break;
            wave_sort_any(T, n, s, s.small[idx], depth, 0, s.grp, &sh.cnt[2]);
        }
        __syncthreads();
        BZ2MI_PHASE(g_bwt_phase, 2, stamp && depth == 1);
        const uint32_t nlarge = uniform(sh.cnt[1]);
        if (nlarge == 0) break;
        if (t == 0) {
            sh.cnt[0] = 0;
            sh.cnt[3] = 0;
        }
        __syncthreads();
        for (uint32_t q = 0; q < nlarge; ++q) wg_partition(T, n, s, large[q], depth, sh, large_next);
        if (t == 0) sh.cnt[1] = sh.cnt[3];
        __syncthreads();
        Seg* tmpl = large;
        large = large_next;
        large_next = tmpl;
        depth++;
    }
    BZ2MI_PHASE(g_bwt_phase, 3, stamp);
    // ---- phase 2: prefix doubling on the unresolved groups
    Seg* g = s.grp;
    Seg* g2 = s.grp2;
    uint32_t ng = uniform(sh.cnt[2]);
    for (long long h = 9; ng > 0 && h < n; h <<= 1) {
        // pass A: snapshot keys label[i+h] for every member of every group
        if (t == 0) sh.cnt[4] = 0;
        __syncthreads();
        for (;;) {
            uint32_t idx = 0;
            if (lane_id() == 0) idx = atomicAdd(&sh.cnt[4], 1u);
            idx = uniform(__shfl(idx, 0));
            if (idx >= ng) break;
            const Seg sg = g[idx];
            for (uint32_t k = lane_id(); k < sg.len; k += 64) {
                const uint32_t i = s.sa[sg.start + k];
                const uint32_t ih = (uint32_t)((i + h) % n);
                s.ka[sg.start + k] = s.rank[ih];
            }
        }
        __syncthreads();
        // pass B: large groups with the workgroup, small ones with waves
        if (t == 0) {
            sh.cnt[5] = 0;  // next round's groups
            sh.cnt[4] = 0;
        }
        __syncthreads();
        for (uint32_t q = 0; q < ng; ++q) {
            const Seg sg = g[q];
            if (uniform(sg.len) > (uint32_t)kSmall) wg_sort_group(s, sg, sh, g2, &sh.cnt[5]);
        }
        __syncthreads();
        for (;;) {
            uint32_t idx = 0;
            if (lane_id() == 0) idx = atomicAdd(&sh.cnt[4], 1u);
            idx = uniform(__shfl(idx, 0));
            if (idx >= ng) break;
            const Seg sg = g[idx];
            if (sg.len <= (uint32_t)kSmall) wave_sort_any(T, n, s, sg, 0, 1, g2, &sh.cnt[5]);
        }
        __syncthreads();
        ng = uniform(sh.cnt[5]);
        Seg* tg = g;
        g = g2;
        g2 = tg;
        __syncthreads();
    }
    BZ2MI_PHASE(g_bwt_phase, 4, stamp);
    // ---- BWT bytes and origPtr
    for (int k = t; k < n; k += NT) {
        const uint32_t i = s.sa[k];
        out[k] = T[i == 0 ? n - 1 : i - 1];
        if (i == 0) *orig = (uint32_t)k;
    }
    __syncthreads();
    BZ2MI_PHASE(g_bwt_phase, 5, stamp);
}

}  // namespace

__global__ __launch_bounds__(256) void bwt_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                  const uint32_t* __restrict__ lens, int nblocks,
                                                  uint8_t* __restrict__ bwt_out, uint32_t* __restrict__ orig_out,
                                                  uint8_t* scratch, size_t scratch_per_slot, int S,
                                                  uint32_t* work_counter) {
    __shared__ BwtShared sh;
    Scratch s = carve(scratch + (size_t)blockIdx.x * scratch_per_slot, S);
    const int t = threadIdx.x;
    for (;;) {
        if (t == 0) sh.bcast[0] = atomicAdd(work_counter, 1u);
        __syncthreads();
        // wave-uniform (SGPR) block index and length keep every branch below
        // uniform; the barrier closing each iteration keeps the back edge
        // convergent even though lane 0 alone handles tiny blocks
        const int b = __builtin_amdgcn_readfirstlane((int)sh.bcast[0]);
        if (b >= nblocks) break;
        const uint8_t* T = blocks + (size_t)b * stride;
        uint8_t* out = bwt_out + (size_t)b * stride;
        const int n = __builtin_amdgcn_readfirstlane((int)lens[b]);
        if (n > 1) {
            bwt_block(T, n, out, orig_out + b, s, sh, b == nblocks / 2);
        } else if (t == 0) {
            if (n == 1) out[0] = T[0];
            orig_out[b] = 0;
        }
        __syncthreads();
    }
}

}  // namespace bz2mi
