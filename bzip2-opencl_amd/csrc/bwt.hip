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

using Seg = BwtSeg;

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

// ---- wave-level register bitonic sort of 64*E items, blocked (item l*E+e
// sits in element e of lane l): partners closer than E are in the same lane,
// farther ones are lane ^ (j/E) reached with DPP / permlane moves.
// WITH_LO: a 32-bit payload travels with each 64-bit key (not compared).
template <int E, bool WITH_LO, int K, int J>
__device__ __forceinline__ void bitonic_stage(uint64_t (&key)[E], uint32_t (&lo)[E]) {
    const int lane = lane_id();
    if constexpr (J < E) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int pe = e ^ J;
            if (pe > e) {
                const bool asc = ((lane * E + e) & K) == 0;
                if ((key[e] > key[pe]) == asc) {
                    const uint64_t tk = key[e];
                    key[e] = key[pe];
                    key[pe] = tk;
                    if (WITH_LO) {
                        const uint32_t tl = lo[e];
                        lo[e] = lo[pe];
                        lo[pe] = tl;
                    }
                }
            }

        }
    } else {
        constexpr int LJ = J / E;
        const bool lower = (lane & LJ) == 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint64_t ok = ((uint64_t)xor_lanes<LJ>((uint32_t)(key[e] >> 32)) << 32) |
                                xor_lanes<LJ>((uint32_t)key[e]);
            const uint32_t ol = WITH_LO ? xor_lanes<LJ>(lo[e]) : 0u;
            const bool asc = ((lane * E + e) & K) == 0;
            // lower slot keeps the min when ascending, the max when descending;
            // both comparisons strict so that equal keys keep their payloads
            const bool lt = ok < key[e], gt = key[e] < ok;
            const bool take = (lower == asc) ? lt : gt;
            if (take) {
                key[e] = ok;
                if (WITH_LO) lo[e] = ol;
            }

        }
    }
}

template <int E, bool WITH_LO, int K, int J>
__device__ __forceinline__ void bitonic_merge(uint64_t (&key)[E], uint32_t (&lo)[E]) {
    bitonic_stage<E, WITH_LO, K, J>(key, lo);
    if constexpr (J > 1) bitonic_merge<E, WITH_LO, K, J / 2>(key, lo);
}

template <int E, bool WITH_LO, int K>
__device__ __forceinline__ void bitonic_from(uint64_t (&key)[E], uint32_t (&lo)[E]) {
    bitonic_merge<E, WITH_LO, K, K / 2>(key, lo);
    if constexpr (K < 64 * E) bitonic_from<E, WITH_LO, K * 2>(key, lo);
}

// every stage is a compile-time (K, J) pair, so all indices are constants
template <int E, bool WITH_LO>
__device__ __forceinline__ void wave_bitonic(uint64_t (&key)[E], uint32_t (&lo)[E]) {
    bitonic_from<E, WITH_LO, 2>(key, lo);
}

// Where a sort puts the groups (equal keys, size > 1) it leaves behind: a list
// with a capacity; the first group of a block can also enlist the block for
// the phase-2 kernel.
struct GroupSink {
    Seg* out;
    uint32_t* counter;
    uint32_t cap;
    uint32_t* worklist;  // nullptr inside the per-block kernel
    uint32_t* wcount;
    uint32_t block;

    __device__ __forceinline__ void push(Seg g) const {
        const uint32_t slot = atomicAdd(counter, 1u);
        if (slot < cap) out[slot] = g;
        if (worklist && slot == 0) worklist[atomicAdd(wcount, 1u)] = block;
    }
};

__device__ __forceinline__ GroupSink local_sink(Seg* out, uint32_t* counter) {
    return GroupSink{out, counter, 0xffffffffu, nullptr, nullptr, 0};
}

__device__ __forceinline__ uint8_t bwt_byte(const uint8_t* __restrict__ T, int n, uint32_t i) {
    return T[i == 0 ? (uint32_t)n - 1 : i - 1];
}

// Sort one small segment with one wave and emit its groups of size > 1 to
// `out` (slot from *counter).
// mode 0 (phase 1): keys = the 8 bytes at depth d, rotation index carried
//   alongside; ties do not matter (equal keys become a group).  Sorted
//   positions get their BWT byte (and origPtr) directly; labels are deferred.
// mode 1 (phase 2): keys = (snapshot label << 20) | index from ka[]; members
//   get their new labels.
template <int E, int MODE>
__device__ void wave_sort_segment(const uint8_t* __restrict__ T, int n, Scratch& s, Seg seg, uint32_t d,
                                  const GroupSink& sink, uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig) {
    const int lane = lane_id();
    uint64_t key[E];
    uint32_t lo[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(lane * E + e);
        if (g < seg.len) {
            if (MODE == 0) {
                // payload: rotation index, its BWT byte T[i-1] in bits 24..31
                const uint32_t i = s.sa[seg.start + g];
                uint32_t p = i + d;
                if (p >= (uint32_t)n) p %= (uint32_t)n;
                key[e] = load8(T, n, p);
                lo[e] = i | ((uint32_t)bwt_byte(T, n, i) << 24);
            } else {
                key[e] = s.ka[seg.start + g];
                lo[e] = 0;
            }
        } else {
            key[e] = ~0ull;
            lo[e] = ~0u;
        }
    }
    wave_bitonic<E, MODE == 0>(key, lo);
    constexpr int kShift = MODE == 0 ? 0 : kIdxBits;
    // group flags (key part only), group starts by a max-scan, group ends by
    // "the next item starts a group"
    const uint64_t last_key = key[E - 1] >> kShift;
    const uint64_t prev_last = ((uint64_t)lane_prev((uint32_t)(last_key >> 32)) << 32) | lane_prev((uint32_t)last_key);
    bool flag[E];
    uint32_t gsl[E];
    uint32_t run = 0, lmax = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(lane * E + e);
        const uint64_t pk = e ? key[e - 1] >> kShift : prev_last;
        flag[e] = g == 0 || (key[e] >> kShift) != pk;
        if (flag[e] && g < seg.len) run = g;
        gsl[e] = run;
        lmax = run;
    }
    const uint32_t before = lane_prev(wave_incl_max(lmax), 0u);
    const bool next_lane_flag = __shfl_down((int)flag[0], 1) != 0;  // (lane 63: unused)
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(lane * E + e);
        if (g >= seg.len) continue;
        const uint32_t i = MODE == 0 ? lo[e] & 0xffffffu : (uint32_t)(key[e] & ((1u << kIdxBits) - 1u));
        const uint32_t gs = gsl[e] > before ? gsl[e] : before;
        s.sa[seg.start + g] = i;
        if (MODE == 0) {
            bwt[seg.start + g] = (uint8_t)(lo[e] >> 24);
            if (i == 0) *orig = seg.start + g;
        } else {
            s.rank[i] = seg.start + gs;
        }
        const bool nf = e + 1 < E ? flag[e + 1 < E ? e + 1 : 0] : next_lane_flag;
        if ((g + 1 == seg.len || nf) && g > gs) sink.push(Seg{seg.start + gs, g - gs + 1});
    }
}

// (see GroupSink)
// dispatch a small segment to the right register width
template <int MODE>
__device__ void wave_sort_any(const uint8_t* T, int n, Scratch& s, Seg seg, uint32_t d, const GroupSink& sink,
                              uint8_t* bwt, uint32_t* orig) {
    seg.start = uniform(seg.start);
    seg.len = uniform(seg.len);
    if (seg.len <= 64) wave_sort_segment<1, MODE>(T, n, s, seg, d, sink, bwt, orig);
    else if (seg.len <= 128) wave_sort_segment<2, MODE>(T, n, s, seg, d, sink, bwt, orig);
    else if (seg.len <= 256) wave_sort_segment<4, MODE>(T, n, s, seg, d, sink, bwt, orig);
    else wave_sort_segment<8, MODE>(T, n, s, seg, d, sink, bwt, orig);
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
        (void)k0;  // keys were snapshotted as (label << 20) | index
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
                             Seg* large_next, const GroupSink& sink, uint8_t* __restrict__ bwt,
                             uint32_t* __restrict__ orig) {
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
        const uint32_t i = s.sa[seg.start + ex];
        bwt[seg.start + ex] = bwt_byte(T, n, i);
        if (i == 0) *orig = seg.start + ex;
    } else if (c > 1) {
        const Seg ch{seg.start + ex, c};
        if (c <= (uint32_t)kSmall) {
            s.small[atomicAdd(&sh.cnt[0], 1u)] = ch;
        } else if (d + 1 >= (uint32_t)kMaxDepth) {
            sink.push(ch);
        } else {
            large_next[atomicAdd(&sh.cnt[3], 1u)] = ch;
        }
    }
    __syncthreads();
}

// ---- phase 1a: counting sort of the rotations by their first byte into sa.
// Thread t gets bucket t: start *ex, size *c.
__device__ void count_sort_first(const uint8_t* __restrict__ T, int n, uint32_t* __restrict__ sa, BwtShared& sh,
                                 uint32_t* c_out, uint32_t* ex_out) {
    const int t = threadIdx.x;
    sh.hist[t] = 0;
    __syncthreads();
    // 16 bytes per thread and step (blocks are 64-byte aligned)
    const int n16 = n >> 4;
    const uint4* T4 = reinterpret_cast<const uint4*>(T);
    for (int v = t; v < n16; v += NT) {
        const uint4 w = T4[v];
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) atomicAdd(&sh.hist[(ww[k >> 2] >> ((k & 3) * 8)) & 255u], 1u);
    }
    for (int i = (n16 << 4) + t; i < n; i += NT) atomicAdd(&sh.hist[T[i]], 1u);
    __syncthreads();
    const uint32_t c = sh.hist[t];
    uint32_t total;
    const uint32_t ex = wg_excl_sum<NT>(c, sh.tmp, &total);
    sh.base[t] = ex;
    __syncthreads();
    for (int v = t; v < n16; v += NT) {
        const uint4 w = T4[v];
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int k = 0; k < 16; ++k)
            sa[atomicAdd(&sh.base[(ww[k >> 2] >> ((k & 3) * 8)) & 255u], 1u)] = (uint32_t)(v * 16 + k);
    }
    for (int i = (n16 << 4) + t; i < n; i += NT) sa[atomicAdd(&sh.base[T[i]], 1u)] = (uint32_t)i;
    __syncthreads();
    *c_out = c;
    *ex_out = ex;
}

// ---- phase 1b: expects the small / large bucket lists (sh.cnt[0], [1])
// (expects the large list in s.large, count sh.cnt[1], no small buckets yet;
// groups go to `sink`)
__device__ void bwt_levels(const uint8_t* __restrict__ T, int n, uint8_t* __restrict__ out,
                           uint32_t* __restrict__ orig, Scratch& s, BwtShared& sh, const GroupSink& sink,
                           bool stamp) {
    const int t = threadIdx.x;
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
            wave_sort_any<0>(T, n, s, s.small[idx], depth, sink, out, orig);
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
        for (uint32_t q = 0; q < nlarge; ++q) wg_partition(T, n, s, large[q], depth, sh, large_next, sink, out, orig);
        if (t == 0) sh.cnt[1] = sh.cnt[3];
        __syncthreads();
        Seg* tmpl = large;
        large = large_next;
        large_next = tmpl;
        depth++;
    }
    BZ2MI_PHASE(g_bwt_phase, 3, stamp);
}

// ---- labels, phase 2 and the reordered BWT bytes: expects the groups left
// by phase 1 in s.grp (count sh.cnt[2])
__device__ void bwt_finish(const uint8_t* __restrict__ T, int n, uint8_t* __restrict__ out,
                           uint32_t* __restrict__ orig, Scratch& s, BwtShared& sh, bool stamp) {
    const int t = threadIdx.x;
    // ---- labels for phase 2 (only when groups are left): every position is
    // its own label, members of a group carry the group's start
    uint32_t ng = uniform(sh.cnt[2]);
    if (ng > 0) {
        for (int k = t; k < n; k += NT) s.rank[s.sa[k]] = (uint32_t)k;
        __syncthreads();
        if (t == 0) sh.cnt[4] = 0;
        __syncthreads();
        for (;;) {
            uint32_t idx = 0;
            if (lane_id() == 0) idx = atomicAdd(&sh.cnt[4], 1u);
            idx = uniform(__shfl(idx, 0));
            if (idx >= ng) break;
            const Seg sg = s.grp[idx];
            for (uint32_t k = lane_id(); k < sg.len; k += 64) s.rank[s.sa[sg.start + k]] = sg.start;
        }
        __syncthreads();
    }
    // ---- phase 2: prefix doubling on the unresolved groups
    Seg* g = s.grp;
    Seg* g2 = s.grp2;
    const bool doubled = ng > 0;
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
                s.ka[sg.start + k] = ((uint64_t)s.rank[ih] << kIdxBits) | i;
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
            if (sg.len <= (uint32_t)kSmall) wave_sort_any<1>(T, n, s, sg, 0, local_sink(g2, &sh.cnt[5]), out, orig);
        }
        __syncthreads();
        ng = uniform(sh.cnt[5]);
        Seg* tg = g;
        g = g2;
        g2 = tg;
        __syncthreads();
    }
    BZ2MI_PHASE(g_bwt_phase, 4, stamp);
    // ---- BWT bytes and origPtr of the positions phase 2 reordered (phase 1
    // wrote the others as it placed them); 4 positions per thread and step
    if (doubled) {
        const int n4 = n >> 2;
        const uint4* SA4 = reinterpret_cast<const uint4*>(s.sa);
        uint32_t* O4 = reinterpret_cast<uint32_t*>(out);
        for (int v = t; v < n4; v += NT) {
            const uint4 q = SA4[v];
            const uint32_t ii[4] = {q.x, q.y, q.z, q.w};
            uint32_t w = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                w |= (uint32_t)bwt_byte(T, n, ii[k]) << (8 * k);
                if (ii[k] == 0) *orig = (uint32_t)(v * 4 + k);
            }
            O4[v] = w;
        }
        for (int k = (n4 << 2) + t; k < n; k += NT) {
            const uint32_t i = s.sa[k];
            out[k] = bwt_byte(T, n, i);
            if (i == 0) *orig = (uint32_t)k;
        }
        __syncthreads();
    }
    BZ2MI_PHASE(g_bwt_phase, 5, stamp);
}

// ---- a first-byte bucket (<= 512 rotations) on one wave: counting sort by
// the second byte into sub-buckets, then every rotation of a sub-bucket of
// <= kSub finds its place by counting the smaller (next 8 bytes, index) pairs
// of its sub-bucket; larger sub-buckets get the wave bitonic sort at depth 2.
// For data with a wide alphabet the sub-buckets hold one or two rotations,
// so this is a few operations per rotation instead of a 512-wide network.
constexpr int kSub = 32;

struct Bucket2Lds {
    uint32_t base[257];
    uint64_t key[kSmall];
    uint32_t idx[kSmall];  // rotation index | BWT byte << 24
};

__device__ void wave_sort_bucket2(const uint8_t* __restrict__ T, int n, Scratch& s, Seg seg, const GroupSink& sink,
                                  uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig, Bucket2Lds& L) {
    constexpr int E = kSmall / 64;
    const int lane = lane_id();
#pragma unroll
    for (int j = 0; j < 4; ++j) L.base[lane * 4 + j] = 0;
    uint32_t ii[E], c2[E], slot[E];
    uint64_t key[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(e * 64 + lane);
        c2[e] = 0;
        slot[e] = 0;
        ii[e] = 0;
        key[e] = 0;
        if (g < seg.len) {
            const uint32_t i = s.sa[seg.start + g];
            uint32_t p1 = i + 1, p2 = i + 2;
            if (p1 >= (uint32_t)n) p1 -= (uint32_t)n;
            if (p2 >= (uint32_t)n) p2 %= (uint32_t)n;
            c2[e] = T[p1];
            key[e] = load8(T, n, p2);
            ii[e] = i | ((uint32_t)bwt_byte(T, n, i) << 24);
        }
    }
#pragma unroll
    for (int e = 0; e < E; ++e)
        if ((uint32_t)(e * 64 + lane) < seg.len) slot[e] = atomicAdd(&L.base[c2[e]], 1u);
    // counts -> sub-bucket starts (lane l: counters 4l..4l+3)
    {
        const uint32_t h0 = L.base[lane * 4], h1 = L.base[lane * 4 + 1], h2 = L.base[lane * 4 + 2],
                       h3 = L.base[lane * 4 + 3];
        const uint32_t sum = h0 + h1 + h2 + h3;
        const uint32_t ex = wave_incl_sum(sum) - sum;
        L.base[lane * 4] = ex;
        L.base[lane * 4 + 1] = ex + h0;
        L.base[lane * 4 + 2] = ex + h0 + h1;
        L.base[lane * 4 + 3] = ex + h0 + h1 + h2;
        if (lane == 0) L.base[256] = seg.len;
    }
    uint32_t pos[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        pos[e] = 0;
        if ((uint32_t)(e * 64 + lane) < seg.len) {
            pos[e] = L.base[c2[e]] + slot[e];
            L.key[pos[e]] = key[e];
            L.idx[pos[e]] = ii[e];
        }
    }
    bool any_big = false;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if ((uint32_t)(e * 64 + lane) >= seg.len) continue;
        const uint32_t b0 = L.base[c2[e]], m = L.base[c2[e] + 1] - b0;
        const uint32_t i = ii[e] & 0xffffffu;
        if (m > (uint32_t)kSub) {  // sorted below as a whole
            s.sa[seg.start + pos[e]] = i;
            any_big = true;
            continue;
        }
        uint32_t lt = 0, le = 0, eqlt = 0;
        for (uint32_t q = 0; q < m; ++q) {
            const uint64_t kq = L.key[b0 + q];
            const uint32_t iq = L.idx[b0 + q] & 0xffffffu;
            lt += kq < key[e];
            le += kq <= key[e];
            eqlt += (kq == key[e]) & (iq < i);
        }
        const uint32_t fin = seg.start + b0 + lt + eqlt;
        s.sa[fin] = i;
        bwt[fin] = (uint8_t)(ii[e] >> 24);
        if (i == 0) *orig = fin;
        if (le - lt >= 2 && eqlt == 0) sink.push(Seg{seg.start + b0 + lt, le - lt});
    }
    // sub-buckets too large for counting: wave bitonic at depth 2
    uint64_t bigmask = __ballot(any_big);
    if (bigmask) {
        __threadfence_block();  // the SA entries just written are read by other lanes
        for (int c = 0; c < 256; ++c) {
            const uint32_t b0 = L.base[c], m = L.base[c + 1] - b0;
            if (m > (uint32_t)kSub) wave_sort_any<0>(T, n, s, Seg{seg.start + b0, m}, 2, sink, bwt, orig);
        }
    }
}

constexpr int kQLenBits = 10, kQStartBits = 20;


}  // namespace

// ---- kernel 1: per block, counting sort of the rotations by their first
// byte.  Buckets of <= 512 go to the queue of kernel 2 (all blocks), larger
// ones to the block's large list for kernel 3.
__global__ __launch_bounds__(256) void bwt_bucket_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                         const uint32_t* __restrict__ lens, int nblocks,
                                                         uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                         uint32_t* __restrict__ orig_out, uint64_t* __restrict__ queue,
                                                         uint32_t* __restrict__ qcount, Seg* __restrict__ large_all,
                                                         uint32_t* __restrict__ nlarge, uint32_t* __restrict__ ngroups,
                                                         uint32_t* __restrict__ clist, uint32_t* __restrict__ ccount,
                                                         uint32_t* __restrict__ present_out) {
    __shared__ BwtShared sh;
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    const int t = threadIdx.x;
    const int n = (int)uniform(lens[b]);
    const uint8_t* T = blocks + (size_t)b * stride;
    uint8_t* out = bwt_out + (size_t)b * stride;
    if (t == 0) ngroups[b] = 0;
    if (n <= 1) {
        if (t == 0) {
            if (n == 1) out[0] = T[0];
            orig_out[b] = 0;
            nlarge[b] = 0;
        }
        if (t < 8) present_out[(size_t)b * 8 + t] = (n == 1 && (T[0] >> 5) == t) ? 1u << (T[0] & 31) : 0u;
        return;
    }
    uint32_t* sa = sa_all + (size_t)b * stride;
    uint32_t c, ex;
    count_sort_first(T, n, sa, sh, &c, &ex);
    {  // symbols in use (the MTF symbol map): bit t of the 256-bit set
        const uint64_t m = __ballot(c != 0);
        if (lane_id() == 0) {
            present_out[(size_t)b * 8 + 2 * wave_id()] = (uint32_t)m;
            present_out[(size_t)b * 8 + 2 * wave_id() + 1] = (uint32_t)(m >> 32);
        }
    }
    if (c == 1) {
        const uint32_t i = sa[ex];
        out[ex] = bwt_byte(T, n, i);
        if (i == 0) orig_out[b] = ex;
    }
    const bool small = c > 1 && c <= (uint32_t)kSmall, large = c > (uint32_t)kSmall;
    uint32_t nq, nl;
    const uint32_t r = wg_excl_sum<NT>(small ? 1u : 0u, sh.tmp, &nq);
    const uint32_t rl = wg_excl_sum<NT>(large ? 1u : 0u, sh.tmp, &nl);
    if (t == 0) {
        sh.bcast[0] = nq ? atomicAdd(qcount, nq) : 0u;
        nlarge[b] = nl;
        if (nl) clist[atomicAdd(ccount, 1u)] = (uint32_t)b;
    }
    __syncthreads();
    if (small)
        queue[sh.bcast[0] + r] = ((uint64_t)b << (kQStartBits + kQLenBits)) | ((uint64_t)ex << kQLenBits) | (c - 1);
    if (large) large_all[(size_t)b * 256 + rl] = Seg{ex, c};
}

// ---- kernel 2: one wave per queued bucket (any block): sort by the next 8
// bytes, write SA, BWT bytes and origPtr; groups go to the block's list
__global__ __launch_bounds__(256) void bwt_small_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                        const uint32_t* __restrict__ lens,
                                                        uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                        uint32_t* __restrict__ orig_out,
                                                        const uint64_t* __restrict__ queue,
                                                        const uint32_t* __restrict__ qcount, Seg* __restrict__ grp_all,
                                                        uint32_t* __restrict__ ngroups, uint32_t* __restrict__ p2list,
                                                        uint32_t* __restrict__ p2count) {
    __shared__ Bucket2Lds lds[NT / 64];
    const uint32_t nq = uniform(*qcount);
    const uint32_t nwaves = gridDim.x * (NT / 64);
    for (uint32_t q = blockIdx.x * (NT / 64) + wave_id(); q < nq; q += nwaves) {
        const uint64_t e = queue[q];
        const uint32_t b = uniform((uint32_t)(e >> (kQStartBits + kQLenBits)));
        const Seg seg{(uint32_t)(e >> kQLenBits) & ((1u << kQStartBits) - 1u),
                      (uint32_t)(e & ((1u << kQLenBits) - 1u)) + 1u};
        const int n = (int)uniform(lens[b]);
        Scratch s{};
        s.sa = sa_all + (size_t)b * stride;
        const GroupSink sink{grp_all + (size_t)b * bwt_group_stride(stride), &ngroups[b], 0xffffffffu, p2list, p2count, b};
        wave_sort_bucket2(blocks + (size_t)b * stride, n, s, seg, sink, bwt_out + (size_t)b * stride, orig_out + b,
                          lds[wave_id()]);
    }
}

// ---- kernel 3: blocks with large first-byte buckets, one workgroup slot
// each (blocks pulled from a counter): levels of partitions by the next byte
// and wave sorts of the small children
__global__ __launch_bounds__(256) void bwt_large_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                        const uint32_t* __restrict__ lens, int nblocks,
                                                        uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                        uint32_t* __restrict__ orig_out, uint8_t* scratch,
                                                        size_t scratch_per_slot, int S,
                                                        const Seg* __restrict__ large_all,
                                                        const uint32_t* __restrict__ nlarge,
                                                        Seg* __restrict__ grp_all, uint32_t* __restrict__ ngroups,
                                                        uint32_t* __restrict__ p2list, uint32_t* __restrict__ p2count,
                                                        const uint32_t* __restrict__ clist,
                                                        const uint32_t* __restrict__ ccount, uint32_t* pull) {
    __shared__ BwtShared sh;
    Scratch s = carve(scratch + (size_t)blockIdx.x * scratch_per_slot, S);
    const int t = threadIdx.x;
    const uint32_t nw = uniform(*ccount);
    for (;;) {
        if (t == 0) sh.bcast[0] = atomicAdd(pull, 1u);
        __syncthreads();
        // wave-uniform (SGPR) values keep every branch below uniform; the
        // barrier closing each iteration keeps the back edge convergent
        const uint32_t k = uniform(sh.bcast[0]);
        if (k >= nw) break;
        const int b = (int)uniform(clist[k]);
        const int n = (int)uniform(lens[b]);
        s.sa = sa_all + (size_t)b * stride;
        const uint32_t nl = uniform(nlarge[b]);
        for (uint32_t q = t; q < nl; q += NT) s.large[q] = large_all[(size_t)b * 256 + q];
        if (t < 8) sh.cnt[t] = 0;
        if (t == 0) sh.cnt[1] = nl;
        __syncthreads();
        const GroupSink sink{grp_all + (size_t)b * bwt_group_stride(stride), &ngroups[b], 0xffffffffu, p2list, p2count,
                             (uint32_t)b};
        bwt_levels(blocks + (size_t)b * stride, n, bwt_out + (size_t)b * stride, orig_out + b, s, sh, sink,
                   b == nblocks / 2);
        __syncthreads();
    }
}

// ---- kernel 4: blocks with groups left: labels, prefix doubling, BWT bytes
__global__ __launch_bounds__(256) void bwt_double_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                         const uint32_t* __restrict__ lens, int nblocks,
                                                         uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                         uint32_t* __restrict__ orig_out, uint8_t* scratch,
                                                         size_t scratch_per_slot, int S, Seg* __restrict__ grp_all,
                                                         const uint32_t* __restrict__ ngroups,
                                                         const uint32_t* __restrict__ p2list,
                                                         const uint32_t* __restrict__ p2count, uint32_t* pull) {
    __shared__ BwtShared sh;
    Scratch s = carve(scratch + (size_t)blockIdx.x * scratch_per_slot, S);
    const int t = threadIdx.x;
    const uint32_t nw = uniform(*p2count);
    for (;;) {
        if (t == 0) sh.bcast[0] = atomicAdd(pull, 1u);
        __syncthreads();
        const uint32_t k = uniform(sh.bcast[0]);
        if (k >= nw) break;
        const int b = (int)uniform(p2list[k]);
        const int n = (int)uniform(lens[b]);
        s.sa = sa_all + (size_t)b * stride;
        s.grp = grp_all + (size_t)b * bwt_group_stride(stride);
        if (t < 8) sh.cnt[t] = 0;
        if (t == 0) sh.cnt[2] = ngroups[b];
        __syncthreads();
        bwt_finish(blocks + (size_t)b * stride, n, bwt_out + (size_t)b * stride, orig_out + b, s, sh,
                   b == nblocks / 2);
        __syncthreads();
    }
}

}  // namespace bz2mi
