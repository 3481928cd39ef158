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
BZ2MI_PHASE_TABLE(g_tbk_stat)
BZ2MI_PHASE_TABLE(g_tbk_res)  // text_resolve sums (PHASES builds)
BZ2MI_PHASE_TABLE(g_tbk_x)    // text kernel: tie-round and tied-pair wave time (PHASES builds)
BZ2MI_PHASE_TABLE(g_dbl_stat)  // bwt_finish sums (PHASES builds)
BZ2MI_PHASE_TABLE(g_blk_phase)  // bwt_block_kernel: per-phase wall time summed over workgroups (PHASES builds)
#ifdef TBK_TRACE
__device__ unsigned int* g_tbk_trace;
#endif

// PHASES builds: bwt_text_kernel sums over all its blocks (wall clock of
// thread 0 in 10 ns units for 0..2, counts for the rest)
int tbk_trace(void* p) {
#ifdef TBK_TRACE
    return hipMemcpyToSymbol(HIP_SYMBOL(g_tbk_trace), &p, sizeof(p)) == hipSuccess ? 1 : -1;
#else
    (void)p;
    return 0;
#endif
}

int tbk_stats(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tbk_stat), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

int blk_phase_stats(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_blk_phase), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

int tbk_extra_stats(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tbk_x), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

int tbk_resolve_stats(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tbk_res), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

int dbl_stats(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbl_stat), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

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
    uint32_t bat_start[256];  // batches of small children (pack_children)
    uint32_t bat_len[256];    // length | one-child flag << 31
    uint32_t wfirst[NW];      // resolve_pairs: first run end in each wave's range
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
    Scratch s{};
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
        // little-endian words: bytes pos.. are (w1:w0) >> 8 (pos & 3), then (w2:w1)
        const uint32_t lo32 = __builtin_amdgcn_alignbyte(w1, w0, pos & 3u);
        const uint32_t hi32 = __builtin_amdgcn_alignbyte(w2, w1, pos & 3u);
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

// 4 bytes of the rotation starting at `pos` (< n), most significant first
__device__ __forceinline__ uint32_t load4(const uint8_t* __restrict__ T, int n, uint32_t pos) {
    if (pos + 4 <= (uint32_t)n) {
        const uint32_t* T32 = (const uint32_t*)T + (pos >> 2);
        return __builtin_bswap32(__builtin_amdgcn_alignbyte(T32[1], T32[0], pos & 3u));
    }
    uint32_t k = 0;
    uint32_t j = pos;
    for (int q = 0; q < 4; ++q) {
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
// Every compare-exchange is branch-free: lane masks (which lanes are the
// upper element of a pair, which sort descending) are per-stage constants,
// the decision is one or two 64-bit compares combined on the scalar unit,
// and the moves are selects.  Equal keys never duplicate a payload: an
// exchange either swaps both elements or neither.
template <int LJ>
__device__ __forceinline__ void lane_pair(uint32_t v, uint32_t& a, uint32_t& b) {
    // a = the pair's lower-lane element, b = its upper-lane element, in both lanes
    if constexpr (LJ == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        a = r[0];
        b = r[1];
    } else {
        static_assert(LJ == 32, "lane_pair: permlane distances");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        a = r[0];
        b = r[1];
    }
}

template <int E, bool WITH_LO, int K, int J>
__device__ __forceinline__ void bitonic_stage(uint64_t (&key)[E], uint32_t (&lo)[E]) {
    const int lane = lane_id();
    if constexpr (J < E) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int pe = e ^ J;
            if (pe > e) {
                // ascending pair: out of order when key[pe] < key[e]
                bool sw;
                if constexpr (K < E) {
                    sw = ((e & K) == 0) ? key[pe] < key[e] : key[e] < key[pe];
                } else if constexpr (!WITH_LO) {
                    // no payload: equal keys are interchangeable, one compare
                    sw = (key[pe] < key[e]) != (((lane * E) & K) != 0);
                } else {
                    const bool asc = ((lane * E) & K) == 0;
                    const bool gt = key[pe] < key[e], lt = key[e] < key[pe];
                    sw = asc ? gt : lt;
                }
                const uint64_t a = key[e], b = key[pe];
                key[e] = sw ? b : a;
                key[pe] = sw ? a : b;
                if (WITH_LO) {
                    const uint32_t la = lo[e], lb = lo[pe];
                    lo[e] = sw ? lb : la;
                    lo[pe] = sw ? la : lb;
                }
            }
        }
    } else {
        constexpr int LJ = J / E;
        const bool up = (lane & LJ) != 0;             // upper element of the pair
        const bool desc = ((lane * E) & K) != 0;      // (K >= 2E here: the same for every e)
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if constexpr (LJ >= 16) {
                // both elements of the pair in both lanes; take b when
                // (b < a) ^ up ^ desc
                uint32_t ah, bh, al, bl, pa = 0, pb = 0;
                lane_pair<LJ>((uint32_t)(key[e] >> 32), ah, bh);
                lane_pair<LJ>((uint32_t)key[e], al, bl);
                if (WITH_LO) lane_pair<LJ>(lo[e], pa, pb);
                const uint64_t a = ((uint64_t)ah << 32) | al, b = ((uint64_t)bh << 32) | bl;
                const bool tb = (b < a) != (up != desc);
                key[e] = tb ? b : a;
                if (WITH_LO) lo[e] = tb ? pb : pa;
            } else {
                const uint64_t ok = ((uint64_t)xor_lanes<LJ>((uint32_t)(key[e] >> 32)) << 32) |
                                    xor_lanes<LJ>((uint32_t)key[e]);
                const uint32_t ol = WITH_LO ? xor_lanes<LJ>(lo[e]) : 0u;
                // lower lane keeps the min when ascending, upper the max
                bool take;
                if constexpr (!WITH_LO) {
                    take = (ok < key[e]) != (up != desc);
                } else {
                    const bool lt = ok < key[e], gt = key[e] < ok;
                    take = (up ? gt : lt) != desc;
                }
                key[e] = take ? ok : key[e];
                if (WITH_LO) lo[e] = take ? ol : lo[e];
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

// Small-queue entries: block | start | len-1 | depth (22 | 20 | 9 | 13 bits).
__host__ __device__ inline uint64_t sq_pack(uint32_t b, uint32_t start, uint32_t len, uint32_t depth) {
    return ((uint64_t)b << 42) | ((uint64_t)start << 22) | ((uint64_t)(len - 1) << 13) | depth;
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
    uint64_t* tq;        // non-null: tie groups go to this global queue (with their depth)
    uint32_t* tcount;
    uint32_t* redo;      // non-null (SA-free pass): a group marks the block for the SA path instead

    __device__ __forceinline__ void push(Seg g) const {
        if (redo) {
            *redo = 1u;
            return;
        }
        const uint32_t slot = atomicAdd(counter, 1u);
        if (slot < cap) out[slot] = g;
        if (worklist && slot == 0) worklist[atomicAdd(wcount, 1u)] = block;
    }
    // Called by every active lane; the lanes with `want` push `g` whose
    // rotations share `depth` bytes.  Tie-queue pushes take one atomic per
    // wave (the queue counter is shared by the whole chip).
    __device__ __forceinline__ void push_agg(bool want, Seg g, uint32_t depth) const {
        if (redo) {
            if (__ballot(want) && lane_id() == 0) *redo = 1u;
            return;
        }
        if (!tq) {
            if (want) push(g);
            return;
        }
        const uint64_t m = __ballot(want);
        if (m == 0) return;
        const int leader = __builtin_ctzll(m);
        uint32_t base = 0;
        if (lane_id() == leader) base = atomicAdd(tcount, (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, leader);
        if (want) tq[base + (uint32_t)__popcll(m & __lanemask_lt())] = sq_pack(block, g.start, g.len, depth);
    }
};

__device__ __forceinline__ GroupSink local_sink(Seg* out, uint32_t* counter) {
    return GroupSink{out, counter, 0xffffffffu, nullptr, nullptr, 0, nullptr, nullptr};
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
__device__ __forceinline__ void wave_sort_emit(const uint8_t* __restrict__ T, int n, Scratch& s, Seg seg, uint32_t d,
                               uint64_t (&key)[E], uint32_t (&lo)[E], const GroupSink& sink,
                               uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig);

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
    wave_sort_emit<E, MODE>(T, n, s, seg, d, key, lo, sink, bwt, orig);
}

// Sort keys already loaded (blocked or any layout; padding = ~0) and emit:
// item g of the sorted order lands at seg.start + g.
template <int E, int MODE>
__device__ __forceinline__ void wave_sort_emit(const uint8_t* __restrict__ T, int n, Scratch& s, Seg seg, uint32_t d,
                               uint64_t (&key)[E], uint32_t (&lo)[E], const GroupSink& sink,
                               uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig) {
    const int lane = lane_id();
    uint32_t d0 = 8;  // bytes the keys compare
    if constexpr (MODE == 0) {
        // a valid key of eight 0xff bytes would tie with the padding: then
        // this segment sorts on 7 bytes first (the deepening goes on from there)
        bool ff = false;
#pragma unroll
        for (int e = 0; e < E; ++e) ff |= lo[e] != ~0u && key[e] == ~0ull;
        if (__ballot(ff)) {
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (lo[e] != ~0u) key[e] >>= 8;
            d0 = 7;
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
        const bool valid = g < seg.len;
        const uint32_t i = MODE == 0 ? lo[e] & 0xffffffu : (uint32_t)(key[e] & ((1u << kIdxBits) - 1u));
        const uint32_t gs = gsl[e] > before ? gsl[e] : before;
        if (valid) {
            if (MODE != 0 || s.sa) s.sa[seg.start + g] = i;
            if (MODE == 0) {
                bwt[seg.start + g] = (uint8_t)(lo[e] >> 24);
                if (i == 0) *orig = seg.start + g;
            } else {
                s.rank[i] = seg.start + gs;
            }
        }
        const bool nf = e + 1 < E ? flag[e + 1 < E ? e + 1 : 0] : next_lane_flag;
        // every lane calls (the tie-queue push is wave-aggregated)
        sink.push_agg(valid && (g + 1 == seg.len || nf) && g > gs, Seg{seg.start + gs, g - gs + 1}, d + d0);
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
// the whole workgroup, then relabel and emit subgroups (emit(Seg), one thread
// per subgroup).
template <class Emit>
__device__ void wg_sort_group(Scratch& s, Seg seg, BwtShared& sh, Emit emit) {
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
                emit(Seg{seg.start + (uint32_t)k, e - (uint32_t)k});
            }
        }
        carry = carry > tot ? carry : tot;
        __syncthreads();
    }
}

// ---- phase 1a: counting sort of the rotations by their first byte into sa.
// Thread t gets bucket t: start *ex, size *c.
__device__ void count_sort_first(const uint8_t* __restrict__ T, int n, uint32_t* __restrict__ sa, BwtShared& sh,
                                 uint32_t* c_out, uint32_t* ex_out, uint32_t* stage, uint32_t* th, uint32_t* ts) {
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
    // scatter, staged per tile of 4096 rotations: ranks inside the tile by
    // LDS atomics, the tile ordered by first byte in LDS, then written out as
    // runs (consecutive threads -> consecutive SA slots of a bucket) instead
    // of one scattered 4-byte store per rotation
    for (int tile0 = 0; tile0 < n; tile0 += NT * 16) {
        th[t] = 0;
        __syncthreads();
        const int i0 = tile0 + t * 16;
        uint32_t bv[16], rk[16];
        if (i0 + 16 <= n) {
            const uint4 w = T4[i0 >> 4];
            const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int k = 0; k < 16; ++k) bv[k] = (ww[k >> 2] >> ((k & 3) * 8)) & 255u;
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) bv[k] = i0 + k < n ? T[i0 + k] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) rk[k] = i0 + k < n ? atomicAdd(&th[bv[k]], 1u) : 0u;
        __syncthreads();
        uint32_t tn;
        ts[t] = wg_excl_sum<NT>(th[t], sh.tmp, &tn);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (i0 + k < n) stage[ts[bv[k]] + rk[k]] = (uint32_t)(i0 + k) | (bv[k] << 24);
        __syncthreads();
        for (uint32_t j = t; j < tn; j += NT) {
            const uint32_t v = stage[j], b = v >> 24;
            sa[sh.base[b] + (j - ts[b])] = v & 0xffffffu;
        }
        __syncthreads();
        sh.base[t] += th[t];
        __syncthreads();
    }
    *c_out = c;
    *ex_out = ex;
}

// ---- repeat pairs.  A group of two rotations {a, b}, b = a + d (mod n), is a
// pair of offset d.  Along a repeated passage every (a + m, b + m) is a pair of
// the same offset, so a and b agree on their first bytes up to the end E of the
// run of positions a, a+1, .. whose partner offset is d, and their order is the
// order of the rotations x = E + 1 and y = x + d -- which the labels give
// whenever x and y lie in different groups (labels are order-consistent at
// every refinement, and the pairs decided during this pass only refine their
// own groups).  One pass over the block (partner offsets, run ends) and O(1)
// per pair replace the log2(repeat length) doubling rounds a long repeated
// passage costs; pairs whose x, y share a larger group, and every larger
// group, go on to the doubling (in g2; returns their count, *undecided the
// pairs among them).
constexpr uint32_t kNoEnd = 0xffffffffu;

__device__ uint32_t resolve_pairs(int n, Scratch& s, BwtShared& sh, const Seg* g, uint32_t ng, Seg* g2,
                                  uint32_t* undecided) {
    const int t = threadIdx.x;
    uint32_t* pd = s.va;  // partner offset of a pair member, 0 elsewhere
    uint32_t* ne = s.vb;  // last position of p's run of equal pd (kNoEnd: not in p's wave range)
    for (int p = t; p < n; p += NT) pd[p] = 0;
    if (t < 2) sh.cnt[6 + t] = 0;
    __syncthreads();
    for (uint32_t q = t; q < ng; q += NT) {
        const Seg sg = g[q];
        if (sg.len == 2) {
            const uint32_t a = s.sa[sg.start], b = s.sa[sg.start + 1];
            pd[a] = b > a ? b - a : b + n - a;
            pd[b] = a > b ? a - b : a + n - b;
        }
    }
    __syncthreads();
    // run ends: wave w scans its range [lo, hi) from the right, 64 positions a step
    const int w = wave_id(), lane = lane_id();
    const uint32_t chunk = (((uint32_t)n + NW - 1) / NW + 63u) & ~63u;
    const uint32_t lo = (uint32_t)w * chunk, hi = min((uint32_t)n, lo + chunk);
    uint32_t carry = kNoEnd;
    if (lo < hi) {
        for (uint32_t ts = lo + ((hi - 1 - lo) & ~63u);; ts -= 64) {
            const uint32_t p = ts + (uint32_t)lane;
            const bool valid = p < hi;
            bool bnd = false;
            if (valid) {
                const uint32_t pn = p + 1 == (uint32_t)n ? 0u : p + 1;
                bnd = pd[p] != pd[pn];
            }
            const uint64_t B = __ballot(bnd);
            const uint64_t above = B & (~0ull << lane);
            if (valid) ne[p] = above ? ts + (uint32_t)__builtin_ctzll(above) : carry;
            if (B) carry = ts + (uint32_t)__builtin_ctzll(B);
            if (ts == lo) break;
        }
    }
    if (lane == 0) sh.wfirst[w] = carry;
    __syncthreads();
    for (uint32_t q = t; q < ng; q += NT) {
        const Seg sg = g[q];
        bool keep = sg.len != 2;
        if (!keep) {
            const uint32_t a = s.sa[sg.start], b = s.sa[sg.start + 1];
            const uint32_t d = pd[a];
            uint32_t e = ne[a];
            if (e == kNoEnd) {  // the run leaves a's wave range: the next range's first end (cyclic)
                const int wa = (int)(a / chunk);
                for (int k = 1; k <= NW && e == kNoEnd; ++k) e = sh.wfirst[(wa + k) % NW];
            }
            bool a_first;
            if (e == kNoEnd) {  // every position pairs with offset d = n / 2: equal rotations
                a_first = a < b;
            } else {
                const uint32_t x = e + 1 == (uint32_t)n ? 0u : e + 1;
                const uint32_t y = x + d >= (uint32_t)n ? x + d - n : x + d;
                const uint32_t la = s.rank[x], lb = s.rank[y];
                keep = la == lb;
                a_first = la < lb;
            }
            if (!keep) {
                const uint32_t f = a_first ? a : b, l = a_first ? b : a;
                s.sa[sg.start] = f;
                s.sa[sg.start + 1] = l;
                s.rank[f] = sg.start;
                s.rank[l] = sg.start + 1;
            } else {
                atomicAdd(&sh.cnt[7], 1u);
            }
        }
        if (keep) g2[atomicAdd(&sh.cnt[6], 1u)] = sg;
    }
    __syncthreads();
    *undecided = uniform(sh.cnt[7]);
    const uint32_t r = uniform(sh.cnt[6]);
    __syncthreads();
    return r;
}

// ---- labels, phase 2 and the reordered BWT bytes: expects the groups left
// by phase 1 in s.grp (count sh.cnt[2])
__device__ void bwt_finish(const uint8_t* __restrict__ T, int n, uint8_t* __restrict__ out,
                           uint32_t* __restrict__ orig, Scratch& s, BwtShared& sh, bool stamp) {
    const int t = threadIdx.x;
    // ---- labels for phase 2 (only when groups are left): every position is
    // its own label, members of a group carry the group's start
    uint32_t ng = uniform(sh.cnt[2]);
#ifdef BZ2MI_PHASES
    const unsigned long long dk0 = wall_clock64();
    unsigned long long dkp = 0, dkl = 0;
    uint32_t rounds = 0, first_pass = 1;
    if (t == 0 && ng > 0) {
        atomicAdd(&g_dbl_stat[0], 1ull);
        atomicAdd(&g_dbl_stat[3], (unsigned long long)ng);
        atomicMax(&g_dbl_stat[10], (unsigned long long)ng);
    }
#endif
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
#ifdef BZ2MI_PHASES
    dkl = wall_clock64() - dk0;
#endif
    // ---- phase 2: prefix doubling on the unresolved groups
    Seg* g = s.grp;
    Seg* g2 = s.grp2;
    const bool doubled = ng > 0;
    bool pairs = true;
    for (long long h = 9; ng > 0 && h < n; h <<= 1) {
        // repeat pairs first (again while the last pass decided some and
        // enough are left to pay for the block-wide pass)
#ifdef BZ2MI_PHASES
        rounds++;
#endif
        if (pairs) {
            uint32_t und;
#ifdef BZ2MI_PHASES
            const unsigned long long dp0 = wall_clock64();
#endif
            const uint32_t ng2 = resolve_pairs(n, s, sh, g, ng, g2, &und);
#ifdef BZ2MI_PHASES
            dkp += wall_clock64() - dp0;
            if (t == 0 && first_pass) {
                atomicAdd(&g_dbl_stat[6], (unsigned long long)(ng - ng2));
                atomicAdd(&g_dbl_stat[7], (unsigned long long)und);
                atomicAdd(&g_dbl_stat[8], (unsigned long long)ng2);
            }
            first_pass = 0;
#endif
            pairs = ng2 < ng && und > 64;
            ng = ng2;
            Seg* tg = g;
            g = g2;
            g2 = tg;
            if (ng == 0) break;
        }
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
            if (uniform(sg.len) > (uint32_t)kSmall)
                wg_sort_group(s, sg, sh, [&](Seg o) { g2[atomicAdd(&sh.cnt[5], 1u)] = o; });
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
#ifdef BZ2MI_PHASES
    if (t == 0 && doubled) {
        const unsigned long long dt = wall_clock64() - dk0;
        atomicAdd(&g_dbl_stat[1], dt);
        atomicMax(&g_dbl_stat[2], dt);
        atomicAdd(&g_dbl_stat[4], (unsigned long long)rounds);
        atomicMax(&g_dbl_stat[5], (unsigned long long)rounds);
        atomicAdd(&g_dbl_stat[11], dkp);
        atomicAdd(&g_dbl_stat[12], dkl);
    }
#endif
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

// ---- a bucket of <= 512 rotations with a common prefix of d bytes, on one
// wave.  The 8-byte keys at depth d are loaded once and counting-sorted by
// their first byte (byte d) into LDS sub-buckets.  Then either
//   * text-like segments (>= 1/8 of the rotations in sub-buckets of > kSub): one wave
//     sort of the whole segment on the keys, or
//   * every rotation of a sub-bucket of <= kSub finds its place by counting
//     the smaller (key, index) pairs of its sub-bucket (wide alphabets: one
//     or two rotations per sub-bucket), and larger sub-buckets get a wave
//     sort of their own;
// all from LDS.  Tie groups go to the sink with their depth.
constexpr int kSub = 32;
constexpr int kBigBucket = 4096;  // largest first-byte bucket bwt_bigbucket_kernel sorts
// sub-bucket ranks by counting (LDS text): members per load round, and whether
// every element's state is loaded before the first count
#ifndef BZ2MI_CNT_UNROLL
#define BZ2MI_CNT_UNROLL 1
#endif
#ifndef BZ2MI_CNT_PREFETCH
#define BZ2MI_CNT_PREFETCH 1
#endif
// the member loops of a lane's elements interleaved (one trip per member
// index over all elements; random BWT 10.08 -> 9.64 ms per GiB) or one
// element after the other
#ifndef BZ2MI_CNT_INTERLEAVE
#define BZ2MI_CNT_INTERLEAVE 1
#endif
constexpr int kCntUnroll = BZ2MI_CNT_UNROLL;
constexpr bool kCntPrefetch = BZ2MI_CNT_PREFETCH != 0;

struct Bucket2Lds {
    static constexpr bool kKeys = true;
    uint32_t base[257];
    uint64_t key[kSmall];  // 8 bytes at depth d, grouped by byte d
    uint32_t idx[kSmall];  // rotation index | BWT byte << 24
};
// the same without the key copies, for a text held in LDS (keys re-read from it)
struct Bucket3Lds {
    static constexpr bool kKeys = false;
    uint32_t base[257];
    uint32_t idx[kSmall];
};

template <class BL>
__device__ __forceinline__ uint64_t lds_key(const uint8_t* __restrict__ T, int n, const BL& L, uint32_t pos,
                                            uint32_t d) {
    if constexpr (BL::kKeys) {
        return L.key[pos];
    } else {
        uint32_t p = (L.idx[pos] & 0x1ffffu) + d;  // LDS text: n < 2^17 (bits 17+: key bits)
        if (p >= (uint32_t)n) p %= (uint32_t)n;
        return load8(T, n, p);
    }
}

// ---- text in LDS: sorts on unique 57-bit keys and resolves ties in the wave.
// A sort key is (6 text bytes at depth d) << 9 | item position, so keys are
// unique and carry no payload (one 64-bit compare and two selects per
// compare-exchange, a third of the cost of key + payload).  Items whose six
// bytes tie are compacted to the front of their LDS index slice as
// (index | destination slot << 17 | group head << 26) and sorted again on
// (group's first slot << 49 | 5 bytes deeper << 9 | item), round after round,
// until none tie; groups still tied at kMaxDepth go to the sink (tie kernel /
// prefix doubling) with their SA entries written.  Requires n < 2^17.
constexpr int kLdsKeyBytes = 6;   // bytes of the first round
constexpr int kLdsTieBytes = 5;   // bytes of every tie round
// the same for IB item-index bits (9: up to 512 items; 8: up to 256, one more
// text byte per round)
__host__ __device__ constexpr int lds_key_bytes(int IB) { return (64 - IB) / 8; }
__host__ __device__ constexpr int lds_tie_bytes(int IB) { return (64 - 2 * IB) / 8; }
static_assert(lds_key_bytes(9) == kLdsKeyBytes && lds_tie_bytes(9) == kLdsTieBytes, "LDS key layout");

__device__ __forceinline__ uint64_t lane_next64(uint64_t v) {
    const uint32_t lo = (uint32_t)__shfl_down((int)(uint32_t)v, 1), hi = (uint32_t)__shfl_down((int)(uint32_t)(v >> 32), 1);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t lane_prev64(uint64_t v) {
    return ((uint64_t)lane_prev((uint32_t)(v >> 32)) << 32) | lane_prev((uint32_t)v);
}

// one emission pass over sorted unique keys (prefix = key >> 9): final items
// are written, tied ones compacted into idx[0, t) for the next round; returns t
template <int E, int IB = 9>
__device__ __forceinline__ uint32_t lds_emit_round(const uint8_t* __restrict__ T, int n, Scratch& s, uint32_t base,
                                                   uint32_t m, const uint64_t (&key)[E], const uint32_t (&src)[E],
                                                   const uint32_t (&dst)[E], uint8_t* __restrict__ bwt,
                                                   uint32_t* __restrict__ orig, uint32_t* __restrict__ idx) {
    const int lane = lane_id();
    uint64_t pk[E];
#pragma unroll
    for (int e = 0; e < E; ++e) pk[e] = key[e] >> IB;
    const uint64_t before = lane_prev64(pk[E - 1]), after = lane_next64(pk[0]);
    bool tie[E], head[E];
    uint32_t cnt = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(lane * E + e);
        const bool valid = g < m;
        const bool tl = g > 0 && pk[e] == (e ? pk[e - 1] : before);
        const bool tr = g + 1 < m && pk[e] == (e + 1 < E ? pk[e + 1 < E ? e + 1 : 0] : after);
        tie[e] = valid && (tl || tr);
        head[e] = tie[e] && !tl;
        cnt += tie[e];
        if (valid && !tie[e]) {
            const uint32_t i = src[e], pos = base + dst[e];
            if (s.sa) s.sa[pos] = i;
            if (bwt) {  // (null: the caller writes the BWT bytes from the final SA)
                bwt[pos] = bwt_byte(T, n, i);
                if (i == 0) *orig = pos;
            }
        }
    }
    const uint32_t inc = wave_incl_sum(cnt);
    const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    if (t) {
        __builtin_amdgcn_wave_barrier();  // every lane has read idx[] (caller) before it is rewritten
        uint32_t o = inc - cnt;
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (tie[e]) idx[o++] = src[e] | (dst[e] << 17) | ((uint32_t)head[e] << 26);
        __builtin_amdgcn_wave_barrier();
    }
    return t;
}

// tie round over the t compacted items idx[0, t) at depth D
template <int E, int IB = 9>
__device__ __forceinline__ uint32_t lds_tie_round(const uint8_t* __restrict__ T, int n, Scratch& s, uint32_t base,
                                               uint32_t t, uint32_t D, uint8_t* __restrict__ bwt,
                                               uint32_t* __restrict__ orig, uint32_t* __restrict__ idx) {
    const int lane = lane_id();
    uint64_t key[E];
    uint32_t gs[E], run = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t q = (uint32_t)(lane * E + e);
        const uint32_t w = q < t ? idx[q] : 0u;
        if (w >> 26) run = (w >> 17) & 511u;  // group heads carry increasing slots
        gs[e] = run;
        key[e] = q < t ? (uint64_t)(w & 0x1ffffu) : ~0ull;  // index, keyed below
    }
    const uint32_t carry = lane_prev(wave_incl_max(run), 0u);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t q = (uint32_t)(lane * E + e);
        if (q < t) {
            const uint32_t g = gs[e] > carry ? gs[e] : carry;
            uint32_t p = (uint32_t)key[e] + D;  // index < n < 2^17, D < 2^16
            if (p >= (uint32_t)n) p %= (uint32_t)n;
            key[e] = ((uint64_t)g << (IB + 8 * lds_tie_bytes(IB))) | ((load8(T, n, p) >> (64 - 8 * lds_tie_bytes(IB))) << IB) | q;
        }
    }
    uint32_t dummy[E];
    wave_bitonic<E, false>(key, dummy);
    uint32_t src[E], dst[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t r = (uint32_t)(lane * E + e);
        src[e] = r < t ? idx[key[e] & ((1u << IB) - 1u)] & 0x1ffffu : 0u;
        dst[e] = r < t ? (idx[r] >> 17) & 511u : 0u;
    }
    return lds_emit_round<E, IB>(T, n, s, base, t, key, src, dst, bwt, orig, idx);
}

__device__ __forceinline__ uint32_t lds_tie_round_any(const uint8_t* T, int n, Scratch& s, uint32_t base, uint32_t t,
                                                      uint32_t D, uint8_t* bwt, uint32_t* orig, uint32_t* idx) {
    if (t <= 64) return lds_tie_round<1>(T, n, s, base, t, D, bwt, orig, idx);
    if (t <= 128) return lds_tie_round<2>(T, n, s, base, t, D, bwt, orig, idx);
    if (t <= 256) return lds_tie_round<4>(T, n, s, base, t, D, bwt, orig, idx);
    return lds_tie_round<8>(T, n, s, base, t, D, bwt, orig, idx);
}

// the same for at most 64 * MAXE items (no instance of the larger rounds)
template <int MAXE, int IB = 9>
__device__ __forceinline__ uint32_t lds_tie_round_upto(const uint8_t* T, int n, Scratch& s, uint32_t base, uint32_t t,
                                                       uint32_t D, uint8_t* bwt, uint32_t* orig, uint32_t* idx) {
    if (t <= 64) return lds_tie_round<1, IB>(T, n, s, base, t, D, bwt, orig, idx);
    if (MAXE <= 2 || t <= 128) return lds_tie_round<MAXE <= 2 ? MAXE : 2, IB>(T, n, s, base, t, D, bwt, orig, idx);
    if (MAXE <= 4 || t <= 256) return lds_tie_round<MAXE <= 4 ? MAXE : 4, IB>(T, n, s, base, t, D, bwt, orig, idx);
    return lds_tie_round<MAXE, IB>(T, n, s, base, t, D, bwt, orig, idx);
}

// groups still tied at the depth limit: SA entries written, groups to the sink
__device__ __forceinline__ void lds_tie_spill(const uint8_t* __restrict__ T, int n, Scratch& s, uint32_t base,
                                           uint32_t t, uint32_t D, const GroupSink& sink,
                                           const uint32_t* __restrict__ idx) {
    for (uint32_t q0 = 0; q0 < t; q0 += 64) {
        const uint32_t q = q0 + (uint32_t)lane_id();
        const uint32_t w = q < t ? idx[q] : 0u;
        const uint32_t slot = (w >> 17) & 511u;
        if (q < t && s.sa) s.sa[base + slot] = w & 0x1ffffu;
        uint32_t len = 0;
        if (q < t && (w >> 26)) {
            len = 1;
            while (q + len < t && !(idx[q + len] >> 26)) ++len;
        }
        sink.push_agg(len >= 2, Seg{base + slot, len}, D);
    }
}

template <int E, class BL>
__device__ __forceinline__ uint32_t wave_sort_lds_text(const uint8_t* __restrict__ T, int n, Scratch& s, uint32_t start,
                                                   uint32_t b0, uint32_t m, uint32_t d, const GroupSink& sink,
                                                   uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig,
                                                   BL& L) {
    const int lane = lane_id();
    uint32_t* idx = L.idx + b0;
    uint64_t key[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(lane * E + e);
        if (g < m) {
            uint32_t p = (idx[g] & 0x1ffffu) + d;
            if (p >= (uint32_t)n) p %= (uint32_t)n;
            key[e] = ((load8(T, n, p) >> (64 - 8 * kLdsKeyBytes)) << 9) | g;
        } else {
            key[e] = ~0ull;
        }
    }
    uint32_t dummy[E];
    wave_bitonic<E, false>(key, dummy);
    uint32_t src[E], dst[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(lane * E + e);
        src[e] = g < m ? idx[key[e] & 511u] & 0x1ffffu : 0u;
        dst[e] = g;
    }
    return lds_emit_round<E>(T, n, s, start + b0, m, key, src, dst, bwt, orig, idx);
}

// The same first round straight from a batch's SA entries held in registers
// (pre[e] = entry e*64+lane): item g = e*64+lane is keyed from pre[e] and its
// index parked at idx[g] (contiguous stores), so the batch is not counting-
// sorted into LDS sub-buckets first and its keys are gathered from the text
// once.  (Any placement of unsorted items over the slots is a valid input of
// the bitonic network.)
template <int ES, int PE, int IB = 9>
__device__ __forceinline__ uint32_t wave_sort_pre_text(const uint8_t* __restrict__ T, int n, Scratch& s,
                                                       uint32_t start, uint32_t m, uint32_t d,
                                                       uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig,
                                                       uint32_t* __restrict__ idx,
                                                       const uint32_t (&pre)[PE]) {
    static_assert(ES <= PE, "slots");
    const int lane = lane_id();
    uint64_t key[ES];
#pragma unroll
    for (int e = 0; e < ES; ++e) {
        const uint32_t g = (uint32_t)(e * 64 + lane);
        if (g < m) {
            const uint32_t i = pre[e];
            idx[g] = i;
            uint32_t p = i + d;
            if (p >= (uint32_t)n) p %= (uint32_t)n;
            key[e] = ((load8(T, n, p) >> (64 - 8 * lds_key_bytes(IB))) << IB) | g;
        } else {
            key[e] = ~0ull;
        }
    }
    __builtin_amdgcn_wave_barrier();  // idx[] written before the reads below
    uint32_t dummy[ES];
    wave_bitonic<ES, false>(key, dummy);
    uint32_t src[ES], dst[ES];
#pragma unroll
    for (int e = 0; e < ES; ++e) {
        const uint32_t r = (uint32_t)(lane * ES + e);
        src[e] = r < m ? idx[key[e] & ((1u << IB) - 1u)] : 0u;
        dst[e] = r;
    }
    return lds_emit_round<ES, IB>(T, n, s, start, m, key, src, dst, bwt, orig, idx);
}

// the tie rounds after a first round left t items tied (depth d + kLdsKeyBytes)
__device__ __forceinline__ void lds_ties(const uint8_t* __restrict__ T, int n, Scratch& s, uint32_t base, uint32_t t,
                                         uint32_t d, const GroupSink& sink, uint8_t* __restrict__ bwt,
                                         uint32_t* __restrict__ orig, uint32_t* __restrict__ idx) {
    uint32_t D = d + kLdsKeyBytes;
    while (t) {
        if (D + kLdsTieBytes > (uint32_t)kMaxDepth) {
            lds_tie_spill(T, n, s, base, t, D, sink, idx);
            return;
        }
        t = uniform(lds_tie_round_any(T, n, s, base, t, D, bwt, orig, idx));
        D += kLdsTieBytes;
    }
}

// wave sort of LDS items [b0, b0+m) (m <= 64*E), emitted at seg.start + b0
template <int E, class BL>
__device__ __forceinline__ void wave_sort_lds(const uint8_t* __restrict__ T, int n, Scratch& s, uint32_t start,
                                              uint32_t b0, uint32_t m, uint32_t d, const GroupSink& sink,
                                              uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig,
                                              BL& L) {
    static_assert(BL::kKeys, "LDS-text buckets sort with wave_sort_lds_text");
    const int lane = lane_id();
    uint64_t key[E];
    uint32_t lo[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(lane * E + e);
        key[e] = g < m ? lds_key(T, n, L, b0 + g, d) : ~0ull;
        lo[e] = g < m ? L.idx[b0 + g] : ~0u;
    }
    wave_sort_emit<E, 0>(T, n, s, Seg{start + b0, m}, d, key, lo, sink, bwt, orig);
}

template <class BL>
__device__ __forceinline__ void wave_sort_lds_any(const uint8_t* __restrict__ T, int n, Scratch& s, uint32_t start,
                                               uint32_t b0, uint32_t m, uint32_t d, const GroupSink& sink,
                                               uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig,
                                               BL& L) {
    if constexpr (!BL::kKeys) {
        uint32_t t;
        if (m <= 64) t = wave_sort_lds_text<1, BL>(T, n, s, start, b0, m, d, sink, bwt, orig, L);
        else if (m <= 128) t = wave_sort_lds_text<2, BL>(T, n, s, start, b0, m, d, sink, bwt, orig, L);
        else if (m <= 256) t = wave_sort_lds_text<4, BL>(T, n, s, start, b0, m, d, sink, bwt, orig, L);
        else t = wave_sort_lds_text<8, BL>(T, n, s, start, b0, m, d, sink, bwt, orig, L);
        if (t) lds_ties(T, n, s, start + b0, t, d, sink, bwt, orig, L.idx + b0);
    } else {
        if (m <= 64) wave_sort_lds<1, BL>(T, n, s, start, b0, m, d, sink, bwt, orig, L);
        else if (m <= 128) wave_sort_lds<2, BL>(T, n, s, start, b0, m, d, sink, bwt, orig, L);
        else if (m <= 256) wave_sort_lds<4, BL>(T, n, s, start, b0, m, d, sink, bwt, orig, L);
        else wave_sort_lds<8, BL>(T, n, s, start, b0, m, d, sink, bwt, orig, L);
    }
}

// `pre`: the batch's SA entries, loaded ahead by the caller (entry e*64+lane in
// pre[e]); E: element slots per lane the batch needs (seg.len <= 64*E), so a
// random block's batches of ~350 rotations run 6 slots, not kSmall/64 = 8
template <int E, class BL>
__device__ __forceinline__ void wave_sort_bucket2_e(const uint8_t* __restrict__ T, int n, Scratch& s, Seg seg,
                                                    uint32_t d, const GroupSink& sink, uint8_t* __restrict__ bwt,
                                                    uint32_t* __restrict__ orig, BL& L,
                                                    const uint32_t (&pre)[kSmall / 64]) {
    static_assert(E <= kSmall / 64, "slots");
    const int lane = lane_id();
#ifdef BZ2MI_PHASES
    // per-phase wave time of the batch sorts of every 64th block (g_blk_phase[11..14])
    const bool bs_on = (blockIdx.x & 63u) == 0 && lane == 0;
    unsigned long long bs_t = bs_on ? wall_clock64() : 0ull;
    auto bs_mark = [&](int k) {
        if (bs_on) {
            const unsigned long long now = wall_clock64();
            atomicAdd(&g_blk_phase[k], now - bs_t);
            bs_t = now;
        }
    };
#else
    auto bs_mark = [](int) {};
#endif
#pragma unroll
    for (int j = 0; j < 4; ++j) L.base[lane * 4 + j] = 0;
    // LDS text: every element's own state for the counting phase, kept in
    // registers from the scatter (word; sub-bucket start | size << 9 | its
    // slot in it << 20, 0 when not a small sub-bucket) -- no LDS reads of it
    uint32_t own_w[E], own_sb[E];
    {
        uint32_t ii[E], slot[E];
        uint64_t key[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t g = (uint32_t)(e * 64 + lane);
            slot[e] = 0;
            ii[e] = 0;
            key[e] = 0;
            if (g < seg.len) {
                const uint32_t i = pre[e];
                uint32_t p = i + d;
                if (p >= (uint32_t)n) p %= (uint32_t)n;
                if constexpr (BL::kKeys) {
                    key[e] = load8(T, n, p);
                    ii[e] = i | ((uint32_t)bwt_byte(T, n, i) << 24);
                } else {  // LDS text (n < 2^17): byte d and the 15 key bits after it ride along
                    const uint32_t k4 = load4(T, n, p);
                    key[e] = (uint64_t)k4 << 32;
                    ii[e] = i | (((k4 >> 9) & 0x7fffu) << 17);
                }
            }
        }
#pragma unroll
        for (int e = 0; e < E; ++e)
            if ((uint32_t)(e * 64 + lane) < seg.len) slot[e] = atomicAdd(&L.base[key[e] >> 56], 1u);
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
#pragma unroll
        for (int e = 0; e < E; ++e) {
            own_w[e] = ii[e];
            own_sb[e] = 0;
            if ((uint32_t)(e * 64 + lane) < seg.len) {
                const uint32_t c = (uint32_t)(key[e] >> 56);
                const uint32_t b0 = L.base[c];
                const uint32_t pos = b0 + slot[e];
                if constexpr (BL::kKeys) {
                    L.key[pos] = key[e];
                } else {
                    const uint32_t m = L.base[c + 1] - b0;
                    own_sb[e] = m <= (uint32_t)kSub ? b0 | (m << 9) | (slot[e] << 20) : 0u;
                }
                L.idx[pos] = ii[e];
            }
        }
    }
    bs_mark(11);
    // rotations in sub-buckets of > kSub (lane l: sub-buckets 4l..4l+3)
    uint32_t inbig = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t c = (uint32_t)(lane * 4 + j);
        const uint32_t m = L.base[c + 1] - L.base[c];
        inbig += m > (uint32_t)kSub ? m : 0u;
    }
    const uint32_t nbig = wave_sum(inbig);
    // (a whole-segment sort unless fewer than 1/8 of the rotations are in big
    // sub-buckets: measured on text, 2 -> 8 saves ~1% of the BWT)
    if (8 * nbig > seg.len) {
        wave_sort_lds_any(T, n, s, seg.start, 0, seg.len, d, sink, bwt, orig, L);
        bs_mark(14);
        return;
    }
    // small sub-buckets: ranks by counting (striped positions p = e*64 + lane)
    if constexpr (BL::kKeys) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t p = (uint32_t)(e * 64 + lane);
            const bool inseg = p < seg.len;
            const uint32_t ii = inseg ? L.idx[p] : 0u;
            const uint64_t k = inseg ? lds_key(T, n, L, p, d) : 0ull;
            const uint32_t c = (uint32_t)(k >> 56);
            const uint32_t i = ii & 0xffffffu;
            const uint32_t b0 = L.base[c], m = inseg ? L.base[c + 1] - b0 : 0u;
            const bool mine = inseg && m <= (uint32_t)kSub;
            uint32_t lt = 0, le = 0, eqlt = 0;
            for (uint32_t q = 0; q < (mine ? m : 0u); ++q) {
                const uint64_t kq = lds_key(T, n, L, b0 + q, d);
                const uint32_t iq = L.idx[b0 + q] & 0xffffffu;
                lt += kq < k;
                le += kq <= k;
                eqlt += (kq == k) & (iq < i);
            }
            const uint32_t fin = seg.start + b0 + lt + eqlt;
            if (mine) {
                if (s.sa) s.sa[fin] = i;
                bwt[fin] = (uint8_t)(ii >> 24);
                if (i == 0) *orig = fin;
            }
            sink.push_agg(mine && le - lt >= 2 && eqlt == 0, Seg{seg.start + b0 + lt, le - lt}, d + 8);
        }
    } else {
        // LDS text: members are compared on the 15 key bits after byte d
        // packed beside their index (one LDS word per member instead of an
        // 8-byte key gathered from the text); only equal prefixes re-read the
        // full keys.  Every element's word, sub-bucket byte and bounds are
        // loaded first (all in flight), then the members four at a time.
        auto elem_state = [&](int e, uint32_t& w, uint32_t& bm) {
            const uint32_t p = (uint32_t)(e * 64 + lane);
            w = p < seg.len ? L.idx[p] : 0u;
            uint32_t pc = (w & 0x1ffffu) + d;
            if (pc >= (uint32_t)n) pc %= (uint32_t)n;
            const uint32_t c = p < seg.len ? (uint32_t)T[pc] : 0u;
            const uint32_t b0 = L.base[c], m = L.base[c + 1] - b0;
            bm = p < seg.len && m <= (uint32_t)kSub ? b0 | (m << 9) : 0u;
        };
        uint32_t iw[E], sb[E];  // word; b0 | m << 9 (m = 0: not a small sub-bucket of this segment)
#if BZ2MI_CNT_INTERLEAVE
        // every element's state (kept from the scatter: the elements are
        // taken in their original order, not by position), then the member
        // loops of all E elements interleaved: trip q reads member q of each
        // element's sub-bucket (E independent LDS reads in flight per trip,
        // trips = the largest sub-bucket instead of the sum over the elements)
#pragma unroll
        for (int e = 0; e < E; ++e) {
            iw[e] = own_w[e];
            sb[e] = own_sb[e];
        }
        // per element: lt | le << 16 (counts < 512), and one tie bit each
        uint32_t cnt[E], ties = 0, omax = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t mm = (sb[e] >> 9) & 63u;
            cnt[e] = mm ? 1u << 16 : 0u;
            omax = max(omax, mm ? mm - 1u : 0u);
        }
        for (uint32_t q = 0; q < omax; ++q) {
            uint32_t pq[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint32_t b0 = sb[e] & 511u, mm = (sb[e] >> 9) & 63u;
                const uint32_t self = sb[e] >> 20;
                pq[e] = L.idx[q + 1u < mm ? b0 + q + (q >= self ? 1u : 0u) : b0] >> 17;
            }
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const bool in = q + 1u < ((sb[e] >> 9) & 63u);
                const uint32_t pk = iw[e] >> 17;
                cnt[e] += (in & (pq[e] < pk) ? 1u : 0u) + (in & (pq[e] <= pk) ? 1u << 16 : 0u);
                ties |= (in & (pq[e] == pk) ? 1u : 0u) << e;
            }
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t b0 = sb[e] & 511u, mm = (sb[e] >> 9) & 63u;
            const uint32_t p = b0 + (sb[e] >> 20);  // the element's position
            const bool mine = mm != 0;
            const uint32_t i = iw[e] & 0x1ffffu;
            uint32_t lt = cnt[e] & 0xffffu, le = cnt[e] >> 16, eqlt = 0;
            if ((ties >> e) & 1u) {  // an equal 15-bit prefix: exact counts from the full keys
                const uint64_t k = lds_key(T, n, L, p, d);
                lt = le = 0;
                for (uint32_t q = 0; q < mm; ++q) {
                    const uint64_t kq = lds_key(T, n, L, b0 + q, d);
                    const uint32_t iq = L.idx[b0 + q] & 0x1ffffu;
                    lt += kq < k;
                    le += kq <= k;
                    eqlt += (kq == k) & (iq < i);
                }
            }
            const uint32_t fin = seg.start + b0 + lt + eqlt;
            if (mine) {
                if (s.sa) s.sa[fin] = i;
                bwt[fin] = bwt_byte(T, n, i);
                if (i == 0) *orig = fin;
            }
            sink.push_agg(mine && le - lt >= 2 && eqlt == 0, Seg{seg.start + b0 + lt, le - lt}, d + 8);
        }
#else
        if constexpr (kCntPrefetch) {
#pragma unroll
            for (int e = 0; e < E; ++e) elem_state(e, iw[e], sb[e]);
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if constexpr (!kCntPrefetch) elem_state(e, iw[e], sb[e]);
            const uint32_t p = (uint32_t)(e * 64 + lane);
            const uint32_t b0 = sb[e] & 511u, mm = sb[e] >> 9;
            const bool mine = mm != 0;
            const uint32_t i = iw[e] & 0x1ffffu, pk = iw[e] >> 17;
            // the other members only (the element itself: le += 1); a
            // singleton sub-bucket takes no trip
            uint32_t lt = 0, le = mine ? 1u : 0u, eqlt = 0;
            bool tie = false;
            const uint32_t self = p - b0, others = mine ? mm - 1u : 0u;
            for (uint32_t q = 0; q < others; q += kCntUnroll) {
                uint32_t pq[kCntUnroll];
#pragma unroll
                for (int j = 0; j < kCntUnroll; ++j) {
                    const uint32_t r = q + (uint32_t)j;
                    pq[j] = L.idx[r < others ? b0 + r + (r >= self ? 1u : 0u) : b0] >> 17;
                }
#pragma unroll
                for (int j = 0; j < kCntUnroll; ++j) {
                    const bool in = q + (uint32_t)j < others;
                    lt += in & (pq[j] < pk);
                    le += in & (pq[j] <= pk);
                    tie |= in & (pq[j] == pk);
                }
            }
            if (tie) {  // an equal 15-bit prefix: exact counts from the full keys
                const uint64_t k = lds_key(T, n, L, p, d);
                lt = le = 0;
                for (uint32_t q = 0; q < mm; ++q) {
                    const uint64_t kq = lds_key(T, n, L, b0 + q, d);
                    const uint32_t iq = L.idx[b0 + q] & 0x1ffffu;
                    lt += kq < k;
                    le += kq <= k;
                    eqlt += (kq == k) & (iq < i);
                }
            }
            const uint32_t fin = seg.start + b0 + lt + eqlt;
            if (mine) {
                if (s.sa) s.sa[fin] = i;
                bwt[fin] = bwt_byte(T, n, i);
                if (i == 0) *orig = fin;
            }
            sink.push_agg(mine && le - lt >= 2 && eqlt == 0, Seg{seg.start + b0 + lt, le - lt}, d + 8);
        }
#endif
    }
    bs_mark(12);
    if (nbig) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t c = (uint32_t)(lane * 4 + j);
            const uint32_t b0 = L.base[c], m = L.base[c + 1] - b0;
            uint64_t big = __ballot(m > (uint32_t)kSub);
            while (big) {
                const int l = __builtin_ctzll(big);
                big &= big - 1;
                wave_sort_lds_any(T, n, s, seg.start, (uint32_t)__shfl((int)b0, l), (uint32_t)__shfl((int)m, l), d,
                                  sink, bwt, orig, L);
            }
        }
    }
    bs_mark(13);
}

template <class BL>
__device__ __forceinline__ void wave_sort_bucket2(const uint8_t* __restrict__ T, int n, Scratch& s, Seg seg, uint32_t d,
                                                  const GroupSink& sink, uint8_t* __restrict__ bwt,
                                                  uint32_t* __restrict__ orig, BL& L,
                                                  const uint32_t (&pre)[kSmall / 64]) {
    if (seg.len <= 384u) wave_sort_bucket2_e<6, BL>(T, n, s, seg, d, sink, bwt, orig, L, pre);
    else if (seg.len <= 448u) wave_sort_bucket2_e<7, BL>(T, n, s, seg, d, sink, bwt, orig, L, pre);
    else wave_sort_bucket2_e<8, BL>(T, n, s, seg, d, sink, bwt, orig, L, pre);
}

// ---- a tie group (<= kTieThread rotations with a common prefix of d
// bytes) on one thread: keys = the next 8 bytes, ranks by counting, ties
// with the rotation index; subgroups go to the sink at depth d+8.
constexpr int kTieThread = 16;

struct TieLds {
    uint64_t key[kTieThread * NT];
    uint32_t idx[kTieThread * NT];
    uint32_t off[NT];  // member offset of each thread's group
    uint32_t gst[NT];  // group start in SA
    uint32_t gdp[NT];  // group depth
    uint32_t tmp[NT / 32];
};

__device__ void thread_rank_ties(const uint8_t* __restrict__ T, int n, uint32_t* __restrict__ sa, Seg seg,
                                 uint32_t d, uint32_t off, const GroupSink& sink, uint8_t* __restrict__ bwt,
                                 uint32_t* __restrict__ orig, const TieLds& L) {
    for (uint32_t a = 0; a < seg.len; ++a) {
        const uint64_t ka = L.key[off + a];
        const uint32_t ia = L.idx[off + a];
        uint32_t lt = 0, le = 0, eqlt = 0;
        for (uint32_t q = 0; q < seg.len; ++q) {
            const uint64_t kq = L.key[off + q];
            lt += kq < ka;
            le += kq <= ka;
            eqlt += (kq == ka) & (L.idx[off + q] < ia);
        }
        const uint32_t fin = seg.start + lt + eqlt;
        sa[fin] = ia;
        bwt[fin] = bwt_byte(T, n, ia);
        if (ia == 0) *orig = fin;
        sink.push_agg(le - lt >= 2 && eqlt == 0, Seg{seg.start + lt, le - lt}, d + 8);
    }
}

// ---- sharded queues: 64 shards (shard = block & 63), each with its own
// counter and capacity, so that the producers of the whole chip do not all
// hit one atomic counter.  Consumers index the concatenation of the shards.
constexpr int kShards = 64;
constexpr uint32_t kXcds = 8;  // MI355X: 8 XCDs, workgroups dealt round-robin (grids are multiples of 8)

template <typename Item>
struct Sharded {
    Item* base;
    uint32_t* counts;  // kShards counters (mask ~0: one per block)
    size_t cap;        // entries per shard
    uint32_t mask = kShards - 1;  // shard of block b = b & mask
    __device__ __forceinline__ uint32_t reserve(uint32_t b, uint32_t k) const {
        return atomicAdd(&counts[b & mask], k);
    }
    __device__ __forceinline__ void put(uint32_t b, uint32_t slot, const Item& it) const {
        base[(size_t)(b & mask) * cap + slot] = it;
    }
};

struct ShardIndex {
    uint32_t pre[kShards + 1];
};

// all threads call; wave 0 builds the prefix table; returns the total
__device__ __forceinline__ uint32_t shard_index_load(const uint32_t* __restrict__ counts, ShardIndex& si) {
    if (threadIdx.x < 64) {
        const uint32_t c = counts[threadIdx.x];
        const uint32_t inc = wave_incl_sum(c);
        si.pre[threadIdx.x + 1] = inc;
        if (threadIdx.x == 0) si.pre[0] = 0;
    }
    __syncthreads();
    return uniform(si.pre[kShards]);
}

// entry offset of the q-th item of the concatenation (q < total)
__device__ __forceinline__ size_t shard_locate(const ShardIndex& si, uint32_t q, size_t cap) {
    uint32_t lo = 0, hi = kShards;  // pre[lo] <= q < pre[hi]
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const uint32_t mid = (lo + hi) >> 1;
        if (si.pre[mid] <= q) lo = mid;
        else hi = mid;
    }
    return (size_t)lo * cap + (q - si.pre[lo]);
}

// Pack the children of a partition (counts in sh.hist, in byte order from
// relative position 0) into batches for the small kernel.  Children of
// > kSmall rotations (partitioned further) and of > kSmall/2 (a batch of
// their own) break runs; inside a run, the children of <= kSmall/2 whose
// run-relative start lies in the same 256-rotation window form one batch
// (so a batch holds < kSmall rotations and never splits a child).  A batch of
// one child is sorted from depth d+1, a batch of several from depth d (byte
// d separates them).  Batches with no child of >= 2 rotations are dropped
// (singletons are final).  Wave 0 packs with wave scans (4 children per
// lane); returns the batch count (sh.bat_*).
// One wave packs `hist`; w0 / w1 are 256-word scratch; returns the batch count.
template <int SMALL = kSmall>
__device__ __forceinline__ uint32_t pack_children_wave(const uint32_t* hist, uint32_t* w0, uint32_t* w1,
                                                       uint32_t* bat_start, uint32_t* bat_len) {
    {
        const int lane = lane_id();
        constexpr uint32_t kHalf = SMALL / 2;
        constexpr int kWin = SMALL == 512 ? 8 : 7;  // log2(kHalf): batch windows
        static_assert((1u << kWin) == kHalf, "window");
        uint32_t m[4], pos[4], sinc[4], brk[4];
        uint32_t tot = 0, stot = 0, btot = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            m[j] = hist[lane * 4 + j];
            pos[j] = tot;
            tot += m[j];
            const bool small = m[j] > 0 && m[j] <= kHalf;
            stot += small ? m[j] : 0u;
            sinc[j] = stot;
            brk[j] = m[j] > kHalf;
            btot += brk[j];
        }
        // child start positions, small-size prefix, breaker count (run id)
        const uint32_t pos_ex = wave_incl_sum(tot) - tot;
        const uint32_t s_ex = wave_incl_sum(stot) - stot;
        const uint32_t b_ex = wave_incl_sum(btot) - btot;
        // S at the last breaker (inclusive): max-scan (S is nondecreasing)
        uint32_t lastb = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (brk[j]) lastb = s_ex + sinc[j];
        const uint32_t base_in = lane_prev(wave_incl_max(lastb), 0u);
        uint32_t key[4], run = b_ex, base = base_in, kmax = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool small = m[j] > 0 && m[j] <= kHalf;
            if (brk[j]) {
                run++;
                base = s_ex + sinc[j];
            }
            const uint32_t P = s_ex + sinc[j] - (small ? m[j] : 0u) - base;  // run-relative start
            key[j] = small ? (run << 14) + (P >> kWin) + 1u : 0u;  // P < 2^20: P >> kWin < 2^14
            kmax = key[j] > kmax ? key[j] : kmax;
        }
        uint32_t prevk = lane_prev(wave_incl_max(kmax), 0u);
        uint32_t st[4], nst = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool mid = m[j] > kHalf && m[j] <= (uint32_t)SMALL;
            st[j] = (key[j] && key[j] != prevk) || mid;
            if (key[j]) prevk = key[j];
            nst += st[j];
        }
        const uint32_t st_ex = wave_incl_sum(nst) - nst;
        const uint32_t nbat = (uint32_t)__builtin_amdgcn_readlane((int)(st_ex + nst), 63);
        // per batch: start, length, children, any child of >= 2
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            w0[lane * 4 + j] = 0;  // length
            w1[lane * 4 + j] = 0;  // children | useful << 16
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t idx = st_ex;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool member = key[j] || (m[j] > kHalf && m[j] <= (uint32_t)SMALL);
            if (st[j]) {
                bat_start[idx] = pos_ex + pos[j];
                idx++;
            }
            if (member) {
                atomicAdd(&w0[idx - 1], m[j]);
                atomicAdd(&w1[idx - 1], 1u | (m[j] >= 2 ? 0x10000u : 0u));
            }
        }
        __builtin_amdgcn_wave_barrier();
        // keep the useful batches (compaction, 4 per lane)
        uint32_t keep[4], nk = 0, bs[4], bl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k = (uint32_t)(lane * 4 + j);
            const uint32_t ch = w1[k];
            keep[j] = k < nbat && (ch >> 16) != 0;
            bs[j] = bat_start[k];
            bl[j] = w0[k] | ((ch & 0xffffu) == 1 ? 0x80000000u : 0u);
            nk += keep[j];
        }
        const uint32_t k_ex = wave_incl_sum(nk) - nk;
        __builtin_amdgcn_wave_barrier();
        uint32_t o = k_ex;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (keep[j]) {
                bat_start[o] = bs[j];
                bat_len[o] = bl[j];
                o++;
            }
        }
        __builtin_amdgcn_wave_barrier();
        return (uint32_t)__builtin_amdgcn_readlane((int)(k_ex + nk), 63);
    }
}

__device__ __forceinline__ uint32_t pack_children(BwtShared& sh) {
    if (threadIdx.x < 64) {
        const uint32_t nb = pack_children_wave(sh.hist, sh.wcnt[0], sh.wcnt[1], sh.bat_start, sh.bat_len);
        if (threadIdx.x == 0) sh.cnt[7] = nb;
    }
    __syncthreads();
    return uniform(sh.cnt[7]);
}

// Partition the large segment `seg` (common prefix of d bytes) of block b by
// byte d with the whole workgroup; children: size 1 is final, runs of small
// ones go to the small queue as batches, larger ones to `large_out` or, at
// the depth limit, to the group sink.  The segment is staged in LDS
// (`stage`, kStage entries) or, when longer, in the global `spill` area.
constexpr int kStage = 2048;

struct LevelLds {
    BwtShared sh;
    ShardIndex si;
    uint32_t stage[kStage];
};

// PHASES builds: per-phase wall-clock sums of partition_segment (thread 0 of
// every workgroup), added to g_bwt_phase[8..13] at the end of the kernel
struct PartTimes {
    unsigned long long acc[6];
};
#ifdef BZ2MI_PHASES
#define PT_MARK(pt, k, last)                          \
    do {                                              \
        if (threadIdx.x == 0) {                       \
            const unsigned long long now_ = wall_clock64(); \
            (pt).acc[k] += now_ - (last);             \
            (last) = now_;                            \
        }                                             \
    } while (0)
#else
#define PT_MARK(pt, k, last) \
    do {                     \
    } while (0)
#endif

template <typename LargeOut>
__device__ void partition_segment(const uint8_t* __restrict__ T, int n, uint32_t b, uint32_t* __restrict__ sa,
                                  Seg seg, uint32_t d, LevelLds& L, uint32_t* __restrict__ spill,
                                  const Sharded<uint64_t>& sq, const LargeOut& large_out, const GroupSink& sink,
                                  uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig, PartTimes& pt) {
    BwtShared& sh = L.sh;
    [[maybe_unused]] unsigned long long last_t = 0;
#ifdef BZ2MI_PHASES
    last_t = wall_clock64();
#endif
    seg.start = uniform(seg.start);
    seg.len = uniform(seg.len);
    const int t = threadIdx.x;
    uint32_t* cp = seg.len <= (uint32_t)kStage ? L.stage : spill;
    sh.hist[t] = 0;
    __syncthreads();
    // staged: rotation index | byte d << 24 (indices < 2^20).  The LDS
    // counters take one atomic per distinct byte of a wave (text is skewed:
    // plain atomics would serialise on the frequent letters).
    // 8 rotations per thread and step: all SA loads, then all byte gathers,
    // are in flight together (one memory latency per step, not per rotation)
    constexpr int U = 8;
    const uint32_t rounds = (seg.len + NT - 1) / NT;
    for (uint32_t r0 = 0; r0 < rounds; r0 += U) {
        uint32_t iv[U], cv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t k = (r0 + j) * NT + t;
            iv[j] = k < seg.len ? sa[seg.start + k] : 0u;
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t k = (r0 + j) * NT + t;
            cv[j] = k < seg.len ? byte_at(T, n, iv[j] + d) : 0u;
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t k = (r0 + j) * NT + t;
            const bool v = k < seg.len;
            if (v) cp[k] = iv[j] | (cv[j] << 24);
            const uint64_t peers = wave_match8(cv[j], v);
            if (v && (peers & __lanemask_lt()) == 0) atomicAdd(&sh.hist[cv[j]], (uint32_t)__popcll(peers));
        }
    }
    __syncthreads();
    PT_MARK(pt, 0, last_t);
    const uint32_t c = sh.hist[t];
    uint32_t total;
    const uint32_t ex = wg_excl_sum<NT>(c, sh.tmp, &total);
    sh.base[t] = ex;
    __syncthreads();
    // stable placement is not needed: later sorts break ties by index
    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t k = r * NT + t;
        const bool v = k < seg.len;
        const uint32_t x = v ? cp[k] : 0u;
        const uint32_t cc = x >> 24;
        const uint64_t peers = wave_match8(cc, v);
        const uint64_t below = peers & __lanemask_lt();
        const int leader = peers ? __builtin_ctzll(peers) : 0;
        uint32_t base = 0;
        if (v && below == 0) base = atomicAdd(&sh.base[cc], (uint32_t)__popcll(peers));
        base = (uint32_t)__shfl((int)base, leader);
        if (v) sa[seg.start + base + (uint32_t)__popcll(below)] = x & 0xffffffu;
    }
    PT_MARK(pt, 1, last_t);
    const uint32_t nbat = pack_children(sh);
    PT_MARK(pt, 2, last_t);
    // large children: one reservation per workgroup
    const bool deep = c > (uint32_t)kSmall && d + 1 >= (uint32_t)kMaxDepth;
    const bool large = c > (uint32_t)kSmall && !deep;
    uint32_t nl;
    const uint32_t rl = wg_excl_sum<NT>(large ? 1u : 0u, sh.tmp, &nl);
    if (t == 0) {
        sh.bcast[1] = nbat ? sq.reserve(b, nbat) : 0u;
        sh.bcast[2] = nl ? large_out.reserve(b, nl) : 0u;
    }
    __syncthreads();  // also orders the SA scatter before the final reads
    PT_MARK(pt, 3, last_t);
    if (c == 1) {
        const uint32_t i = sa[seg.start + ex];
        bwt[seg.start + ex] = bwt_byte(T, n, i);
        if (i == 0) *orig = seg.start + ex;
    } else if (large) {
        large_out.put(b, sh.bcast[2] + rl, BwtItem{b, seg.start + ex, c, d + 1});
    } else if (deep) {
        sink.push(Seg{seg.start + ex, c});
    }
    if ((uint32_t)t < nbat) {
        const uint32_t bl = sh.bat_len[t];
        const uint32_t one = bl >> 31;
        sq.put(b, sh.bcast[1] + t, sq_pack(b, seg.start + sh.bat_start[t], bl & 0x7fffffffu, d + one));
    }
    __syncthreads();
    PT_MARK(pt, 4, last_t);
}

// next-level queue (global, all blocks) or the workgroup's own list
struct GlobalLarge {
    Sharded<BwtItem> q;
    __device__ uint32_t reserve(uint32_t b, uint32_t k) const { return q.reserve(b, k); }
    __device__ void put(uint32_t b, uint32_t slot, BwtItem it) const { q.put(b, slot, it); }
};
struct LocalLarge {
    Seg* q;
    uint32_t* count;  // LDS
    __device__ uint32_t reserve(uint32_t, uint32_t k) const { return atomicAdd(count, k); }
    __device__ void put(uint32_t, uint32_t slot, BwtItem it) const { q[slot] = Seg{it.start, it.len}; }
};


// Wave-level partition (levels before the last): one wave per segment, its
// own LDS counters and stage, no workgroup barriers, so a workgroup works on
// NW segments at once.  Segments longer than kWStage stage in `spill` (a
// per-rotation array parallel to SA: segments never overlap).
constexpr int kWStage = 1280;

struct WaveLvl {
    uint32_t hist[256];
    uint32_t base[256];
    uint32_t bat_start[256];
    uint32_t bat_len[256];
    uint32_t stage[kWStage];  // pack scratch after the scatter
};

struct WLevelLds {
    ShardIndex si;
    WaveLvl w[NW];
};

__device__ __forceinline__ void wave_sync_mem() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

__device__ void partition_segment_wave(const uint8_t* __restrict__ T, int n, uint32_t b, uint32_t* __restrict__ sa,
                                       Seg seg, uint32_t d, WaveLvl& W, uint32_t* __restrict__ spill,
                                       const Sharded<uint64_t>& sq, const Sharded<BwtItem>& lq,
                                       const GroupSink& sink, uint8_t* __restrict__ bwt, uint32_t* __restrict__ orig) {
    const int lane = lane_id();
    seg.start = uniform(seg.start);
    seg.len = uniform(seg.len);
    uint32_t* cp = seg.len <= (uint32_t)kWStage ? W.stage : spill + seg.start;
#pragma unroll
    for (int j = 0; j < 4; ++j) W.hist[lane * 4 + j] = 0;
    __builtin_amdgcn_wave_barrier();
    constexpr int U = 8;
    const uint32_t rounds = (seg.len + 63) / 64;
    for (uint32_t r0 = 0; r0 < rounds; r0 += U) {
        uint32_t iv[U], cv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t k = (r0 + j) * 64 + lane;
            iv[j] = k < seg.len ? sa[seg.start + k] : 0u;
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t k = (r0 + j) * 64 + lane;
            cv[j] = k < seg.len ? byte_at(T, n, iv[j] + d) : 0u;
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t k = (r0 + j) * 64 + lane;
            const bool v = k < seg.len;
            if (v) cp[k] = iv[j] | (cv[j] << 24);
            const uint64_t peers = wave_match8(cv[j], v);
            if (v && (peers & __lanemask_lt()) == 0) atomicAdd(&W.hist[cv[j]], (uint32_t)__popcll(peers));
        }
    }
    wave_sync_mem();
    // children: bytes 4*lane .. 4*lane+3
    uint32_t c[4], ex[4], tot = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        c[j] = W.hist[lane * 4 + j];
        ex[j] = tot;
        tot += c[j];
    }
    const uint32_t lex = wave_incl_sum(tot) - tot;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ex[j] += lex;
        W.base[lane * 4 + j] = ex[j];
    }
    __builtin_amdgcn_wave_barrier();
    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t k = r * 64 + lane;
        const bool v = k < seg.len;
        const uint32_t x = v ? cp[k] : 0u;
        const uint32_t cc = x >> 24;
        const uint64_t peers = wave_match8(cc, v);
        const uint64_t below = peers & __lanemask_lt();
        const int leader = peers ? __builtin_ctzll(peers) : 0;
        uint32_t base = 0;
        if (v && below == 0) base = atomicAdd(&W.base[cc], (uint32_t)__popcll(peers));
        base = (uint32_t)__shfl((int)base, leader);
        if (v) sa[seg.start + base + (uint32_t)__popcll(below)] = x & 0xffffffu;
    }
    wave_sync_mem();  // stage reads done (pack scratch), SA scatter visible to the final reads
    const uint32_t nbat = pack_children_wave(W.hist, W.stage, W.stage + 256, W.bat_start, W.bat_len);
    bool large[4], deep[4];
    uint32_t nl = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        deep[j] = c[j] > (uint32_t)kSmall && d + 1 >= (uint32_t)kMaxDepth;
        large[j] = c[j] > (uint32_t)kSmall && !deep[j];
        nl += large[j];
    }
    const uint32_t nl_ex = wave_incl_sum(nl) - nl;
    const uint32_t nl_tot = (uint32_t)__builtin_amdgcn_readlane((int)(nl_ex + nl), 63);
    uint32_t rs = 0, rl = 0;
    if (lane == 0) {
        rs = nbat ? sq.reserve(b, nbat) : 0u;
        rl = nl_tot ? lq.reserve(b, nl_tot) : 0u;
    }
    rs = uniform(rs);
    rl = uniform(rl) + nl_ex;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (c[j] == 1) {
            const uint32_t i = sa[seg.start + ex[j]];
            bwt[seg.start + ex[j]] = bwt_byte(T, n, i);
            if (i == 0) *orig = seg.start + ex[j];
        } else if (large[j]) {
            lq.put(b, rl++, BwtItem{b, seg.start + ex[j], c[j], d + 1});
        } else if (deep[j]) {
            sink.push(Seg{seg.start + ex[j], c[j]});
        }
    }
    for (uint32_t k = lane; k < nbat; k += 64) {
        const uint32_t bl = W.bat_len[k];
        sq.put(b, rs + k, sq_pack(b, seg.start + W.bat_start[k], bl & 0x7fffffffu, d + (bl >> 31)));
    }
    __builtin_amdgcn_wave_barrier();
}

}  // namespace

// ---- kernel 1: per block, counting sort of the rotations by their first
// byte.  Runs of small buckets go to the small queue as batches (all
// blocks), larger buckets to the level-1 queue of the partition kernel.
__global__ __launch_bounds__(256) void bwt_bucket_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                         const uint32_t* __restrict__ lens, int nblocks,
                                                         uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                         uint32_t* __restrict__ orig_out, uint64_t* __restrict__ squeue,
                                                         uint32_t* __restrict__ scount, size_t scap,
                                                         BwtItem* __restrict__ lq, uint32_t* __restrict__ lcount,
                                                         size_t lcap, uint32_t* __restrict__ present_out,
                                                         uint64_t* __restrict__ bq, uint32_t* __restrict__ bq_count,
                                                         size_t bq_cap) {
    __shared__ BwtShared sh;
    __shared__ uint32_t stage[NT * 16], th[256], ts[256];
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    const int t = threadIdx.x;
    const int n = (int)uniform(lens[b]);
    const uint8_t* T = blocks + (size_t)b * stride;
    uint8_t* out = bwt_out + (size_t)b * stride;
    if (n <= 1) {
        if (t == 0) {
            if (n == 1) out[0] = T[0];
            orig_out[b] = 0;
            if (bq) bq_count[b] = 0;  // no mid-size buckets: the big-bucket kernel sees an empty list
        }
        if (t < 8) present_out[(size_t)b * 8 + t] = (n == 1 && (T[0] >> 5) == t) ? 1u << (T[0] & 31) : 0u;
        return;
    }
    uint32_t* sa = sa_all + (size_t)b * stride;
    uint32_t c, ex;
    count_sort_first(T, n, sa, sh, &c, &ex, stage, th, ts);
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
    const Sharded<uint64_t> sq{squeue, scount, scap};
    const Sharded<BwtItem> lqs{lq, lcount, lcap};
    const uint32_t nbat = pack_children(sh);
    // buckets of kSmall < c <= kBigBucket: one workgroup each (bwt_bigbucket_kernel)
    const bool mid = bq && c > (uint32_t)kSmall && c <= (uint32_t)kBigBucket;
    const bool large = c > (uint32_t)kSmall && !mid;
    uint32_t nl, nm;
    const uint32_t rl = wg_excl_sum<NT>(large ? 1u : 0u, sh.tmp, &nl);
    const uint32_t rm = wg_excl_sum<NT>(mid ? 1u : 0u, sh.tmp, &nm);
    if (t == 0) {
        sh.bcast[0] = nbat ? sq.reserve((uint32_t)b, nbat) : 0u;
        sh.bcast[1] = nl ? lqs.reserve((uint32_t)b, nl) : 0u;
        if (bq) bq_count[b] = nm;
    }
    __syncthreads();
    if ((uint32_t)t < nbat) {
        const uint32_t bl = sh.bat_len[t];
        sq.put((uint32_t)b, sh.bcast[0] + t, sq_pack((uint32_t)b, sh.bat_start[t], bl & 0x7fffffffu, bl >> 31));
    }
    if (large) lqs.put((uint32_t)b, sh.bcast[1] + rl, BwtItem{(uint32_t)b, ex, c, 1});
    if (mid) bq[(size_t)b * bq_cap + rm] = ((uint64_t)ex << 32) | c;
}

// ---- kernel 1b (blocks beyond the LDS text): one workgroup per first-byte
// bucket of kSmall < c <= kBigBucket rotations.  Every rotation's 8 bytes at
// depth 1 and its BWT byte are gathered once into LDS, counting-sorted by the
// first of them, and each sub-bucket ranked in LDS (by counting when small, a
// wave sort otherwise); ties go to the tie list at depth 9.  Replaces the
// depth-1 partition (a gather, an SA round trip) and the small sorts of its
// batches (a second gather) for these buckets -- a random 900 KB block's
// first-byte buckets are ~3,500 rotations.
struct BigLds {
    static constexpr bool kKeys = true;
    uint64_t key[kBigBucket];
    uint32_t idx[kBigBucket];  // rotation index | BWT byte << 24
    uint32_t base[257];
    uint32_t tmp[16];
};
// (BZ2MI_BIG_XCD, kernels.hpp: the big-bucket grid dealt to the XCDs by block;
// A/B -DBZ2MI_BIG_XCD=0 = the block-major 2-D grid)
// threads per big-bucket workgroup (A/B: -DBZ2MI_BIG_NT=256)
#ifndef BZ2MI_BIG_NT
#define BZ2MI_BIG_NT 512
#endif
constexpr int kBigNT = BZ2MI_BIG_NT;

__global__ __launch_bounds__(kBigNT) void bwt_bigbucket_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                            const uint32_t* __restrict__ lens,
                                                            uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                            uint32_t* __restrict__ orig_out,
                                                            const uint64_t* __restrict__ bq,
                                                            const uint32_t* __restrict__ bq_count, size_t bq_cap,
                                                            uint64_t* __restrict__ tl, uint32_t* __restrict__ tcount,
                                                            size_t tcap, BwtItem* __restrict__ lq,
                                                            uint32_t* __restrict__ lcount, size_t lcap, int nblocks) {
    __shared__ BigLds L;
#if BZ2MI_BIG_XCD
    // 1-D grid of 8 x 256 x ceil(blocks / 8): the dispatcher deals workgroup
    // w to XCD w mod 8, so XCD x takes the blocks b = x (mod 8), the 256
    // buckets of one block after another -- a block's text is fetched into
    // one XCD's L2 once and its few concurrent blocks stay there
    const uint32_t xcd = blockIdx.x & 7u, sl = blockIdx.x >> 3;
    const uint32_t b = (sl >> 8) * 8u + xcd, bk = sl & 255u;
    if (b >= (uint32_t)nblocks) return;
#else
    // grid (256, blocks): consecutive workgroups share a block, so the
    // concurrent ones gather from a few blocks' text (L2-resident), not all
    const uint32_t b = blockIdx.y, bk = blockIdx.x;
    (void)nblocks;
#endif
    if (bk >= bq_count[b]) return;
    const uint64_t e = bq[(size_t)b * bq_cap + bk];
    const uint32_t start = (uint32_t)(e >> 32), len = (uint32_t)e;
    const int n = (int)lens[b];
    const uint8_t* T = blocks + (size_t)b * stride;
    uint32_t* sa = sa_all + (size_t)b * stride;
    uint8_t* bw = bwt_out + (size_t)b * stride;
    uint32_t* orig = orig_out + b;
    const int t = threadIdx.x;
    constexpr int PER = kBigBucket / kBigNT;
    if (t < 256) L.base[t] = 0;
    __syncthreads();
    uint64_t key[PER];
    uint32_t ii[PER], slot[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t g = (uint32_t)(j * kBigNT + t);
        ii[j] = g < len ? sa[start + g] : 0u;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t g = (uint32_t)(j * kBigNT + t);
        key[j] = 0;
        if (g < len) {
            const uint32_t i = ii[j];
            key[j] = load8(T, n, i + 1 == (uint32_t)n ? 0u : i + 1);
            ii[j] = i | ((uint32_t)bwt_byte(T, n, i) << 24);
        }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j)
        if ((uint32_t)(j * kBigNT + t) < len) slot[j] = atomicAdd(&L.base[key[j] >> 56], 1u);
    __syncthreads();
    {
        uint32_t tot;
        const uint32_t ex = wg_excl_sum<kBigNT>(t < 256 ? L.base[t] : 0u, L.tmp, &tot);
        __syncthreads();
        if (t < 256) L.base[t] = ex;
        if (t == 0) L.base[256] = len;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if ((uint32_t)(j * kBigNT + t) < len) {
            const uint32_t pos = L.base[key[j] >> 56] + slot[j];
            L.key[pos] = key[j];
            L.idx[pos] = ii[j];
        }
    }
    __syncthreads();
    const GroupSink sink{nullptr, nullptr, 0, nullptr, nullptr, b, tl + (size_t)b * tcap, tcount + b};
    // small sub-buckets: ranks by counting
    for (int j = 0; j < PER; ++j) {
        const uint32_t p = (uint32_t)(j * kBigNT + t);
        const bool inseg = p < len;
        const uint64_t k = inseg ? L.key[p] : 0ull;
        const uint32_t w = inseg ? L.idx[p] : 0u;
        const uint32_t c = (uint32_t)(k >> 56);
        const uint32_t b0 = L.base[c], m = inseg ? L.base[c + 1] - b0 : 0u;
        const bool mine = inseg && m <= (uint32_t)kSub;
        const uint32_t i = w & 0xffffffu;
        uint32_t lt = 0, le = 0, eqlt = 0;
        for (uint32_t q = 0; q < (mine ? m : 0u); ++q) {
            const uint64_t kq = L.key[b0 + q];
            const uint32_t iq = L.idx[b0 + q] & 0xffffffu;
            lt += kq < k;
            le += kq <= k;
            eqlt += (kq == k) & (iq < i);
        }
        const uint32_t fin = start + b0 + lt + eqlt;
        if (mine) {
            sa[fin] = i;
            bw[fin] = (uint8_t)(w >> 24);
            if (i == 0) *orig = fin;
        }
        sink.push_agg(mine && le - lt >= 2 && eqlt == 0, Seg{start + b0 + lt, le - lt}, 9);
    }
    // larger sub-buckets: a wave sort each (wave w: sub-buckets 64w..64w+63);
    // beyond kSmall the level queue at depth 2
    const int lane = lane_id();
    if (wave_id() >= 4) return;  // (waves 0-3 take the 256 sub-buckets)
    const uint32_t c = (uint32_t)(wave_id() * 64 + lane);
    const uint32_t b0 = L.base[c], m = L.base[c + 1] - b0;
    Scratch s{};
    s.sa = sa;
    uint64_t big = __ballot(m > (uint32_t)kSub);
    while (big) {
        const int l = __builtin_ctzll(big);
        big &= big - 1;
        const uint32_t lb0 = uniform((uint32_t)__shfl((int)b0, l)), lm = uniform((uint32_t)__shfl((int)m, l));
        if (lm <= (uint32_t)kSmall) {
            wave_sort_lds_any(T, n, s, start, lb0, lm, 1u, sink, bw, orig, L);
        } else {
            for (uint32_t q = (uint32_t)lane; q < lm; q += 64) sa[start + lb0 + q] = L.idx[lb0 + q] & 0xffffffu;
            if (lane == 0) {
                const Sharded<BwtItem> lqs{lq, lcount, lcap};
                lqs.put(b, lqs.reserve(b, 1u), BwtItem{b, start + lb0, lm, 2});
            }
        }
    }
}

// ---- kernel 1' (blocks of <= kBwtLdsText bytes, replaces kernel 1 and the
// small kernel's share of its batches): the block's text is copied into LDS
// once (16-byte loads, the first-byte histogram on the way), the first-byte
// counting sort is staged per 8192-rotation tile as in count_sort_first, and
// then the workgroup's 16 waves sort the block's small batches themselves --
// every 8-byte key and BWT byte is an LDS read instead of a gather from HBM
// (the small kernel's text gathers missed L2 ~16x: 24 GB fetched per GiB).
// Large buckets go to the level-1 queue as before.
constexpr int FT = 1024;
constexpr int FW = FT / 64;

// Text-like blocks (at least half of the rotations in first-byte buckets of
// more than kSmall) are deferred by mode 0 to bwt_text_kernel (redo[b] = 1),
// which hands back the ones it cannot finish (redo[b] = 2: periodic blocks, a
// full work queue or pair list) to mode 1.  Random-like blocks (buckets of
// ~n/256) stay on this path.
constexpr int kTextMinN = 4096;   // smaller blocks stay on this path

// Pair path of bwt_block_kernel: up to kPair of a block's largest first-byte
// buckets (> kSmall rotations) are split by their second byte in the same
// pass (the level-1 partition, with the text in LDS instead of gathered from
// HBM by the level kernel).
constexpr int kPair = 16;
static_assert(kPair <= FW, "one pair slot per wave");

struct BlockLds {
    uint4 text[kBwtLdsText / 16];
    union {
        uint32_t stage[FT * 8 + kPair * 256];  // the tile stage, then the pair cursors
        Bucket3Lds w[FW];
    } u;
    BwtShared sh;
    uint32_t th[256], ts[256], tmp[FW];
    uint32_t pbyte[kPair];   // pair slot -> first byte
    uint8_t pslot[256];      // first byte -> pair slot (0xff: not a pair bucket)
};

__global__ __launch_bounds__(FT) void bwt_block_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                       const uint32_t* __restrict__ lens, int nblocks,
                                                       uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                       uint32_t* __restrict__ orig_out, BwtItem* __restrict__ lq,
                                                       uint32_t* __restrict__ lcount, size_t lcap,
                                                       uint32_t* __restrict__ present_out, uint64_t* __restrict__ tl,
                                                       uint32_t* __restrict__ tcount, size_t tcap,
                                                       uint32_t* __restrict__ redo, int mode,
                                                       uint64_t* __restrict__ squeue, uint32_t* __restrict__ scount,
                                                       size_t scap) {
    __shared__ BlockLds L;
    BwtShared& sh = L.sh;
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    // mode 1: only the blocks the text kernel handed back
    if (mode == 1 && redo[b] < 2u) return;
    const int t = threadIdx.x;
    const int n = (int)uniform(lens[b]);
    const uint8_t* T = blocks + (size_t)b * stride;
    uint8_t* out = bwt_out + (size_t)b * stride;
    if (n <= 1) {
        if (t == 0) {
            if (n == 1) out[0] = T[0];
            orig_out[b] = 0;
        }
        if (t < 8) present_out[(size_t)b * 8 + t] = (n == 1 && (T[0] >> 5) == t) ? 1u << (T[0] & 31) : 0u;
        return;
    }
    uint32_t* sa = sa_all + (size_t)b * stride;
    const uint8_t* Tl = reinterpret_cast<const uint8_t*>(L.text);
#ifdef BZ2MI_PHASES
    unsigned long long blk_t = wall_clock64();
    auto blk_mark = [&](int k) {
        __syncthreads();
        if (t == 0) {
            const unsigned long long now = wall_clock64();
            atomicAdd(&g_blk_phase[k], now - blk_t);
            blk_t = now;
        }
    };
#else
    auto blk_mark = [](int) {};
#endif
    // ---- text -> LDS (whole 16-byte chunks: the block buffer is padded),
    // first-byte histogram
    if (t < 256) sh.hist[t] = 0;
    __syncthreads();
    {
        const int n16 = (n + 15) >> 4;
        const uint4* T4 = reinterpret_cast<const uint4*>(T);
        for (int v = t; v < n16; v += FT) {
            const uint4 w = T4[v];
            L.text[v] = w;
            const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
            const int lim = n - v * 16;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k < lim) atomicAdd(&sh.hist[(ww[k >> 2] >> ((k & 3) * 8)) & 255u], 1u);
        }
    }
    __syncthreads();
    const uint32_t c = t < 256 ? sh.hist[t] : 0u;
    uint32_t total;
    const uint32_t ex = wg_excl_sum<FT>(c, L.tmp, &total);
    if (t < 256) sh.base[t] = ex;
    if (mode == 0) {
        // text-like blocks: the symbol map, then bwt_text_kernel
        uint32_t bigsum;
        (void)wg_excl_sum<FT>(c > (uint32_t)kSmall ? c : 0u, L.tmp, &bigsum);
        if (2 * bigsum >= (uint32_t)n && n >= kTextMinN) {
            if (t < 256) {
                const uint64_t m = __ballot(c != 0);
                if (lane_id() == 0) {
                    present_out[(size_t)b * 8 + 2 * wave_id()] = (uint32_t)m;
                    present_out[(size_t)b * 8 + 2 * wave_id() + 1] = (uint32_t)(m >> 32);
                }
            }
            if (t == 0) redo[b] = 1u;
            return;
        }
    }
    blk_mark(0);
    // ---- pair path: the kPair largest buckets of > kSmall rotations (ties by
    // byte) get a histogram of their second bytes; wave w < npair turns pair
    // slot w's counts into child cursors (counts and starts kept in registers)
    uint32_t* const pair = L.u.stage + FT * 8;
    const bool big = t < 256 && c > (uint32_t)kSmall;
    const int npair = min(__syncthreads_count(big), kPair);
    uint32_t pcnt[4] = {0, 0, 0, 0}, pst[4] = {0, 0, 0, 0};
    if (npair) {
        if (t < 256) {
            uint32_t rk = 0xffu;
            if (big) {
                uint32_t above = 0;
                for (int u = 0; u < 256; ++u) {
                    const uint32_t cu = sh.hist[u];
                    above += (cu > c || (cu == c && u < t)) ? 1u : 0u;
                }
                if (above < (uint32_t)npair) {
                    rk = above;
                    L.pbyte[above] = (uint32_t)t;
                }
            }
            L.pslot[t] = (uint8_t)rk;
        }
        for (int k = t; k < kPair * 256; k += FT) pair[k] = 0;
        __syncthreads();
        for (int i0 = t * 8; i0 < n; i0 += FT * 8) {
            const uint2 wv = reinterpret_cast<const uint2*>(Tl)[i0 >> 3];
            const uint32_t nx = Tl[i0 + 8 < n ? i0 + 8 : 0];
            uint32_t bv[9];
#pragma unroll
            for (int k = 0; k < 8; ++k) bv[k] = ((k < 4 ? wv.x : wv.y) >> ((k & 3) * 8)) & 255u;
            bv[8] = nx;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = i0 + k;
                if (i < n) {
                    const uint32_t ps = L.pslot[bv[k]];
                    if (ps != 0xffu) {
                        const uint32_t b1 = i + 1 < n ? bv[k + 1] : (uint32_t)Tl[0];
                        atomicAdd(&pair[ps * 256u + b1], 1u);
                    }
                }
            }
        }
        __syncthreads();
        const int w = wave_id(), lane = lane_id();
        if (w < npair) {
            uint32_t tot = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pcnt[j] = pair[w * 256 + lane * 4 + j];
                pst[j] = tot;
                tot += pcnt[j];
            }
            const uint32_t b0 = sh.base[L.pbyte[w]] + wave_incl_sum(tot) - tot;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pst[j] += b0;
                pair[w * 256 + lane * 4 + j] = pst[j];
            }
        }
        __syncthreads();
    } else if (t < 256) {
        L.pslot[t] = 0xffu;
    }
    blk_mark(1);
    // ---- first-byte scatter, one 8192-rotation tile at a time (8 per thread);
    // rotations of pair buckets go to their (first, second byte) child
    for (int tile0 = 0; tile0 < n; tile0 += FT * 8) {
        if (t < 256) L.th[t] = 0;
        __syncthreads();
        const int i0 = tile0 + t * 8;
        uint32_t bv[8], rk[8];
        {
            const uint2 w = i0 < n ? reinterpret_cast<const uint2*>(Tl)[i0 >> 3] : make_uint2(0u, 0u);
#pragma unroll
            for (int k = 0; k < 8; ++k) bv[k] = ((k < 4 ? w.x : w.y) >> ((k & 3) * 8)) & 255u;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) rk[k] = i0 + k < n ? atomicAdd(&L.th[bv[k]], 1u) : 0u;
        __syncthreads();
        uint32_t tn;
        const uint32_t tsv = wg_excl_sum<FT>(t < 256 ? L.th[t] : 0u, L.tmp, &tn);
        if (t < 256) L.ts[t] = tsv;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (i0 + k < n) L.u.stage[L.ts[bv[k]] + rk[k]] = (uint32_t)(i0 + k) | (bv[k] << 24);
        __syncthreads();
        if (npair == 0) {
            for (uint32_t j = t; j < tn; j += FT) {
                const uint32_t v = L.u.stage[j], b8 = v >> 24;
                sa[sh.base[b8] + (j - L.ts[b8])] = v & 0xffffffu;
            }
        } else {
            for (uint32_t j = t; j < tn; j += FT) {
                const uint32_t v = L.u.stage[j], b8 = v >> 24, i = v & 0xffffffu;
                const uint32_t ps = L.pslot[b8];
                if (ps == 0xffu) {
                    sa[sh.base[b8] + (j - L.ts[b8])] = i;
                } else {
                    const uint32_t b1 = Tl[i + 1 < (uint32_t)n ? i + 1 : 0u];
                    sa[atomicAdd(&pair[ps * 256u + b1], 1u)] = i;
                }
            }
        }
        __syncthreads();
        if (t < 256) sh.base[t] += L.th[t];
    }
    __syncthreads();
    blk_mark(2);
    if (t < 256) {  // symbols in use (the MTF symbol map): bit t of the 256-bit set
        const uint64_t m = __ballot(c != 0);
        if (lane_id() == 0) {
            present_out[(size_t)b * 8 + 2 * wave_id()] = (uint32_t)m;
            present_out[(size_t)b * 8 + 2 * wave_id() + 1] = (uint32_t)(m >> 32);
        }
        if (c == 1) {
            const uint32_t i = sa[ex];
            out[ex] = bwt_byte(Tl, n, i);
            if (i == 0) orig_out[b] = ex;
        }
    }
    const Sharded<BwtItem> lqs{lq, lcount, lcap};
    const uint32_t nbat = pack_children(sh);
    const bool large = big && L.pslot[t] == 0xffu;
    uint32_t nl;
    const uint32_t rl = wg_excl_sum<FT>(large ? 1u : 0u, L.tmp, &nl);
    if (t == 0) sh.bcast[1] = nl ? lqs.reserve((uint32_t)b, nl) : 0u;
    __syncthreads();
    if (large) lqs.put((uint32_t)b, sh.bcast[1] + rl, BwtItem{(uint32_t)b, ex, c, 1});
    if (npair) {
        // the pair buckets' children, as a level-1 partition leaves them: size
        // 1 final, runs of small ones batched for bwt_block_small_kernel (the
        // block's list), larger ones to the level queue at depth 2.  Eight
        // waves at a time (4 KB of packing scratch each).
        const Sharded<uint64_t> sq{squeue, scount, scap, 0xffffffffu};
        const int w = wave_id(), lane = lane_id();
        for (int r0 = 0; r0 < npair; r0 += 8) {
            if (w >= r0 && w < r0 + 8 && w < npair) {
                uint32_t* row = pair + w * 256;
                uint32_t* scr = L.u.stage + (w - r0) * 1024;  // the tile stage is free now
#pragma unroll
                for (int j = 0; j < 4; ++j) row[lane * 4 + j] = pcnt[j];
                __builtin_amdgcn_wave_barrier();
                const uint32_t nb2 = pack_children_wave(row, scr, scr + 256, scr + 512, scr + 768);
                uint32_t nlc = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) nlc += pcnt[j] > (uint32_t)kSmall;
                const uint32_t lex = wave_incl_sum(nlc) - nlc;
                const uint32_t ltot = (uint32_t)__builtin_amdgcn_readlane((int)(lex + nlc), 63);
                uint32_t rs = 0, rlq = 0;
                if (lane == 0) {
                    rs = nb2 ? sq.reserve((uint32_t)b, nb2) : 0u;
                    rlq = ltot ? lqs.reserve((uint32_t)b, ltot) : 0u;
                }
                rs = uniform(rs);
                rlq = uniform(rlq) + lex;
                // the bucket's start: child 0's start (lane 0, element 0)
                const uint32_t seg0 = (uint32_t)__builtin_amdgcn_readlane((int)pst[0], 0);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (pcnt[j] == 1u) {
                        const uint32_t i = sa[pst[j]];
                        out[pst[j]] = bwt_byte(Tl, n, i);
                        if (i == 0) orig_out[b] = pst[j];
                    } else if (pcnt[j] > (uint32_t)kSmall) {
                        lqs.put((uint32_t)b, rlq++, BwtItem{(uint32_t)b, pst[j], pcnt[j], 2});
                    }
                }
                for (uint32_t k = lane; k < nb2; k += 64) {
                    const uint32_t bl = scr[768 + k];
                    sq.put((uint32_t)b, rs + k, sq_pack((uint32_t)b, seg0 + scr[512 + k], bl & 0x7fffffffu, 1u + (bl >> 31)));
                }
            }
            __syncthreads();
        }
    }
    blk_mark(3);
    // ---- the small batches, one wave each, keys from the LDS text; the next
    // batch's SA entries are loaded while the current one is sorted
    constexpr int E = kSmall / 64;
    const int w = wave_id(), lane = lane_id();
    auto load_batch = [&](uint32_t k, uint32_t (&pre)[E]) {
        const uint32_t st = sh.bat_start[k], len = sh.bat_len[k] & 0x7fffffffu;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t g = (uint32_t)(e * 64 + lane);
            pre[e] = g < len ? sa[st + g] : 0u;
        }
    };
    Scratch s{};
    s.sa = sa;
    const GroupSink sink{nullptr, nullptr, 0, nullptr, nullptr, (uint32_t)b, tl + (size_t)b * tcap, tcount + b};
// (loading the next batch's SA entries during a sort held 8 VGPRs across it:
// without the prefetch the kernel spills less, 8.90 -> 8.74 ms per GiB)
#ifndef BZ2MI_BATCH_PREFETCH
#define BZ2MI_BATCH_PREFETCH 0
#endif
    uint32_t cur[E];
    if (BZ2MI_BATCH_PREFETCH && (uint32_t)w < nbat) load_batch((uint32_t)w, cur);
    for (uint32_t k = (uint32_t)w; k < nbat; k += FW) {
#if BZ2MI_BATCH_PREFETCH
        uint32_t nxt[E];
        if (k + FW < nbat) load_batch(k + FW, nxt);
#else
        load_batch(k, cur);
#endif
        const uint32_t bl = uniform(sh.bat_len[k]);
        const Seg seg{uniform(sh.bat_start[k]), bl & 0x7fffffffu};
        wave_sort_bucket2(Tl, n, s, seg, bl >> 31, sink, out, orig_out + b, L.u.w[w], cur);
#if BZ2MI_BATCH_PREFETCH
#pragma unroll
        for (int e = 0; e < E; ++e) cur[e] = nxt[e];
#endif
    }
#ifdef BZ2MI_PHASES
    blk_mark(4);
    if (t == 0) {
        atomicAdd(&g_blk_phase[8], 1ull);
        atomicAdd(&g_blk_phase[9], (unsigned long long)nbat);
        atomicAdd(&g_blk_phase[10], (unsigned long long)npair);
    }
#endif
}


// ---- kernel 2 (one launch per level, all blocks at once): every large
// segment of the level queue is partitioned by one workgroup.  The last level
// (`last` != 0) keeps partitioning its segment's large children itself, level
// by level, up to kMaxDepth.
__global__ __launch_bounds__(256) void bwt_level_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                        const uint32_t* __restrict__ lens,
                                                        uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                        uint32_t* __restrict__ orig_out, uint8_t* scratch, uint32_t* __restrict__ spill_all,
                                                        size_t scratch_per_slot, int S, const BwtItem* __restrict__ lin,
                                                        const uint32_t* __restrict__ lin_count, BwtItem* __restrict__ lout,
                                                        uint32_t* __restrict__ lout_count, size_t lcap,
                                                        uint64_t* __restrict__ squeue, uint32_t* __restrict__ scount,
                                                        size_t scap, Seg* __restrict__ grp_all,
                                                        uint32_t* __restrict__ ngroups, uint32_t* __restrict__ p2list,
                                                        uint32_t* __restrict__ p2count, int last, uint32_t smask) {
    __shared__ LevelLds L;
    const uint32_t nin = shard_index_load(lin_count, L.si);
    if (nin == 0) return;
    // slot scratch (bwt_level_slot_bytes): the local lists; a segment's spill
    // area is its own range of the block's per-rotation spill (segments of a
    // level, and sub-segments of one, are disjoint ranges of the SA)
    Scratch s{};
    {
        uint8_t* p = scratch + (size_t)blockIdx.x * scratch_per_slot;
        s.large = (Seg*)p;
        p += 8 * ((size_t)S / kSmall + 8);
        s.large2 = (Seg*)p;
    }
    const int t = threadIdx.x;
    const Sharded<uint64_t> sq{squeue, scount, scap, smask};
    PartTimes pt{};
    unsigned long long item_t = 0;
    // XCD-aware: workgroups are dealt to the 8 XCDs round-robin; XCD x takes
    // the x-th eighth of the queue, so the segments (and blocks) one XCD
    // works on at a time are neighbours and stay in its L2
    const uint32_t xcd = blockIdx.x % kXcds, nloc = gridDim.x / kXcds;
    const uint32_t qlo = (uint32_t)((uint64_t)nin * xcd / kXcds), qhi = (uint32_t)((uint64_t)nin * (xcd + 1) / kXcds);
    for (uint32_t q = qlo + blockIdx.x / kXcds; q < qhi; q += nloc) {
#ifdef BZ2MI_PHASES
        item_t = wall_clock64();
#endif
        const BwtItem it = lin[shard_locate(L.si, q, lcap)];
        const uint32_t b = uniform(it.block);
        const int n = (int)uniform(lens[b]);
        const uint8_t* T = blocks + (size_t)b * stride;
        uint32_t* sa = sa_all + (size_t)b * stride;
        uint8_t* bw = bwt_out + (size_t)b * stride;
        const GroupSink sink{grp_all + (size_t)b * bwt_group_stride(stride), &ngroups[b], 0xffffffffu, p2list,
                             p2count, b, nullptr, nullptr};
        uint32_t d = uniform(it.depth);
        uint32_t* spill = spill_all + (size_t)b * stride;
        if (!last) {
            partition_segment(T, n, b, sa, Seg{it.start, it.len}, d, L, spill + it.start, sq,
                              GlobalLarge{Sharded<BwtItem>{lout, lout_count, lcap}}, sink, bw, orig_out + b, pt);
            continue;
        }
        // local levels: s.large / s.large2 ping-pong, counter in L.sh.cnt[3]
        if (t == 0) {
            s.large[0] = Seg{it.start, it.len};
            L.sh.cnt[1] = 1;
        }
        __syncthreads();
        Seg* cur = s.large;
        Seg* nxt = s.large2;
        for (;;) {
            const uint32_t nc = uniform(L.sh.cnt[1]);
            if (nc == 0) break;
            if (t == 0) L.sh.cnt[3] = 0;
            __syncthreads();
            for (uint32_t k = 0; k < nc; ++k)
                partition_segment(T, n, b, sa, cur[k], d, L, spill + cur[k].start, sq, LocalLarge{nxt, &L.sh.cnt[3]}, sink, bw,
                                  orig_out + b, pt);
            if (t == 0) L.sh.cnt[1] = L.sh.cnt[3];
            __syncthreads();
            Seg* tmp = cur;
            cur = nxt;
            nxt = tmp;
            d++;
        }
        __syncthreads();
    }
#ifdef BZ2MI_PHASES
    if (t == 0) {
        for (int k = 0; k < 5; ++k) atomicAdd(&g_bwt_phase[8 + k], pt.acc[k]);
        atomicAdd(&g_bwt_phase[14], 1ull);
    }
#endif
    (void)item_t;
}

// ---- kernel 2w (levels before the last): one wave per large segment of the
// level queue (wave-level partition, NW segments per workgroup at a time).
// XCD split as in bwt_level_kernel.
__global__ __launch_bounds__(256) void bwt_wlevel_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                         const uint32_t* __restrict__ lens,
                                                         uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                         uint32_t* __restrict__ orig_out, uint32_t* __restrict__ spill_all,
                                                         const BwtItem* __restrict__ lin,
                                                         const uint32_t* __restrict__ lin_count,
                                                         BwtItem* __restrict__ lout, uint32_t* __restrict__ lout_count,
                                                         size_t lcap, uint64_t* __restrict__ squeue,
                                                         uint32_t* __restrict__ scount, size_t scap,
                                                         Seg* __restrict__ grp_all, uint32_t* __restrict__ ngroups,
                                                         uint32_t* __restrict__ p2list, uint32_t* __restrict__ p2count,
                                                         uint32_t smask) {
    __shared__ WLevelLds L;
    const uint32_t nin = shard_index_load(lin_count, L.si);
    if (nin == 0) return;
    const Sharded<uint64_t> sq{squeue, scount, scap, smask};
    const Sharded<BwtItem> lq{lout, lout_count, lcap};
    WaveLvl& W = L.w[wave_id()];
    const uint32_t xcd = blockIdx.x % kXcds, nloc = gridDim.x / kXcds;
    const uint32_t qlo = (uint32_t)((uint64_t)nin * xcd / kXcds), qhi = (uint32_t)((uint64_t)nin * (xcd + 1) / kXcds);
    for (uint32_t q = qlo + (blockIdx.x / kXcds) * NW + wave_id(); q < qhi; q += nloc * NW) {
        const BwtItem it = lin[shard_locate(L.si, q, lcap)];
        const uint32_t b = uniform(it.block);
        const int n = (int)uniform(lens[b]);
        const GroupSink sink{grp_all + (size_t)b * bwt_group_stride(stride), &ngroups[b], 0xffffffffu, p2list,
                             p2count, b, nullptr, nullptr};
        partition_segment_wave(blocks + (size_t)b * stride, n, b, sa_all + (size_t)b * stride,
                               Seg{it.start, it.len}, uniform(it.depth), W, spill_all + (size_t)b * stride, sq, lq,
                               sink, bwt_out + (size_t)b * stride, orig_out + b);
    }
}

// ---- kernel 3: one wave per queued batch of small segments (any block, any
// depth): sort, write SA, BWT bytes and origPtr; tie groups go to the
// block's tie list for the tie rounds
__global__ __launch_bounds__(256, 4) void bwt_small_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                        const uint32_t* __restrict__ lens,
                                                        uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                        uint32_t* __restrict__ orig_out,
                                                        const uint64_t* __restrict__ squeue,
                                                        const uint32_t* __restrict__ scount, size_t scap,
                                                        uint64_t* __restrict__ tl, uint32_t* __restrict__ tcount,
                                                        size_t tcap) {
    __shared__ Bucket2Lds lds[NT / 64];
    __shared__ ShardIndex si;
    const uint32_t nq = shard_index_load(scount, si);
    // XCD-aware split of the queue (see bwt_level_kernel)
    const uint32_t xcd = blockIdx.x % kXcds, nwaves = gridDim.x / kXcds * (NT / 64);
    const uint32_t qlo = (uint32_t)((uint64_t)nq * xcd / kXcds), qhi = (uint32_t)((uint64_t)nq * (xcd + 1) / kXcds);
    // software pipeline over the wave's batches: the queue entry two batches
    // ahead and the SA entries (and block length) of the next batch are
    // loaded while the current one is sorted, so a batch waits for one
    // memory round trip (its text gathers) instead of three
    constexpr int E = kSmall / 64;
    const int lane = lane_id();
    auto entry = [&](uint32_t q) -> uint64_t { return q < qhi ? squeue[shard_locate(si, uniform(q), scap)] : 0ull; };
    auto load_batch = [&](uint64_t e, uint32_t (&sa)[E], uint32_t& n) {
        const uint32_t b = uniform((uint32_t)(e >> 42));
        const uint32_t start = uniform((uint32_t)(e >> 22) & 0xfffffu), len = uniform((uint32_t)(e >> 13) & 511u) + 1u;
        n = lens[b];
        const uint32_t* sab = sa_all + (size_t)b * stride + start;
#pragma unroll
        for (int k = 0; k < E; ++k) {
            const uint32_t g = (uint32_t)(k * 64 + lane);
            sa[k] = g < len ? sab[g] : 0u;
        }
    };
    uint32_t q = qlo + blockIdx.x / kXcds * (NT / 64) + wave_id();
    uint64_t ec = entry(q), en = entry(q + nwaves);
    uint32_t sac[E], nc = 0;
    if (q < qhi) load_batch(ec, sac, nc);
    for (; q < qhi; q += nwaves) {
        uint32_t san[E], nn = 0;
        if (q + nwaves < qhi) load_batch(en, san, nn);
        const uint64_t enn = entry(q + 2 * nwaves);
        const uint32_t b = uniform((uint32_t)(ec >> 42));
        const Seg seg{uniform((uint32_t)(ec >> 22) & 0xfffffu), uniform((uint32_t)(ec >> 13) & 511u) + 1u};
        const uint32_t d = uniform((uint32_t)ec & 0x1fffu);
        Scratch s{};
        s.sa = sa_all + (size_t)b * stride;
        const GroupSink sink{nullptr, nullptr, 0, nullptr, nullptr, b, tl + (size_t)b * tcap, tcount + b};
        wave_sort_bucket2(blocks + (size_t)b * stride, (int)uniform(nc), s, seg, d, sink, bwt_out + (size_t)b * stride,
                          orig_out + b, lds[wave_id()], sac);
#pragma unroll
        for (int k = 0; k < E; ++k) sac[k] = san[k];
        nc = nn;
        ec = en;
        en = enn;
    }
}

// ---- kernel 3' (with kernel 1'): the batches the levels queued, per block
// (one list per block), sorted by one 1024-thread workgroup per block with
// the block's text in LDS; blocks with an empty list return at once.
// bwt_block_small_kernel: batches sorted whole from their SA entries in
// registers (wave_sort_pre_text) instead of wave_sort_bucket2's sub-buckets
#ifndef BZ2MI_BWT_PRETEXT
#define BZ2MI_BWT_PRETEXT 1
#endif
constexpr bool kBwtPreText = BZ2MI_BWT_PRETEXT != 0;

struct BlockSmallLds {
    uint4 text[kBwtLdsText / 16];
    Bucket3Lds w[FW];
};

__global__ __launch_bounds__(FT) void bwt_block_small_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                             const uint32_t* __restrict__ lens, int nblocks,
                                                             uint32_t* __restrict__ sa_all,
                                                             uint8_t* __restrict__ bwt_out,
                                                             uint32_t* __restrict__ orig_out,
                                                             const uint64_t* __restrict__ squeue,
                                                             const uint32_t* __restrict__ scount, size_t scap,
                                                             uint64_t* __restrict__ tl, uint32_t* __restrict__ tcount,
                                                             size_t tcap) {
    __shared__ BlockSmallLds L;
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    const uint32_t nq = uniform(scount[b]);
    if (nq == 0) return;
    const int t = threadIdx.x;
    const int n = (int)uniform(lens[b]);
    {
        const int n16 = (n + 15) >> 4;
        const uint4* T4 = reinterpret_cast<const uint4*>(blocks + (size_t)b * stride);
        for (int v = t; v < n16; v += FT) L.text[v] = T4[v];
    }
    __syncthreads();
    const uint8_t* Tl = reinterpret_cast<const uint8_t*>(L.text);
    uint32_t* sa = sa_all + (size_t)b * stride;
    uint8_t* out = bwt_out + (size_t)b * stride;
    const uint64_t* q = squeue + (size_t)b * scap;
    constexpr int E = kSmall / 64;
    const int w = wave_id(), lane = lane_id();
    Scratch s{};
    s.sa = sa;
    const GroupSink sink{nullptr, nullptr, 0, nullptr, nullptr, (uint32_t)b, tl + (size_t)b * tcap, tcount + b};
    auto load_batch = [&](uint64_t e, uint32_t (&pre)[E]) {
        const uint32_t st = uniform((uint32_t)(e >> 22) & 0xfffffu), len = uniform((uint32_t)(e >> 13) & 511u) + 1u;
#pragma unroll
        for (int k = 0; k < E; ++k) {
            const uint32_t g = (uint32_t)(k * 64 + lane);
            pre[k] = g < len ? sa[st + g] : 0u;
        }
    };
    uint32_t cur[E];
    uint64_t ec = (uint32_t)w < nq ? q[w] : 0ull;
    if ((uint32_t)w < nq) load_batch(ec, cur);
    for (uint32_t k = (uint32_t)w; k < nq; k += FW) {
        uint32_t nxt[E];
        const uint64_t en = k + FW < nq ? q[k + FW] : 0ull;
        if (k + FW < nq) load_batch(en, nxt);
        const Seg seg{uniform((uint32_t)(ec >> 22) & 0xfffffu), uniform((uint32_t)(ec >> 13) & 511u) + 1u};
        const uint32_t d = uniform((uint32_t)ec & 0x1fffu);
        if constexpr (kBwtPreText) {
            // the levels' batches are text-like: one sort of the whole batch
            uint32_t* idx = L.w[w].idx;
            uint32_t tt;
            if (seg.len <= 64) tt = wave_sort_pre_text<1>(Tl, n, s, seg.start, seg.len, d, out, orig_out + b, idx, cur);
            else if (seg.len <= 128) tt = wave_sort_pre_text<2>(Tl, n, s, seg.start, seg.len, d, out, orig_out + b, idx, cur);
            else if (seg.len <= 256) tt = wave_sort_pre_text<4>(Tl, n, s, seg.start, seg.len, d, out, orig_out + b, idx, cur);
            else tt = wave_sort_pre_text<8>(Tl, n, s, seg.start, seg.len, d, out, orig_out + b, idx, cur);
            tt = uniform(tt);
            if (tt) lds_ties(Tl, n, s, seg.start, tt, d, sink, out, orig_out + b, idx);
        } else {
            wave_sort_bucket2(Tl, n, s, seg, d, sink, out, orig_out + b, L.w[w], cur);
        }
#pragma unroll
        for (int e = 0; e < E; ++e) cur[e] = nxt[e];
        ec = en;
    }
}

// ---- kernel 1t: text-like blocks (most rotations in first-byte buckets of
// more than kSmall), one 1024-thread workgroup per block with the block's
// text in LDS.  Induced sorting in the manner of bzip2's main sort (Seward's
// "copy" step):
//   * every rotation is scattered into its two-byte bucket (a, b): a counting
//     sort by the first byte, then every first-byte row split by the second
//     byte (one wave per row, largest rows first).  The non-empty pair buckets
//     form a sparse index: a 256-bit mask of second bytes per first byte and
//     the row's entries in a list, so any alphabet (up to 256 bytes, ~2,000
//     non-empty pairs in a 90 KB block of real text) fits;
//   * the first-byte buckets are processed in ascending size; for bucket ss
//     every pair bucket (ss, b) whose b is not yet processed (and (ss, ss)) is
//     sorted -- partitions by the next byte and wave sorts, all keys read from
//     the LDS text, work spread over the 16 waves -- while the pair buckets
//     (ss, b) of processed b are already in order;
//   * then bucket ss is complete, and for every unprocessed x the pair bucket
//     (x, ss) follows for free: the rotations i-1 of the sorted bucket ss with
//     T[i-1] = x, in that order (a stable partition by the preceding byte).
// About half of the rotations of text are placed by the copy step without
// being sorted.  BWT bytes and origPtr are written as positions become final.
// Long repeats: rotations still tied after kTextTieCap bytes (two-rotation
// groups: kTextPairCap) are not sorted further in the sort phase.  Their SA
// entries are flagged (kUnres) and the group goes to a deferred list.  After
// the sort phase, before any copy step, every deferred group is ordered
// (text_resolve_all): a pair (i, j) sharing d bytes has the order of (i + x,
// j + x) for any x <= d, so it is decided at the first x where both rotations
// already have their final positions (sorted rotations: isa), or it links to
// the deferred pair (i + x, j + x) -- the next one of the same repeat; the
// links of a repeat form a chain down to the pair that meets the repeat's end,
// collapsed by pointer jumping.  So a repeat of any length costs a few steps
// per pair.  Blocks it cannot finish (periodic blocks, a group of more than 64
// rotations, a group that waits on itself -- a tandem repeat --, a full work
// queue or pair list) get redo[b] = 2 and go through the general path
// (bwt_block_kernel mode 1).
constexpr int kTextDcap = 512;    // depth at which a partition gives up
constexpr int kTextChain = 32;    // levels a partition goes down with one child before its segment is deferred
#ifndef BZ2MI_TEXT_TIECAP
#define BZ2MI_TEXT_TIECAP 64
#endif
constexpr int kTextTieCap = BZ2MI_TEXT_TIECAP;  // tie depth after which a wave sort defers its tied groups
#ifndef BZ2MI_TEXT_PAIRCAP
#define BZ2MI_TEXT_PAIRCAP 32
#endif
constexpr int kTextPairCap = BZ2MI_TEXT_PAIRCAP;  // depth to which two tied rotations are compared directly
// largest segment the text kernel sorts in one wave (A/B: -DBZ2MI_TEXT_SMALL=512):
// 256 keeps every sort at <= 4 keys per lane, so the kernel's state fits the
// 128 VGPRs of a 1024-thread workgroup; larger segments are partitioned
#ifndef BZ2MI_TEXT_SMALL
#define BZ2MI_TEXT_SMALL 256
#endif
constexpr int kTS = BZ2MI_TEXT_SMALL;
constexpr int kTIB = kTS == 256 ? 8 : 9;  // item-index bits of its sort keys (7 text bytes in the first round, 6 per tie round)
static_assert(kTS == 256 || kTS == 512, "text sort size");
constexpr int kTQ = 512;          // work items per round
constexpr int kCopyR = 4;         // rotations per lane and chunk of a copy step
constexpr int kTW = 768;          // per-wave LDS words
constexpr uint32_t kUnres = 0x80000000u;  // SA entry flag: a member of a deferred group (not yet ordered)
// non-empty (first, second byte) pairs of a text-path block (~2,000 in a 90 KB
// block of real text): counted in the per-wave scratch during the setup, and
// the pair list (uint64 entries) lives in the block's group area, which holds
// stride / 2 of them (more than kPairCap at every level with S >= 20,000)
constexpr int kPairCap = FW * kTW - FW * 256 - 1;  // the copy steps keep the starts in LDS beside 16 x 256 cursors
// copy-processed first-byte buckets (the largest ones); the smaller buckets are
// sorted whole and copied from in one step
#ifndef BZ2MI_TEXT_COPYSTEPS
#define BZ2MI_TEXT_COPYSTEPS 12
#endif
constexpr int kCopySteps = BZ2MI_TEXT_COPYSTEPS;

struct TextLds {
    uint4 text[kBwtLdsText / 16];
    uint32_t w[FW][kTW];              // per-wave scratch
    uint64_t q[2][kTQ];               // work items of this round / the next: depth | len | start
    uint32_t mask[256][8];            // pair index: second bytes present, per first byte
    uint32_t rowoff[256];             // a first byte's first entry in the pair list
    uint32_t pcol[256];               // start of (x, ss) for the copy targets
    uint32_t cstart[257];             // first-byte bucket starts
    uint32_t tmp[FW];
    uint32_t wlo[FW], whi[FW];        // a wave's range of pair entries (the deal)
    uint32_t qn[2], fail, nflag, ndef, nitems, next_item;  // next_item: the work queue's next dl2 item
    uint32_t wq_head, wq_tail, wq_used, wq_out;  // work queue (BZ2MI_TEXT_WQ): claimed, reserved, read, unfinished
    uint32_t wq_cap;                  // usable ring slots (kWqRing; fewer under BZ2MI_DEBUG_WQ_RING)
    uint8_t order[256];               // bytes by ascending bucket size
    uint8_t rank[256];                // position of a byte in that order
    uint8_t target[256];
    uint8_t own[kTQ];                 // the wave of a round's item
#ifdef BZ2MI_PHASES
    uint32_t stat[16];
#endif
};
static_assert(sizeof(TextLds) <= 160 * 1024, "text kernel LDS");

// Pair-list entry: start (17) | len (17) | second byte (8) | first byte (8) |
// sorted explicitly (1) | owner wave (4)
__device__ __forceinline__ uint64_t pe_make(uint32_t start, uint32_t len, uint32_t b, uint32_t a, bool expl) {
    return (uint64_t)start | ((uint64_t)len << 17) | ((uint64_t)b << 34) | ((uint64_t)a << 42) |
           ((uint64_t)(expl ? 1u : 0u) << 50);
}
__device__ __forceinline__ uint32_t pe_start(uint64_t e) { return (uint32_t)e & 0x1ffffu; }
__device__ __forceinline__ uint32_t pe_len(uint64_t e) { return (uint32_t)(e >> 17) & 0x1ffffu; }
__device__ __forceinline__ bool pe_expl(uint64_t e) { return (e >> 50) & 1u; }
__device__ __forceinline__ uint32_t pe_owner(uint64_t e) { return (uint32_t)(e >> 51) & 15u; }

// SA / spill words the text kernel reads back after this wave or another of
// the workgroup rewrote them: plain loads.  The waves of a workgroup share the
// CU's vector L1, which keeps their stores and loads in order, so the
// workgroup fences / barriers in between are all the ordering needed.  (An
// L1-bypassing agent-scope load here can overtake the wave's own earlier
// store: it read stale spill words.)
__device__ __forceinline__ uint32_t ld_fresh(const uint32_t* p) { return *p; }

// the block goes back to the general path; PHASES builds count the reasons
// (g_tbk_res[10 + why]: 0 group > 64, 1 periodic, 2 no progress, 3 pair list,
// 4 work queue, 5 partition depth)
#ifdef BZ2MI_PHASES
#define TBK_FAIL(why)                                  \
    do {                                               \
        atomicOr(&L.fail, 1u);                         \
        atomicAdd(&g_tbk_res[10 + (why)], 1ull);       \
    } while (0)
#else
#define TBK_FAIL(why) atomicOr(&L.fail, 1u)
#endif

__device__ __forceinline__ uint64_t tq_item(uint32_t start, uint32_t len, uint32_t depth) {
    return ((uint64_t)(depth & 0xffffu) << 34) | ((uint64_t)len << 17) | (uint64_t)start;  // start, len < 2^17
}

// append the items of the lanes with `want` to the next round's list
// (wave-aggregated); a full list means the block gives up
// the work queue of BZ2MI_TEXT_WQ builds: a ring over L.q (2 * kTQ entries);
// an entry is an item with bit 63 set (0: empty), the ring positions grow
// without bound (slot = position mod the ring size)
constexpr uint32_t kWqRing = 2 * kTQ;
constexpr uint64_t kWqValid = 1ull << 63;
constexpr int kWqPush = 2;  // tq_push's `nxt` for the ring

__device__ __forceinline__ void tq_push(TextLds& L, int nxt, bool want, uint32_t start, uint32_t len,
                                        uint32_t depth) {
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    if (nxt == kWqPush) {
        // unfinished count first (a waiting wave must not see 0 while these
        // items exist), then the slots.  Slots are reserved only when they
        // fit (a CAS on the tail against the slots not yet read), so every
        // reserved position is written right below and a consumer that
        // claimed one always sees its item; a ring that would overrun
        // reserves nothing and sends the block back (L.fail: every wave then
        // leaves the queue loop, whatever wq_out says).
        uint32_t base = 0, over = 0;
        if (lane_id() == 0) {
            const uint32_t c = (uint32_t)__popcll(m);
            atomicAdd(&L.wq_out, c);
            uint32_t tl = *(volatile uint32_t*)&L.wq_tail;
            for (;;) {
                if (tl + c - *(volatile uint32_t*)&L.wq_used > L.wq_cap) {
                    over = 1u;
                    TBK_FAIL(4);
                    break;
                }
                const uint32_t old = atomicCAS(&L.wq_tail, tl, tl + c);
                if (old == tl) break;
                tl = old;
            }
            base = tl;
        }
        base = uniform(base);
        if (uniform(over)) return;  // (the block goes back; nothing was reserved)
        if (want) {
            const uint32_t pos = base + (uint32_t)__popcll(m & __lanemask_lt());
            (&L.q[0][0])[pos % kWqRing] = tq_item(start, len, depth) | kWqValid;
        }
        return;
    }
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&L.qn[nxt], (uint32_t)__popcll(m));
    base = uniform(base);
    if (want) {
        const uint32_t pos = base + (uint32_t)__popcll(m & __lanemask_lt());
        if (pos < (uint32_t)kTQ) L.q[nxt][pos] = tq_item(start, len, depth);
        else TBK_FAIL(4);
    }
}

// TBK_TRACE builds: every wave's last position in the text kernel, stored to
// host-mapped memory (bz2mi_debug_trace) so a host thread can read it while a
// launch hangs; code = what << 24 | detail
#ifdef TBK_TRACE
#define TBK_T(what, detail)                                                                                \
    do {                                                                                                   \
        if (g_tbk_trace && lane_id() == 0)                                                                 \
            __hip_atomic_store(&g_tbk_trace[blockIdx.x * 16 + (threadIdx.x >> 6)],                         \
                               ((unsigned)(what) << 24) | ((unsigned)(detail) & 0xffffffu), __ATOMIC_RELAXED, \
                               __HIP_MEMORY_SCOPE_SYSTEM);                                                  \
    } while (0)
#else
#define TBK_T(what, detail) \
    do {                    \
    } while (0)
#endif

#ifdef TBK_CHECK
#define TBK_ASSERT(cond, what, a, b)                                                                  \
    do {                                                                                              \
        if (!(cond)) {                                                                                \
            if (lane_id() == 0) printf("[tbk] block %d wave %d: %s (%u, %u)\n", (int)blockIdx.x,       \
                                       (int)(threadIdx.x >> 6), what, (unsigned)(a), (unsigned)(b)); \
            if (lane_id() == 0) atomicOr(&L.fail, 1u);                                                \
            return;                                                                                   \
        }                                                                                             \
    } while (0)
#else
#define TBK_ASSERT(cond, what, a, b) \
    do {                             \
    } while (0)
#endif
#ifdef BZ2MI_PHASES
#define TBK_COUNT(k, v)                                           \
    do {                                                          \
        if (lane_id() == 0) atomicAdd(&L.stat[k], (uint32_t)(v)); \
    } while (0)
#else
#define TBK_COUNT(k, v) \
    do {                \
    } while (0)
#endif

// Work of an item for the dealing: a sort ~ its padded size, a partition ~ half
// its length (one pass, the children are items of their own)
__device__ __forceinline__ uint32_t text_work(uint32_t len) {
    return len > (uint32_t)kTS ? (len >> 1) : len <= 64u ? 64u : len <= 128u ? 128u : len <= 256u ? 256u : 512u;
}
// the wave of an item whose work starts at `run` (of `total`): equal shares
__device__ __forceinline__ uint8_t text_owner(uint32_t run, uint32_t wk, uint32_t total) {
    const uint64_t mid = (uint64_t)run + (wk >> 1);
    return (uint8_t)min((uint64_t)(FW - 1), mid * FW / (total ? total : 1u));
}

// a rotation's final position: its BWT byte (and origPtr)
// BZ2MI_TEXT_FINALPASS (default): the BWT bytes and origPtr are written by
// one coalesced pass over the finished SA at the end of the kernel instead of
// a byte store per placed rotation (realtext BWT 46.3 -> 42.8 ms per GiB, A/B
// on one box; write traffic unchanged at ~39 GB: the byte stores were not
// where the writes are)
#ifndef BZ2MI_TEXT_FINALPASS
#define BZ2MI_TEXT_FINALPASS 1
#endif
// BZ2MI_TEXT_SCATTER2 (A/B, off): the pair scatter through a first-byte
// order in the spill area; measured 42.8 -> 44.3 ms, writes 38.9 -> 40.7 GB
#ifndef BZ2MI_TEXT_SCATTER2
#define BZ2MI_TEXT_SCATTER2 0
#endif
__device__ __forceinline__ void text_final(const uint8_t* Tl, int n, uint32_t pos, uint32_t i, uint8_t* out,
                                           uint32_t* orig) {
    if (out) {  // (null under BZ2MI_TEXT_FINALPASS)
        out[pos] = bwt_byte(Tl, n, i);
        if (i == 0) *orig = pos;
    }
}

// Deferred-group entries (a per-block list, capacity n / 2): start (17) |
// len - 1 (9) | depth (16) | bucket rank (8, set when the list is sorted)
__device__ __forceinline__ uint64_t dg_make(uint32_t start, uint32_t len, uint32_t depth) {
    return (uint64_t)start | ((uint64_t)(len - 1) << 17) | ((uint64_t)min(depth, 0xffffu) << 26);
}
__device__ __forceinline__ uint32_t dg_start(uint64_t e) { return (uint32_t)e & 0x1ffffu; }
__device__ __forceinline__ uint32_t dg_len(uint64_t e) { return ((uint32_t)(e >> 17) & 511u) + 1; }
__device__ __forceinline__ uint32_t dg_depth(uint64_t e) { return (uint32_t)(e >> 26) & 0xffffu; }

// the lanes with `want` append a group (wave-aggregated); a group of more than
// 64 rotations sends the block back
__device__ __forceinline__ void dg_push(TextLds& L, uint64_t* dl, bool want, uint32_t start, uint32_t len,
                                        uint32_t depth) {
    if (want && len > 64u) TBK_FAIL(0);
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&L.ndef, (uint32_t)__popcll(m));
    base = uniform(base);
    if (want) dl[base + (uint32_t)__popcll(m & __lanemask_lt())] = dg_make(start, len, depth);
}

// Order of rotations i0 != i1 of deferred group g that share their first d
// bytes (long repeats), before any copy step.  isa holds the final position
// of every rotation already placed (sorted, or resolved), kNoIsa for the
// rotations of the pair buckets the copy steps fill, and kDefMark | group for
// the members of deferred groups.  Walking x = 1, 2, ...: differing bytes
// decide (x >= d); so do rotations i + x whose positions are both known
// (rotations that share x bytes keep the order of their rotations i + x).
// Rotations i + x that are the two members of another deferred pair h give a
// link (*link = h, *x): the order is h's.  Returns -1 (i0 first), 1 (i1
// first), 3 (link), 2 (wait: they reach a deferred group of more than two or
// the group itself -- a later round may know more), 0 (equal rotations: a
// periodic block).
constexpr uint32_t kNoIsa = 0xffffffffu;
// i + x mod n for i, x < n (no integer division)
__device__ __forceinline__ uint32_t wrap_n(uint32_t v, int n) { return v >= (uint32_t)n ? v - (uint32_t)n : v; }
constexpr uint32_t kDefMark = 0x80000000u;
__device__ __forceinline__ int text_cmp_deferred(const uint8_t* Tl, int n, uint32_t i0, uint32_t i1, uint32_t d,
                                                 uint32_t g, const uint32_t* isa, const uint64_t* dl, uint32_t* link,
                                                 uint32_t* xo);

// Tied items of a wave sort (W[0, tt): index | slot << 17 | group head << 26,
// groups in slot order) at depth D: every group of exactly two rotations is
// ordered by comparing the LDS text directly, 8 bytes at a time, up to
// kTextPairCap bytes (one lane per pair; the repeats of text tie in pairs),
// or flagged (kUnres) when they still tie there; the items of larger groups
// are compacted to W[0, return) for another tie round.
__device__ __forceinline__ uint32_t text_pairs(const uint8_t* Tl, int n, uint32_t* sa, uint32_t base, uint32_t tt,
                                               uint32_t D, uint8_t* out, uint32_t* orig, uint32_t* W, TextLds& L,
                                               uint64_t* dl) {
    constexpr int E = kTS / 64;
    const int lane = lane_id();
    uint32_t wv[E];
    bool keep[E], ph[E];
    uint32_t nkeep = 0, nfl = 0;
    // items are blocked (item lane * E + e in element e): the neighbours
    // q - 1, q + 1, q + 2 are the lane's own elements or the adjacent lanes'
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t q = (uint32_t)(lane * E + e);
        wv[e] = q < tt ? W[q] : 0u;
    }
    uint32_t nxt[2];  // the next lane's elements 0 and 1
    nxt[0] = (uint32_t)__shfl_down((int)wv[0], 1);
    nxt[1] = E > 1 ? (uint32_t)__shfl_down((int)wv[E > 1 ? 1 : 0], 1) : 0u;
    const uint32_t prv = lane_prev(wv[E - 1], 0u);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t q = (uint32_t)(lane * E + e);
        const uint32_t w1 = e + 1 < E ? wv[e + 1 < E ? e + 1 : 0] : nxt[0];
        const uint32_t w2 = e + 2 < E ? wv[e + 2 < E ? e + 2 : 0] : nxt[e + 2 - E < 2 ? e + 2 - E : 0];
        const uint32_t wm = e > 0 ? wv[e > 0 ? e - 1 : 0] : prv;
        const bool h0 = q < tt && (wv[e] >> 26);
        const bool h1 = q + 1 < tt && (w1 >> 26);
        const bool h2 = q + 2 >= tt || (w2 >> 26);
        ph[e] = h0 && q + 1 < tt && !h1 && h2;  // the head of a group of two
        const bool hm = q >= 1 && (wm >> 26) && !h0 && (q + 1 >= tt || h1);  // its second item
        keep[e] = q < tt && !ph[e] && !hm;
        nkeep += keep[e] ? 1u : 0u;
    }
    // the pair heads' (first, second) items compacted to W[256, 256 + 2 np):
    // the comparisons then run one pair per lane, in one divergent pass
    uint32_t* PW = W + 256;
    uint32_t myp = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) myp += ph[e] ? 1u : 0u;
    const uint32_t pinc = wave_incl_sum(myp);
    const uint32_t np = (uint32_t)__builtin_amdgcn_readlane((int)pinc, 63);
    if (np) {
        uint32_t j = pinc - myp;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (ph[e]) {
                PW[2 * j] = wv[e];
                PW[2 * j + 1] = e + 1 < E ? wv[e + 1 < E ? e + 1 : 0] : nxt[0];
                ++j;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    for (uint32_t k0 = 0; k0 < np; k0 += 64) {
        const uint32_t k = k0 + (uint32_t)lane;
        bool dwant = false;
        uint32_t dst = 0, ddep = 0;
        if (k < np) {
            const uint32_t w0 = PW[2 * k], w1 = PW[2 * k + 1];
            const uint32_t i0 = w0 & 0x1ffffu, i1 = w1 & 0x1ffffu;
            const uint32_t s0 = (w0 >> 17) & 511u, s1 = (w1 >> 17) & 511u;
            const uint32_t lo = min(s0, s1);
            uint32_t p0 = i0 + D, p1 = i1 + D;
            if (p0 >= (uint32_t)n) p0 %= (uint32_t)n;
            if (p1 >= (uint32_t)n) p1 %= (uint32_t)n;
            int cmp = 0;
            uint32_t dd = D;
            for (; dd < (uint32_t)kTextPairCap; dd += 8) {
                const uint64_t x0 = load8(Tl, n, p0), x1 = load8(Tl, n, p1);
                if (x0 != x1) {
                    cmp = x0 < x1 ? -1 : 1;
                    break;
                }
                p0 += 8;
                p1 += 8;
                if (p0 >= (uint32_t)n) p0 -= (uint32_t)n;
                if (p1 >= (uint32_t)n) p1 -= (uint32_t)n;
            }
            if (cmp) {
                const uint32_t a = cmp < 0 ? i0 : i1, c = cmp < 0 ? i1 : i0;
                sa[base + lo] = a;
                sa[base + lo + 1] = c;
                text_final(Tl, n, base + lo, a, out, orig);
                text_final(Tl, n, base + lo + 1, c, out, orig);
            } else {  // deferred: a group of two sharing dd bytes
                sa[base + lo] = i0 | kUnres;
                sa[base + lo + 1] = i1 | kUnres;
                nfl += 2;
                dwant = true;
                dst = base + lo;
                ddep = dd;
            }
        }
        dg_push(L, dl, dwant, dst, 2, ddep);
    }
    const uint32_t nf = wave_sum(nfl);
    if (nf && lane == 0) atomicAdd(&L.nflag, nf);
    const uint32_t inc = wave_incl_sum(nkeep);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    __builtin_amdgcn_wave_barrier();  // every lane has read W before it is compacted
    if (tot != tt) {
        uint32_t o = inc - nkeep;
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (keep[e]) W[o++] = wv[e];
        __builtin_amdgcn_wave_barrier();
    }
    return tot;
}

// sort a segment of <= kTS rotations with a common prefix of d bytes (one
// wave; keys from the LDS text); final SA entries, BWT bytes, origPtr.  Items
// still tied after kTextTieCap bytes keep their slots with the kUnres flag
// (ordered by the resolve pass).
#ifndef TBK_SORT_INL
#define TBK_SORT_INL __forceinline__
#endif
// the batched sort items' SA entries loaded one item ahead (A/B: -DBZ2MI_TEXT_PREFETCH=1;
// off: its 16 live registers spilled 99 VGPRs of the sort loop, text BWT
// 31.99 -> 31.64 ms, realtext 74.5 -> 73.6 without it)
#ifndef BZ2MI_TEXT_PREFETCH
#define BZ2MI_TEXT_PREFETCH 0
#endif
// the whole sort phase as one work queue (no rounds; A/B: -DBZ2MI_TEXT_WQ=0
// = the round-4 static deal and barrier-separated rounds)
#ifndef BZ2MI_TEXT_WQ
#define BZ2MI_TEXT_WQ 1
#endif
constexpr bool kTextPrefetch = BZ2MI_TEXT_PREFETCH != 0;
#ifndef TBK_PART_INL
#define TBK_PART_INL __forceinline__
#endif
__device__ TBK_SORT_INL void text_sort_pre(const uint8_t* Tl, int n, uint32_t* sa, Seg seg, uint32_t d, uint8_t* out,
                                            uint32_t* orig, uint32_t* W, TextLds& L, uint64_t* dl,
                                            const uint32_t (&pre)[kTS / 64]) {
    const int lane = lane_id();
    TBK_ASSERT(seg.start + seg.len <= (uint32_t)n && seg.len >= 2u && seg.len <= (uint32_t)kTS, "sort seg", seg.start,
               seg.len);
    Scratch s{};
    s.sa = sa;
    uint32_t tt;
    if (seg.len <= 64) tt = wave_sort_pre_text<1, kTS / 64, kTIB>(Tl, n, s, seg.start, seg.len, d, out, orig, W, pre);
    else if (seg.len <= 128) tt = wave_sort_pre_text<2, kTS / 64, kTIB>(Tl, n, s, seg.start, seg.len, d, out, orig, W, pre);
    else if (kTS <= 256 || seg.len <= 256) tt = wave_sort_pre_text<kTS <= 256 ? kTS / 64 : 4, kTS / 64, kTIB>(Tl, n, s, seg.start, seg.len, d, out, orig, W, pre);
    else tt = wave_sort_pre_text<kTS / 64, kTS / 64, kTIB>(Tl, n, s, seg.start, seg.len, d, out, orig, W, pre);
    tt = uniform(tt);
    TBK_COUNT(4, 1);
    TBK_COUNT(7, seg.len);
    uint32_t D = d + lds_key_bytes(kTIB);
    while (tt) {
#ifdef BZ2MI_PHASES
        const unsigned long long tp0 = wall_clock64();
#endif
        tt = uniform(text_pairs(Tl, n, sa, seg.start, tt, D, out, orig, W, L, dl));
#ifdef BZ2MI_PHASES
        TBK_COUNT(15, wall_clock64() - tp0);
#endif
        if (!tt) break;
        TBK_T(8, D << 12 | tt);
        TBK_COUNT(10, 1);
        if (D + lds_tie_bytes(kTIB) > (uint32_t)kTextTieCap) {
            // deferred: the tied items keep their slots, flagged; every group
            // (a head item and the items up to the next head, consecutive
            // slots from the head's) to the deferred list
            for (uint32_t q0 = 0; q0 < tt; q0 += 64) {
                const uint32_t q = q0 + (uint32_t)lane;
                const uint32_t w = q < tt ? W[q] : 0u;
                if (q < tt) sa[seg.start + ((w >> 17) & 511u)] = (w & 0x1ffffu) | kUnres;
                uint32_t glen = 0;
                const bool hd = q < tt && (w >> 26);
                if (hd) {
                    glen = 1;
                    while (q + glen < tt && !(W[q + glen] >> 26)) ++glen;
                }
                dg_push(L, dl, hd, seg.start + ((w >> 17) & 511u), glen, D);
            }
            if (lane == 0) atomicAdd(&L.nflag, tt);
            return;
        }
#ifdef BZ2MI_PHASES
        const unsigned long long tr0 = wall_clock64();
#endif
        tt = uniform(lds_tie_round_upto<kTS / 64, kTIB>(Tl, n, s, seg.start, tt, D, out, orig, W));
#ifdef BZ2MI_PHASES
        TBK_COUNT(14, wall_clock64() - tr0);
#endif
        D += lds_tie_bytes(kTIB);
    }
}

__device__ TBK_SORT_INL void text_sort(const uint8_t* Tl, int n, uint32_t* sa, Seg seg, uint32_t d, uint8_t* out,
                                        uint32_t* orig, uint32_t* W, TextLds& L, uint64_t* dl) {
    constexpr int E = kTS / 64;
    const int lane = lane_id();
    uint32_t pre[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t g = (uint32_t)(e * 64 + lane);
        pre[e] = g < seg.len ? ld_fresh(sa + seg.start + g) : 0u;
    }
    text_sort_pre(Tl, n, sa, seg, d, out, orig, W, L, dl, pre);
}

// partition a segment of > kTS rotations with a common prefix of d bytes
// by byte d (one wave): children of one rotation are final, runs of small
// ones go to the queue as batches, large ones as items of depth d+1.  A
// segment that is still one child kTextChain levels down (or at kTextDcap) is
// deferred whole (flagged).
__device__ TBK_PART_INL void text_partition(const uint8_t* Tl, int n, uint32_t* sa, uint32_t* spill, Seg seg, uint32_t d,
                               uint8_t* out, uint32_t* orig, uint32_t* W, TextLds& L, int nxt) {
    const int lane = lane_id();
    uint32_t* hist = W;        // then the batch starts
    uint32_t* base = W + 256;  // then pack scratch / the batch lengths
    constexpr int U = 8;
    const uint32_t rounds = (seg.len + 63) / 64;
    TBK_ASSERT(seg.start + seg.len <= (uint32_t)n && seg.len > (uint32_t)kTS, "partition seg", seg.start, seg.len);
    uint32_t c[4];
    const uint32_t dcap = min((uint32_t)kTextDcap, d + (uint32_t)kTextChain);
    for (;;) {
        if (d >= dcap) {  // more than kTS rotations sharing d bytes: the general path
            if (lane == 0) TBK_FAIL(5);
            return;
        }
        TBK_COUNT(5, 1);
        TBK_COUNT(6, seg.len);
        TBK_T(7, d << 17 | seg.len);
#pragma unroll
        for (int j = 0; j < 4; ++j) hist[lane * 4 + j] = 0;
        __builtin_amdgcn_wave_barrier();
        for (uint32_t r0 = 0; r0 < rounds; r0 += U) {
            uint32_t iv[U], cv[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const uint32_t k = (r0 + j) * 64 + lane;
                iv[j] = k < seg.len ? ld_fresh(sa + seg.start + k) : 0u;
            }
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const uint32_t k = (r0 + j) * 64 + lane;
                uint32_t p = iv[j] + d;
                if (p >= (uint32_t)n) p %= (uint32_t)n;
                cv[j] = k < seg.len ? (uint32_t)Tl[p] : 0u;
                if (k < seg.len) spill[seg.start + k] = iv[j] | (cv[j] << 24);
            }
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const uint32_t k = (r0 + j) * 64 + lane;
                const bool v = k < seg.len;
                const uint64_t peers = wave_match8(cv[j], v);
                if (v && (peers & __lanemask_lt()) == 0) atomicAdd(&hist[cv[j]], (uint32_t)__popcll(peers));
            }
        }
        wave_sync_mem();
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = hist[lane * 4 + j];
        bool one = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) one |= c[j] == seg.len;
        if (!__ballot(one)) break;
        d++;  // every rotation has the same byte here: one level deeper, nothing moves
    }
    uint32_t ex[4], tot = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ex[j] = tot;
        tot += c[j];
    }
    const uint32_t lex = wave_incl_sum(tot) - tot;
    TBK_ASSERT((uint32_t)__builtin_amdgcn_readlane((int)(lex + tot), 63) == seg.len, "partition hist",
               __builtin_amdgcn_readlane((int)(lex + tot), 63), seg.len);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ex[j] += lex;
        base[lane * 4 + j] = ex[j];
    }
    __builtin_amdgcn_wave_barrier();
    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t k = r * 64 + lane;
        const bool v = k < seg.len;
        const uint32_t x = v ? ld_fresh(spill + seg.start + k) : 0u;
        const uint32_t cc = x >> 24;
        const uint64_t peers = wave_match8(cc, v);
        const uint64_t below = peers & __lanemask_lt();
        const int leader = peers ? __builtin_ctzll(peers) : 0;
        uint32_t bs = 0;
        if (v && below == 0) bs = atomicAdd(&base[cc], (uint32_t)__popcll(peers));
        bs = (uint32_t)__shfl((int)bs, leader);
        TBK_ASSERT(!__ballot(v && bs + (uint32_t)__popcll(below) >= seg.len), "partition scatter", bs, seg.len);
        if (v) sa[seg.start + bs + (uint32_t)__popcll(below)] = x & 0xffffffu;
    }
    wave_sync_mem();  // the scatter is visible to the reads below
    // batches of the small children (pack scratch: the hist and base areas)
    const uint32_t nbat = pack_children_wave<kTS>(hist, base, W + 512, hist, base);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (c[j] == 1u) {
            const uint32_t pos = seg.start + ex[j];
            text_final(Tl, n, pos, ld_fresh(sa + pos), out, orig);
        }
    }
    bool big[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) big[j] = c[j] > (uint32_t)kTS;
#pragma unroll
    for (int j = 0; j < 4; ++j) tq_push(L, nxt, big[j], seg.start + ex[j], c[j], d + 1);
    for (uint32_t k0 = 0; k0 < nbat; k0 += 64) {
        const uint32_t k = k0 + lane;
        const bool v = k < nbat;
        const uint32_t bl = v ? base[k] : 0u;
        const uint32_t bst = v ? hist[k] : 0u;
        tq_push(L, nxt, v, seg.start + bst, bl & 0x7fffffffu, d + (bl >> 31));
    }
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int text_cmp_deferred(const uint8_t* Tl, int n, uint32_t i0, uint32_t i1, uint32_t d,
                                                 uint32_t g, const uint32_t* isa, const uint64_t* dl, uint32_t* link,
                                                 uint32_t* xo) {
    uint32_t p0 = i0 + 1 < (uint32_t)n ? i0 + 1 : 0u, p1 = i1 + 1 < (uint32_t)n ? i1 + 1 : 0u;
#ifdef BZ2MI_PHASES
    struct WalkStat {
        uint32_t x = 0;
        __device__ ~WalkStat() {
            atomicAdd(&g_tbk_x[4], (unsigned long long)x);
            atomicMax(&g_tbk_x[5], (unsigned long long)x);
        }
    } ws;
#endif
    for (uint32_t x = 1; x < (uint32_t)n; ++x) {
#ifdef BZ2MI_PHASES
        ws.x = x;
#endif
        if (x >= d) {
            const uint32_t c0 = Tl[p0], c1 = Tl[p1];
            if (c0 != c1) return c0 < c1 ? -1 : 1;
        }
        const uint32_t a0 = isa[p0], a1 = isa[p1];
        if (a0 < kDefMark && a1 < kDefMark) return a0 < a1 ? -1 : 1;
        if (a0 == a1 && a0 != kNoIsa) {  // both in deferred group h
            const uint32_t h = a0 & ~kDefMark;
            if (h == g) return 2;
            *link = h;
            *xo = x;
            return 3;
        }
        if (++p0 == (uint32_t)n) p0 = 0;
        if (++p1 == (uint32_t)n) p1 = 0;
    }
    return 0;
}

constexpr uint64_t kDgDone = 1ull << 63;
constexpr uint64_t kLkLink = 1ull << 62;  // link state of a pair: target << 32 | offset

// a deferred pair's rotations in order: SA entries, isa, BWT bytes, origPtr
__device__ __forceinline__ void dg_place(const uint8_t* Tl, int n, uint32_t* sa, uint32_t* isa, uint8_t* out,
                                         uint32_t* orig, uint32_t st, uint32_t a, uint32_t b) {
    sa[st] = a;
    sa[st + 1] = b;
    isa[a] = st;
    isa[b] = st + 1;
    text_final(Tl, n, st, a, out, orig);
    text_final(Tl, n, st + 1, b, out, orig);
}

// Order of rotations a != b from their first byte on, by bytes and known
// positions only (deferred and not yet copied rotations are walked over):
// -1 (a first), 1, or 0 (equal: periodic).  Eight bytes at a time from the
// LDS text; the known positions (global isa) only once per 64 bytes -- any x
// up to which the rotations agree and where both a + x and b + x are placed
// decides the same way as the first differing byte, so the checks only end
// the walk early (a walk through a long repeat is bytes, not isa loads).
__device__ __forceinline__ int text_cmp_plain(const uint8_t* Tl, int n, uint32_t a, uint32_t b, const uint32_t* isa) {
    uint32_t p0 = a, p1 = b;
#ifdef BZ2MI_PHASES
    struct WalkStat {
        uint32_t x = 0;
        __device__ ~WalkStat() {
            atomicAdd(&g_tbk_x[2], (unsigned long long)x);
            atomicMax(&g_tbk_x[3], (unsigned long long)x);
        }
    } ws;
#endif
    for (uint32_t x = 0; x < (uint32_t)n + 8; x += 8) {
#ifdef BZ2MI_PHASES
        ws.x = x;
#endif
        if ((x & 63u) == 0 && x) {
            const uint32_t a0 = isa[p0], a1 = isa[p1];
            if (a0 < kDefMark && a1 < kDefMark) return a0 < a1 ? -1 : 1;
        }
        const uint64_t w0 = load8(Tl, n, p0), w1 = load8(Tl, n, p1);
        if (w0 != w1) return w0 < w1 ? -1 : 1;
        p0 += 8;
        p1 += 8;
        if (p0 >= (uint32_t)n) p0 -= (uint32_t)n;
        if (p1 >= (uint32_t)n) p1 -= (uint32_t)n;
    }
    return 0;
}

// Rank of member k of deferred group g whose members' rotations i + x all
// have known positions (isa): the members keep the order of their images.
// Serial over the m members (m <= 64; nearly always 2 or 3), with no local
// arrays (they went to scratch): the ranks by counting over reloaded images
// (isa of the members themselves -- their new slots, set in the first loop --
// is never an image: an image is placed, a member is not), then the SA slots
// permuted in place by following cycles.
__device__ __forceinline__ void dg_place_by_images(const uint8_t* Tl, int n, uint32_t* sa, uint32_t* isa,
                                                   uint8_t* out, uint32_t* orig, uint32_t st, uint32_t m,
                                                   uint32_t x) {
    auto image = [&](uint32_t k) { return isa[wrap_n((ld_fresh(sa + st + k) & 0x1ffffu) + x, n)]; };
    for (uint32_t k = 0; k < m; ++k) {
        const uint32_t mk = ld_fresh(sa + st + k) & 0x1ffffu, key = image(k);
        uint32_t r = 0;
        for (uint32_t j = 0; j < m; ++j) r += image(j) < key ? 1u : 0u;
        isa[mk] = st + r;
        text_final(Tl, n, st + r, mk, out, orig);
    }
    for (uint32_t q = 0; q < m; ++q) {
        uint32_t v = ld_fresh(sa + st + q) & 0x1ffffu;
        uint32_t to = isa[v] - st;
        while (to != q) {
            const uint32_t w = ld_fresh(sa + st + to) & 0x1ffffu;
            sa[st + to] = v;
            v = w;
            to = isa[v] - st;
        }
        sa[st + q] = v;
    }
}

// Every deferred group of the block (dl[0, ndef)), ordered before the copy
// steps.  Rounds of: (1) every open group walks x = 1, 2, ... (pairs: one
// thread each, text_cmp_deferred; larger groups: one wave, a lane per
// member) until its members' rotations i + x all have known positions --
// placed by their order -- or all lie in one other deferred group h -- a link
// (h, x): the group's order is that of its images in h; (2) pointer jumping
// over the links (a group whose target is placed is placed by its images; one
// whose target is linked takes that link, offsets added), so the chain of a
// repeat -- group (i, j, ...) links to (i + x, j + x, ...), and so on down to
// the group that meets the repeat's end -- collapses in a logarithmic number
// of steps; (3) larger groups whose members' bytes part before any decision
// rank every member by comparing it with the others.  A round that places
// nothing sends the block back (a group waiting on itself: a tandem repeat).
// lk: a state per group (0 open, kDgDone, or a link).
#ifndef TBK_RES_INL
#define TBK_RES_INL
#endif
__device__ TBK_RES_INL void text_resolve_all(const uint8_t* Tl, int n, uint32_t* sa, uint32_t* isa, const uint64_t* dl,
                                 uint32_t ndef, uint64_t* lk, uint8_t* out, uint32_t* orig, TextLds& L) {
    const int t = threadIdx.x, w = wave_id(), lane = lane_id();
    uint32_t* W = L.w[w];
    for (uint32_t g = t; g < ndef; g += FT) lk[g] = 0;
    __threadfence_block();
    __syncthreads();
    uint32_t before = 0xffffffffu;
    bool forced = false;  // the previous round ordered the open roots by plain comparison
#ifdef BZ2MI_PHASES
    unsigned long long rt0 = 0;
#endif
    for (uint32_t rr = 0;; ++rr) {
        TBK_T(12, rr << 12 | min(ndef, 4095u));
#ifdef BZ2MI_PHASES
        if (rr) {
            if (t == 0) atomicAdd(&g_tbk_res[6], wall_clock64() - rt0);
        }
        rt0 = wall_clock64();
#endif
#ifdef BZ2MI_PHASES
        if (t == 0) atomicAdd(&g_tbk_res[3], 1ull);
#endif
        // (1) pairs
        for (uint32_t g = t; g < ndef; g += FT) {
            const uint64_t e = dl[g];
            if (dg_len(e) != 2 || lk[g] != 0) continue;
            const uint32_t st = dg_start(e);
            const uint32_t i0 = ld_fresh(sa + st) & 0x1ffffu, i1 = ld_fresh(sa + st + 1) & 0x1ffffu;
            uint32_t h = 0, x = 0;
            const int c = text_cmp_deferred(Tl, n, i0, i1, dg_depth(e), g, isa, dl, &h, &x);
            if (c == 0) {
                TBK_FAIL(1);
                continue;
            }
            if (c == 2) continue;
            if (c == 3) {
                lk[g] = kLkLink | ((uint64_t)h << 32) | x;
                continue;
            }
            dg_place(Tl, n, sa, isa, out, orig, st, c < 0 ? i0 : i1, c < 0 ? i1 : i0);
            lk[g] = kDgDone;
        }
        // (1) larger groups: a wave each, lane = member, while the members
        // share their bytes (x < depth)
        for (uint32_t gb = (uint32_t)w * 64; gb < ndef; gb += FT) {
            const uint32_t g = gb + (uint32_t)lane;
            const uint64_t e = g < ndef ? dl[g] : 0ull;
            for (uint64_t mm = __ballot(g < ndef && dg_len(e) > 2 && lk[g] == 0); mm; mm &= mm - 1) {
                const int l = __builtin_ctzll(mm);
                const uint32_t gg = gb + (uint32_t)l;
                const uint32_t lo = uniform((uint32_t)__shfl((int)(uint32_t)e, l));
                const uint32_t hi = uniform((uint32_t)__shfl((int)(uint32_t)(e >> 32), l));
                const uint64_t ee = ((uint64_t)hi << 32) | lo;
                const uint32_t st = dg_start(ee), m = dg_len(ee), dep = dg_depth(ee);
                const bool mine = (uint32_t)lane < m;
                const uint32_t me = mine ? ld_fresh(sa + st + lane) & 0x1ffffu : 0u;
                for (uint32_t x = 1; x < dep; ++x) {
                    const uint32_t a = mine ? isa[wrap_n(me + x, n)] : 0u;
                    if (!__ballot(mine && a >= kDefMark)) {  // every image placed
                        const uint32_t key = mine ? a : 0xffffffffu;
                        uint32_t r = 0;
                        for (uint32_t k = 0; k < m; ++k) r += (uint32_t)__shfl((int)key, (int)k) < key ? 1u : 0u;
                        if (mine) {
                            sa[st + r] = me;
                            isa[me] = st + r;
                            text_final(Tl, n, st + r, me, out, orig);
                        }
                        if (lane == 0) lk[gg] = kDgDone;
                        break;
                    }
                    const uint32_t a0 = (uint32_t)__shfl((int)a, 0);
                    if (a0 != kNoIsa && a0 >= kDefMark && (a0 & ~kDefMark) != gg && !__ballot(mine && a != a0)) {
                        if (lane == 0) lk[gg] = kLkLink | ((uint64_t)(a0 & ~kDefMark) << 32) | x;
                        break;
                    }
                }
            }
        }
        __threadfence_block();
        __syncthreads();
#ifdef BZ2MI_PHASES
        if (t == 0) atomicAdd(&g_tbk_res[1], wall_clock64() - rt0);
        rt0 = wall_clock64();
#endif
        // (2) links
        for (int jump = 0; jump < 32; ++jump) {
            TBK_T(13, rr << 8 | (uint32_t)jump);
#ifdef BZ2MI_PHASES
            if (t == 0) atomicAdd(&g_tbk_res[4], 1ull);
#endif
            if (t == 0) L.qn[1] = 0;
            __syncthreads();
            for (uint32_t g = t; g < ndef; g += FT) {
                const uint64_t v = lk[g];
                if (!(v & kLkLink)) continue;
                const uint32_t h = (uint32_t)(v >> 32) & 0x3fffffffu, x = (uint32_t)v;
                const uint64_t e = dl[g];
                const uint32_t st = dg_start(e), m = dg_len(e);
                bool known = true;
                for (uint32_t k = 0; k < m && known; ++k)
                    known = isa[wrap_n((ld_fresh(sa + st + k) & 0x1ffffu) + x, n)] < kDefMark;
                if (known) {
                    dg_place_by_images(Tl, n, sa, isa, out, orig, st, m, x);
                    lk[g] = kDgDone;
                    atomicAdd(&L.qn[1], 1u);
                    continue;
                }
                const uint64_t th = lk[h];
                if ((th & kLkLink) && (uint32_t)(th >> 32 & 0x3fffffffu) != g) {
                    const uint32_t nx = x + (uint32_t)th;
                    if (nx >= (uint32_t)n) {
                        TBK_FAIL(1);
                        continue;
                    }
                    lk[g] = kLkLink | (th & (0x3fffffffull << 32)) | nx;
                    atomicAdd(&L.qn[1], 1u);
                }
            }
            __threadfence_block();
            __syncthreads();
            if (uniform(L.qn[1]) == 0 || uniform(L.fail)) break;  // nothing placed or jumped
        }
#ifdef BZ2MI_PHASES
        if (t == 0) atomicAdd(&g_tbk_res[5], wall_clock64() - rt0);
        rt0 = wall_clock64();
#endif
        // (3) larger groups still open: every member against the others
        for (uint32_t gb = (uint32_t)w * 64; gb < ndef; gb += FT) {
            const uint32_t g = gb + (uint32_t)lane;
            const uint64_t e = g < ndef ? dl[g] : 0ull;
            for (uint64_t mm = __ballot(g < ndef && dg_len(e) > 2 && lk[g] == 0); mm; mm &= mm - 1) {
                const int l = __builtin_ctzll(mm);
                const uint32_t lo = uniform((uint32_t)__shfl((int)(uint32_t)e, l));
                const uint32_t hi = uniform((uint32_t)__shfl((int)(uint32_t)(e >> 32), l));
                const uint64_t ee = ((uint64_t)hi << 32) | lo;
                const uint32_t st = dg_start(ee), m = dg_len(ee), dep = dg_depth(ee);
                const uint32_t me = (uint32_t)lane < m ? ld_fresh(sa + st + lane) & 0x1ffffu : 0u;
                // a tandem repeat u^m t: the members (by position) step by the
                // period P and the text is P-periodic from the first to the
                // last; then their order is monotone -- every comparison
                // reduces to u t against t, i.e. the last member against the
                // rotation one period after it
                {
                    const uint32_t key = (uint32_t)lane < m ? me : 0xffffffffu;
                    uint32_t pr = 0;  // rank by position
                    for (uint32_t k = 0; k < m; ++k) pr += (uint32_t)__shfl((int)key, (int)k) < key ? 1u : 0u;
                    if ((uint32_t)lane < m) W[pr] = me;
                    __builtin_amdgcn_wave_barrier();
                    const uint32_t q0 = uniform(W[0]), P = uniform(W[1] - W[0]), qe = uniform(W[m - 1]);
                    bool prog = true;
                    for (uint32_t k = lane + 1; k < m; k += 64) prog &= W[k] - W[k - 1] == P;
                    prog = !__ballot(!prog) && P > 0 && qe + P < (uint32_t)n;
                    if (prog) {  // periodic over [q0, qe)?
                        bool per = true;
                        for (uint32_t x = q0 + lane; x < qe && per; x += 64) per = Tl[x] == Tl[x + P];
                        prog = !__ballot(!per);
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (prog) {
                        int dir = 0;
                        if (lane == 0) dir = text_cmp_plain(Tl, n, qe, qe + P, isa);
                        dir = (int)uniform((uint32_t)dir);
                        if (dir == 0) {
                            if (lane == 0) TBK_FAIL(1);
                            continue;
                        }
                        if ((uint32_t)lane < m) {
                            const uint32_t slot = dir < 0 ? pr : m - 1 - pr;
                            sa[st + slot] = me;
                            isa[me] = st + slot;
                            text_final(Tl, n, st + slot, me, out, orig);
                        }
                        if (lane == 0) lk[gb + l] = kDgDone;
                        continue;
                    }
                }
                uint32_t below = 0;
                bool bad = false, wait = false;
                for (uint32_t k = 0; k < m; ++k) {
                    const uint32_t other = (uint32_t)__shfl((int)me, (int)k);
                    if ((uint32_t)lane < m && k != (uint32_t)lane && !wait && !bad) {
                        uint32_t h = 0, x = 0;
                        const int c = text_cmp_deferred(Tl, n, other, me, dep, gb + l, isa, dl, &h, &x);
                        below += c == -1 ? 1u : 0u;
                        bad |= c == 0;
                        wait |= c == 2 || c == 3;
                    }
                }
                if (__ballot(bad)) {
                    if (lane == 0) TBK_FAIL(1);
                    continue;
                }
                if (__ballot(wait)) continue;
                __builtin_amdgcn_wave_barrier();  // every lane has read its member before the writes
                if ((uint32_t)lane < m) {
                    sa[st + below] = me;
                    isa[me] = st + below;
                    text_final(Tl, n, st + below, me, out, orig);
                }
                if (lane == 0) lk[gb + l] = kDgDone;
            }
        }
        __threadfence_block();
        if (t == 0) L.qn[0] = 0;
        __syncthreads();
        for (uint32_t g = t; g < ndef; g += FT)
            if (lk[g] != kDgDone) atomicAdd(&L.qn[0], 1u);
        __syncthreads();
        const uint32_t left = uniform(L.qn[0]);
        if (left == 0 || uniform(L.fail)) break;
        TBK_T(14, rr << 12 | min(left, 4095u));
        if (left >= before && !forced) {
            // no group placed this round: the open groups that are not
            // linked (the roots the linked ones wait on) are ordered by plain
            // comparison -- bytes and known positions only, walking over the
            // rest (however long) -- and the rounds go on
            for (uint32_t gb = (uint32_t)w * 64; gb < ndef; gb += FT) {
                const uint32_t g = gb + (uint32_t)lane;
                const bool root = g < ndef && lk[g] == 0;
                for (uint64_t mm = __ballot(root); mm; mm &= mm - 1) {
                    const int l = __builtin_ctzll(mm);
                    const uint64_t ee = dl[gb + l];
                    const uint32_t st = dg_start(ee), m = dg_len(ee);
                    const uint32_t me = (uint32_t)lane < m ? ld_fresh(sa + st + lane) & 0x1ffffu : 0u;
                    uint32_t below = 0;
                    bool bad = false;
                    for (uint32_t k = 0; k < m; ++k) {
                        const uint32_t other = (uint32_t)__shfl((int)me, (int)k);
                        if ((uint32_t)lane < m && k != (uint32_t)lane && !bad) {
                            const int c = text_cmp_plain(Tl, n, other, me, isa);
                            below += c == -1 ? 1u : 0u;
                            bad |= c == 0;
                        }
                    }
                    if (__ballot(bad)) {
                        if (lane == 0) TBK_FAIL(1);
                        continue;
                    }
                    __builtin_amdgcn_wave_barrier();
                    if ((uint32_t)lane < m) {
                        sa[st + below] = me;
                        isa[me] = st + below;
                        text_final(Tl, n, st + below, me, out, orig);
                    }
                    if (lane == 0) lk[gb + l] = kDgDone;
                }
            }
            __threadfence_block();
            __syncthreads();
            forced = true;
#ifdef BZ2MI_PHASES
            if (t == 0) atomicAdd(&g_tbk_res[7], 1ull);
#endif
            continue;
        }
        forced = false;
        if (left >= before) {  // no group placed this round, nor by the plain comparisons
            if (t == 0) TBK_FAIL(2);
#ifdef TBK_NOPROG_DEBUG
            if (t == 0) {
                int shown = 0;
                for (uint32_t g = 0; g < ndef && shown < 4; ++g) {
                    if (lk[g] == kDgDone) continue;
                    const uint64_t e = dl[g];
                    const uint32_t st = dg_start(e), m = dg_len(e);
                    printf("[noprog] block %d n %d group %u/%u len %u depth %u lk %llx members", (int)blockIdx.x, n, g,
                           ndef, m, dg_depth(e), (unsigned long long)lk[g]);
                    for (uint32_t k = 0; k < m && k < 6; ++k) printf(" %u", ld_fresh(sa + st + k) & 0x1ffffu);
                    printf("\n");
                    for (uint32_t x = 1; x < 6; ++x) {
                        printf("   x=%u:", x);
                        for (uint32_t k = 0; k < m && k < 6; ++k) {
                            const uint32_t i = ld_fresh(sa + st + k) & 0x1ffffu;
                            printf(" %08x", isa[(i + x) % (uint32_t)n]);
                        }
                        printf("\n");
                    }
                    ++shown;
                }
            }
#endif
            break;
        }
        before = left;
    }
}

__global__ __launch_bounds__(FT) void bwt_text_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                      const uint32_t* __restrict__ lens, int nblocks,
                                                      uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                      uint32_t* __restrict__ orig_out, uint32_t* __restrict__ redo,
                                                      uint32_t* __restrict__ spill_all, Seg* __restrict__ grp_all,
                                                      uint64_t* __restrict__ key_all, uint64_t* __restrict__ glist_all,
                                                      size_t tcap, uint32_t wq_cap) {
    __shared__ TextLds L;
    const int b = blockIdx.x;
    if (b >= nblocks || redo[b] != 1u) return;
#ifdef BZ2MI_PHASES
    const unsigned long long tk0 = wall_clock64();
    unsigned long long tks = 0, tkc = 0, tk1 = 0;
#endif
    const int t = threadIdx.x, w = wave_id(), lane = lane_id();
    const int n = (int)uniform(lens[b]);
    const uint8_t* T = blocks + (size_t)b * stride;
    uint8_t* out = bwt_out + (size_t)b * stride;
    uint8_t* const bw = BZ2MI_TEXT_FINALPASS ? nullptr : out;  // BWT bytes written as rotations are placed
    uint32_t* orig = orig_out + b;
    uint32_t* sa = sa_all + (size_t)b * stride;
    uint32_t* spill = spill_all + (size_t)b * stride;
    // the pair list (kPairCap entries at most; a block with more goes back)
    uint64_t* pl = reinterpret_cast<uint64_t*>(grp_all + (size_t)b * bwt_group_stride(stride));
    // deferred groups (n / 2 at most) as found, then sorted by bucket rank
    uint64_t* dl = key_all + (size_t)b * tcap;
    uint64_t* dl2 = glist_all + (size_t)b * tcap;
    const uint8_t* Tl = reinterpret_cast<const uint8_t*>(L.text);
    uint32_t* W = L.w[w];
    {
        const int n16 = (n + 15) >> 4;
        const uint4* T4 = reinterpret_cast<const uint4*>(T);
        for (int v = t; v < n16; v += FT) L.text[v] = T4[v];
    }
    // ---- the pair index: which second bytes follow each first byte (mask),
    // then the non-empty pairs numbered row-major (rowpre: the number of the
    // first pair of every 32-byte word of a row) and counted in LDS (the
    // per-wave scratch is free until the sort phase)
    uint32_t* cnt = &L.w[0][0];            // kPairCap pair counters, then starts, then cursors
    uint32_t* rowpre = cnt + kPairCap;     // 256 x 8
    if (t < 256) {
#pragma unroll
        for (int j = 0; j < 8; ++j) L.mask[t][j] = 0;
    }
    if (t == 0) {
        L.fail = 0;
        L.nflag = 0;
        L.ndef = 0;
    }
    if (t < FW) {
        L.wlo[t] = 0xffffffffu;
        L.whi[t] = 0;
    }
#ifdef BZ2MI_PHASES
    if (t < 16) L.stat[t] = 0;
#endif
    __syncthreads();
    for (int i = t; i < n; i += FT) {
        const uint32_t a = Tl[i], c2 = Tl[i + 1 < n ? i + 1 : 0];
        atomicOr(&L.mask[a][c2 >> 5], 1u << (c2 & 31u));
    }
    __syncthreads();
#ifdef BZ2MI_PHASES
    if (t == 0) atomicAdd(&g_tbk_x[8], wall_clock64() - tk0);
#endif
    uint32_t P;
    {
        const uint32_t q0 = (uint32_t)t * 2;  // (first byte, word) = (q >> 3, q & 7)
        const uint32_t c0 = (uint32_t)__popc(L.mask[q0 >> 3][q0 & 7u]), c1 = (uint32_t)__popc(L.mask[q0 >> 3][(q0 & 7u) + 1]);
        const uint32_t ex = wg_excl_sum<FT>(c0 + c1, L.tmp, &P);
        rowpre[q0] = ex;
        rowpre[q0 + 1] = ex + c0;
        if ((q0 & 7u) == 0) L.rowoff[q0 >> 3] = ex;
    }
    if (P > min((uint32_t)kPairCap, (uint32_t)bwt_group_stride(stride))) {  // uniform (a workgroup sum)
#ifdef BZ2MI_PHASES
        if (t == 0) atomicAdd(&g_tbk_res[13], 1ull);
#endif
        if (t == 0) redo[b] = 2u;
        return;
    }
    for (uint32_t j = t; j < P; j += FT) cnt[j] = 0;
    __syncthreads();
    auto pair_of = [&](uint32_t a, uint32_t c2) {
        const uint32_t wq = c2 >> 5;
        return rowpre[a * 8 + wq] + (uint32_t)__popc(L.mask[a][wq] & ((1u << (c2 & 31u)) - 1u));
    };
    for (int i = t; i < n; i += FT) atomicAdd(&cnt[pair_of(Tl[i], Tl[i + 1 < n ? i + 1 : 0])], 1u);
    __syncthreads();
#ifdef BZ2MI_PHASES
    if (t == 0) atomicAdd(&g_tbk_x[9], wall_clock64() - tk0);
#endif
    {
        // pair starts in place (each thread a contiguous run of pairs)
        const uint32_t per = (P + FT - 1) / FT;
        const uint32_t j0 = min(P, (uint32_t)t * per), j1 = min(P, j0 + per);
        uint32_t sum = 0;
        for (uint32_t j = j0; j < j1; ++j) sum += cnt[j];
        uint32_t tot;
        uint32_t run = wg_excl_sum<FT>(sum, L.tmp, &tot);
        for (uint32_t j = j0; j < j1; ++j) {
            const uint32_t v = cnt[j];
            cnt[j] = run;
            run += v;
        }
    }
    __syncthreads();
    // first-byte bucket starts and the processing order (ascending size)
    if (t <= 256) {
        const uint32_t j = t < 256 ? rowpre[t * 8] : P;
        L.cstart[t] = j < P ? cnt[j] : (uint32_t)n;
    }
    __syncthreads();
    if (t < 256) {
        const uint32_t c = L.cstart[t + 1] - L.cstart[t];
        uint32_t rk = 0;
        for (uint32_t q = 0; q < 256; ++q) {
            const uint32_t o = L.cstart[q + 1] - L.cstart[q];
            rk += (o < c || (o == c && q < (uint32_t)t)) ? 1u : 0u;
        }
        L.order[rk] = (uint8_t)t;
        L.rank[t] = (uint8_t)rk;
    }
    // the buckets in the order before s_big are sorted whole (no copies into
    // them); the last kCopySteps non-empty ones are the copy-processed buckets
    const uint32_t K = (uint32_t)__syncthreads_count(t < 256 && L.cstart[t + 1] > L.cstart[t]);
    const uint32_t s0 = 256u - K;
    const uint32_t s_big = max(s0, 256u - (uint32_t)kCopySteps);
#ifdef BZ2MI_PHASES
    if (t == 0) atomicAdd(&g_tbk_x[10], wall_clock64() - tk0);
#endif
    // the pair list (global): start, length, bytes, sorted-explicitly flag
    for (uint32_t q = t; q < 2048; q += FT) {
        const uint32_t a = q >> 3, wq = q & 7u;
        uint32_t m = L.mask[a][wq], j = rowpre[q];
        const uint32_t ra = L.rank[a];
        while (m) {
            const uint32_t c2 = wq * 32 + (uint32_t)__builtin_ctz(m);
            m &= m - 1;
            const uint32_t st = cnt[j], en = j + 1 < P ? cnt[j + 1] : (uint32_t)n;
            pl[j] = pe_make(st, en - st, c2, a, L.rank[c2] >= ra || ra < s_big);
            ++j;
        }
    }
    __syncthreads();
#ifdef BZ2MI_PHASES
    if (t == 0) atomicAdd(&g_tbk_x[11], wall_clock64() - tk0);
#endif
    // ---- every rotation to its pair bucket.  BZ2MI_TEXT_SCATTER2: through
    // the first-byte order in `spill` (free until the sort phase): a 256-way
    // scatter there (each bucket's append point is one L2 line, so the
    // partial writes merge before they leave L2), then the pair scatter in
    // that order, whose appends go to the pair buckets of one or two first
    // bytes at a time -- instead of one 2,000-way scatter whose partial-line
    // writes reached HBM one sector per rotation
#if BZ2MI_TEXT_SCATTER2
    if (t < 256) L.pcol[t] = L.cstart[t];
    __syncthreads();
    for (int i = t; i < n; i += FT) spill[atomicAdd(&L.pcol[Tl[i]], 1u)] = (uint32_t)i;
    __threadfence_block();
    __syncthreads();
    for (int k = t; k < n; k += FT) {
        const uint32_t i = ld_fresh(spill + k);
        sa[atomicAdd(&cnt[pair_of(Tl[i], Tl[i + 1 < (uint32_t)n ? i + 1 : 0])], 1u)] = i;
    }
#else
    for (int i = t; i < n; i += FT)
        sa[atomicAdd(&cnt[pair_of(Tl[i], Tl[i + 1 < n ? i + 1 : 0])], 1u)] = (uint32_t)i;
#endif
    __threadfence_block();
    __syncthreads();
#ifdef BZ2MI_PHASES
    if (t == 0) atomicAdd(&g_tbk_stat[0], wall_clock64() - tk0);
#endif
    TBK_T(1, P);
    // ---- sort phase: the pair buckets (a, c) with rank(c) >= rank(a) are
    // sorted directly (the others are filled by the copies below), all at
    // once: round 0 deals the pair buckets over the waves in equal shares of
    // work (contiguous ranges of the pair list), partitions put their
    // children into the next round's list; a round ends at a barrier
#ifdef BZ2MI_PHASES
    tk1 = wall_clock64();
#endif
    if (t < 2) L.qn[t] = 0;
    if (t == 0) L.nitems = 0;
    __syncthreads();
    // sort items (dl2, free until the deferred groups are sorted): a thread
    // per first-byte row walks its pair buckets in order; runs of consecutive
    // explicit pairs of <= kTS / 2 rotations become batches of <= kTS
    // (sorted from depth 1: the second byte separates them), larger pairs
    // items of their own (depth 2: a wave sort or a partition); explicit
    // pairs of one rotation are final.  (cnt[j] is pair j's end after the
    // scatter, so its start is cnt[j - 1].)
    if (t < 256) {
        const uint32_t a = (uint32_t)t, ra = L.rank[a];
        uint32_t j = rowpre[a * 8];
        uint32_t bst = 0, blen = 0, bcnt = 0;
        auto flush = [&]() {
            if (blen >= 2) dl2[atomicAdd(&L.nitems, 1u)] = tq_item(bst, blen, bcnt > 1 ? 1u : 2u);
            else if (blen == 1) text_final(Tl, n, bst, ld_fresh(sa + bst), bw, orig);
            blen = bcnt = 0;
        };
        for (uint32_t wq = 0; wq < 8; ++wq) {
            uint32_t m = L.mask[a][wq];
            while (m) {
                const uint32_t c2 = wq * 32 + (uint32_t)__builtin_ctz(m);
                m &= m - 1;
                const uint32_t st = j ? cnt[j - 1] : 0u, len = cnt[j] - st;
                ++j;
                if (!(L.rank[c2] >= ra || ra < s_big)) {
                    flush();
                    continue;
                }
                if (len > (uint32_t)kTS / 2) {
                    flush();
                    dl2[atomicAdd(&L.nitems, 1u)] = tq_item(st, len, 2u);
                    continue;
                }
                if (blen + len > (uint32_t)kTS) flush();
                if (blen == 0) bst = st;
                blen += len;
                bcnt++;
            }
        }
        flush();
    }
    __threadfence_block();
    __syncthreads();
    const uint32_t nitems = uniform(L.nitems);
#if BZ2MI_TEXT_WQ
    // One work queue for the whole sort phase, no rounds: a wave takes the
    // oldest item of the ring (children of partitions) or else the next sort
    // item of dl2, and pushes a partition's children to the ring.  wq_out
    // counts the items not yet finished (dl2's and the ring's): a wave with
    // nothing to take waits until it is 0 (every wave of the workgroup is
    // resident, so the waves it waits on make progress) or the block fails.
    if (t == 0) {
        L.next_item = 0;
        L.wq_head = L.wq_tail = L.wq_used = 0;
        L.wq_out = nitems;
        L.wq_cap = wq_cap < kWqRing ? wq_cap : kWqRing;
    }
    for (int k = t; k < (int)kWqRing; k += FT) (&L.q[0][0])[k] = 0;
    __syncthreads();
    for (;;) {
        if (uniform(*(volatile uint32_t*)&L.fail)) break;
        uint32_t got = 0, lo32 = 0, hi32 = 0;
        if (lane == 0) {
            const uint32_t h = *(volatile uint32_t*)&L.wq_head, tl = *(volatile uint32_t*)&L.wq_tail;
            if (h < tl && atomicCAS(&L.wq_head, h, h + 1) == h) {
                // claimed ring position h: its item is written right after the
                // push reserved it (tq_push reserves only slots that fit, so
                // it comes; the wait also ends when the block has failed)
                volatile uint64_t* slot = &(&L.q[0][0])[h % kWqRing];
                uint64_t v;
                while (!((v = *slot) & kWqValid) && *(volatile uint32_t*)&L.fail == 0u) __builtin_amdgcn_s_sleep(1);
                if (v & kWqValid) {
                    *slot = 0;
                    atomicAdd(&L.wq_used, 1u);
                    lo32 = (uint32_t)v;
                    hi32 = (uint32_t)(v >> 32) & 0x7fffffffu;
                    got = 1;
                }
            } else if (h >= tl) {
                const uint32_t k = atomicAdd(&L.next_item, 1u);
                if (k < nitems) {
                    const uint64_t v = dl2[k];
                    lo32 = (uint32_t)v;
                    hi32 = (uint32_t)(v >> 32);
                    got = 1;
                }
            }
        }
        if (!uniform(got)) {
            if (uniform(*(volatile uint32_t*)&L.wq_out) == 0) break;
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        const uint64_t it = ((uint64_t)uniform(hi32) << 32) | uniform(lo32);
        const Seg seg{(uint32_t)it & 0x1ffffu, (uint32_t)(it >> 17) & 0x1ffffu};
        const uint32_t d = (uint32_t)(it >> 34) & 0xffffu;
        TBK_T(3, seg.len);
#ifdef BZ2MI_PHASES
        const unsigned long long ti0 = wall_clock64();
#endif
        if (seg.len <= (uint32_t)kTS) text_sort(Tl, n, sa, seg, d, bw, orig, W, L, dl);
        else text_partition(Tl, n, sa, spill, seg, d, bw, orig, W, L, kWqPush);
        TBK_T(11, seg.len);
#ifdef BZ2MI_PHASES
        TBK_COUNT(seg.len <= (uint32_t)kTS ? 12 : 13, wall_clock64() - ti0);
#endif
        if (lane == 0) atomicSub(&L.wq_out, 1u);
    }
    __threadfence_block();
    __syncthreads();
    if (false)
#endif
    {
        // deal the items in equal shares of work (contiguous ranges of the list)
        const uint32_t per = (nitems + FT - 1) / FT;
        const uint32_t e0 = min(nitems, (uint32_t)t * per), e1 = min(nitems, e0 + per);
        uint32_t sum = 0;
        for (uint32_t e = e0; e < e1; ++e) sum += text_work((uint32_t)(dl2[e] >> 17) & 0x1ffffu);
        uint32_t total;
        uint32_t run = wg_excl_sum<FT>(sum, L.tmp, &total);
        for (uint32_t e = e0; e < e1; ++e) {
            const uint32_t wk = text_work((uint32_t)(dl2[e] >> 17) & 0x1ffffu);
            const uint32_t o = text_owner(run, wk, total);
            run += wk;
            atomicMin(&L.wlo[o], e);
            atomicMax(&L.whi[o], e + 1);
        }
    }
    __threadfence_block();
    __syncthreads();
#if BZ2MI_TEXT_WQ
    if (false)
#endif
    {
        // this wave's items, the next one's SA entries loaded while the
        // current one is sorted
        const uint32_t lo = uniform(L.wlo[w]), hi = uniform(L.whi[w]);
        constexpr int E = kTS / 64;
        uint32_t pre[E];
        auto load = [&](uint32_t k, uint32_t (&dst)[E]) {
            const uint64_t it = dl2[k];
            const uint32_t st = (uint32_t)it & 0x1ffffu, len = (uint32_t)(it >> 17) & 0x1ffffu;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint32_t g = (uint32_t)(e * 64 + lane);
                dst[e] = (len <= (uint32_t)kTS && g < len) ? ld_fresh(sa + st + g) : 0u;
            }
        };
        if (kTextPrefetch && lo < hi) load(lo, pre);
        for (uint32_t k = lo; k < hi; ++k) {
            if (uniform(*(volatile uint32_t*)&L.fail)) break;  // the block goes back to the general path
            uint32_t nxt[E];
            if (kTextPrefetch && k + 1 < hi) load(k + 1, nxt);
            if (!kTextPrefetch) load(k, pre);
            const uint64_t it = dl2[k];
            const Seg seg{uniform((uint32_t)it & 0x1ffffu), uniform((uint32_t)(it >> 17) & 0x1ffffu)};
            const uint32_t d = uniform((uint32_t)(it >> 34) & 0xffffu);
            TBK_T(2, seg.len);
#ifdef BZ2MI_PHASES
            const unsigned long long ti0 = wall_clock64();
#endif
            if (seg.len <= (uint32_t)kTS) text_sort_pre(Tl, n, sa, seg, d, bw, orig, W, L, dl, pre);
            else text_partition(Tl, n, sa, spill, seg, d, bw, orig, W, L, 0);
            TBK_T(10, seg.len);
#ifdef BZ2MI_PHASES
            TBK_COUNT(seg.len <= (uint32_t)kTS ? 12 : 13, wall_clock64() - ti0);
#endif
            if (kTextPrefetch) {
#pragma unroll
                for (int e = 0; e < E; ++e) pre[e] = nxt[e];
            }
        }
    }
    __threadfence_block();
    __syncthreads();
    for (int cur = 0; !BZ2MI_TEXT_WQ; cur ^= 1) {
        // loop conditions from LDS go through readfirstlane: scalar branches
        // (a vector-condition loop around the item calls lost the exec mask)
        const uint32_t nit = uniform(min(L.qn[cur], (uint32_t)kTQ));
        if (nit == 0 || uniform(L.fail)) break;
        if (t == 0) TBK_COUNT(3, 1);
        TBK_T(4, cur << 16 | nit);
        __syncthreads();  // every thread has read the count
        if (t == 0) L.qn[cur ^ 1] = 0;
        if (w == 0) {  // deal the round's items in equal shares of work
            uint32_t wk[kTQ / 64], sum = 0;
#pragma unroll
            for (int j = 0; j < kTQ / 64; ++j) {
                const uint32_t k = (uint32_t)lane * (kTQ / 64) + j;
                wk[j] = k < nit ? text_work((uint32_t)(L.q[cur][k] >> 17) & 0x1ffffu) : 0u;
                sum += wk[j];
            }
            const uint32_t inc = wave_incl_sum(sum);
            const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            uint32_t run = inc - sum;
#pragma unroll
            for (int j = 0; j < kTQ / 64; ++j) {
                const uint32_t k = (uint32_t)lane * (kTQ / 64) + j;
                if (k < nit) L.own[k] = text_owner(run, wk[j], total);
                run += wk[j];
            }
        }
        __syncthreads();
        for (uint32_t k0 = 0; k0 < nit; k0 += 64) {
            const bool mine = k0 + (uint32_t)lane < nit && L.own[k0 + lane] == (uint8_t)w;
            for (uint64_t mm = __ballot(mine); mm; mm &= mm - 1) {
            const uint32_t k = k0 + (uint32_t)__builtin_ctzll(mm);
            if (uniform(*(volatile uint32_t*)&L.fail)) break;
            const uint64_t it = L.q[cur][k];
            const Seg seg{uniform((uint32_t)it & 0x1ffffu), uniform((uint32_t)(it >> 17) & 0x1ffffu)};
            const uint32_t d = uniform((uint32_t)(it >> 34) & 0xffffu);
            TBK_T(3, seg.len);
#ifdef BZ2MI_PHASES
            const unsigned long long ti0 = wall_clock64();
#endif
            if (seg.len <= (uint32_t)kTS) text_sort(Tl, n, sa, seg, d, bw, orig, W, L, dl);
            else text_partition(Tl, n, sa, spill, seg, d, bw, orig, W, L, cur ^ 1);
            TBK_T(11, seg.len);
#ifdef BZ2MI_PHASES
            TBK_COUNT(seg.len <= (uint32_t)kTS ? 12 : 13, wall_clock64() - ti0);
#endif
            }
        }
        __threadfence_block();
        __syncthreads();
    }
    __syncthreads();
#ifdef BZ2MI_PHASES
    tks = wall_clock64() - tk1;
#endif
    // ---- deferred groups (long repeats), every one before the copy steps:
    // isa (in spill, free after the sort phase) = the positions known now
    // (every sorted rotation; kNoIsa for the pair buckets (x, c) the copy
    // steps fill -- rank(x) >= s_big, rank(c) < rank(x) -- and kDefMark | g for
    // the members of deferred group g)
    const uint32_t ndef = uniform(L.ndef);
    uint32_t* isa = spill;
#ifdef BZ2MI_PHASES
    unsigned long long tkr = wall_clock64();
#endif
    if (ndef != 0 && !uniform(L.fail)) {
        // kNoIsa everywhere (coalesced), then the positions of the placed
        // rotations (scattered stores for about half of them: the copy
        // targets and the deferred members keep kNoIsa), 8 SA entries per
        // thread in flight
        {
            uint4* I4 = reinterpret_cast<uint4*>(isa);
            const uint4 none = make_uint4(kNoIsa, kNoIsa, kNoIsa, kNoIsa);
            for (uint32_t k = t; k < ((uint32_t)n + 3) / 4; k += FT) I4[k] = none;
        }
        __threadfence_block();
        __syncthreads();
        constexpr int U = 8;
        for (uint32_t k0 = t; k0 < (uint32_t)n; k0 += FT * U) {
            uint32_t v[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const uint32_t k = k0 + (uint32_t)j * FT;
                v[j] = k < (uint32_t)n ? ld_fresh(sa + k) : 0u;
            }
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const uint32_t k = k0 + (uint32_t)j * FT;
                if (k < (uint32_t)n) {
                    const uint32_t i = v[j] & 0x1ffffu;
                    const uint32_t rx = L.rank[Tl[i]], rc = L.rank[Tl[i + 1 < (uint32_t)n ? i + 1 : 0u]];
                    const bool implicit = rx >= s_big && rc < rx;
                    if (!implicit && !(v[j] & kUnres)) isa[i] = k;
                }
            }
        }
        __threadfence_block();
        __syncthreads();
        for (uint32_t g = t; g < ndef; g += FT) {
            const uint64_t e = dl[g];
            for (uint32_t k = 0; k < dg_len(e); ++k) isa[ld_fresh(sa + dg_start(e) + k) & 0x1ffffu] = kDefMark | g;
        }
        __threadfence_block();
        __syncthreads();
#ifdef BZ2MI_PHASES
        if (t == 0) atomicAdd(&g_tbk_res[0], wall_clock64() - tkr);
#endif
        text_resolve_all(Tl, n, sa, isa, dl, ndef, dl2, bw, orig, L);
        __threadfence_block();
        __syncthreads();
    }
#ifdef BZ2MI_PHASES
    tkr = wall_clock64() - tkr;
#endif
    // ---- copy steps.  The pair starts go to LDS (the per-wave scratch is
    // free now: 16 x 256 copy counters, then the starts).
    const uint32_t failed = uniform(L.fail);
    uint32_t* pstart = &L.w[0][0] + FW * 256;
    for (uint32_t j = t; j <= P; j += FT) pstart[j] = j < P ? pe_start(pl[j]) : (uint32_t)n;
    __syncthreads();
    // (a) the buckets before s_big were sorted whole (every pair explicit):
    // their copies are independent -- a wave per source bucket fills (x, ss)
    // for every copy-processed x at once
    if (!failed && s_big > s0) {
        uint32_t* C = &L.w[0][0] + w * 256;  // this wave's cursor per x (0xffffffff: not a target)
        for (uint32_t s = s0 + (uint32_t)w; s < s_big; s += FW) {
            const uint32_t ss = L.order[s];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t x = (uint32_t)lane * 4 + j, wq = ss >> 5, bit = ss & 31u;
                const uint32_t mw = L.mask[x][wq];
                uint32_t c = 0xffffffffu;
                if (L.rank[x] >= s_big && ((mw >> bit) & 1u)) {
                    uint32_t q = L.rowoff[x] + (uint32_t)__popc(mw & ((1u << bit) - 1u));
                    for (uint32_t r = 0; r < wq; ++r) q += (uint32_t)__popc(L.mask[x][r]);
                    c = pstart[q];
                }
                C[x] = c;
            }
            __builtin_amdgcn_wave_barrier();
            const uint32_t cs = L.cstart[ss], ce = L.cstart[ss + 1];
            for (uint32_t k0 = cs; k0 < ce; k0 += 64) {
                const uint32_t k = k0 + (uint32_t)lane;
                const uint32_t v = k < ce ? ld_fresh(sa + k) : 0u;
                const uint32_t i = v & 0x1ffffu;
                const uint32_t j = i ? i - 1 : (uint32_t)n - 1;
                const uint32_t x = k < ce ? (uint32_t)Tl[j] : 0u;
                const uint32_t bs = C[x];
                const bool tgt = k < ce && bs != 0xffffffffu;
                const uint64_t peers = wave_match8(x, tgt);
                if (tgt) {
                    const uint32_t below = (uint32_t)__popcll(peers & __lanemask_lt());
                    sa[bs + below] = j;
                    text_final(Tl, n, bs + below, j, bw, orig);
                }
                __builtin_amdgcn_wave_barrier();
                if (tgt && (peers & __lanemask_lt()) == 0) C[x] = bs + (uint32_t)__popcll(peers);
                __builtin_amdgcn_wave_barrier();
            }
        }
        __threadfence_block();
        __syncthreads();
    }
    // (b) the copy-processed buckets in ascending size: bucket ss is complete
    // (its sorted pair buckets, and (ss, c) for every earlier c from that
    // step's copy); it fills (x, ss) for every later x
    for (uint32_t s = s_big; s < 256 && !failed; ++s) {
        const uint32_t ss = L.order[s];
        TBK_T(5, s);
#ifdef BZ2MI_PHASES
        tk1 = wall_clock64();
#endif
        bool tg = false;
        if (t < 256) {
            const uint32_t x = (uint32_t)t, wq = ss >> 5, bit = ss & 31u;
            const uint32_t mw = L.mask[x][wq];
            tg = L.rank[x] > s && ((mw >> bit) & 1u);
            if (tg) {
                uint32_t j = L.rowoff[x] + (uint32_t)__popc(mw & ((1u << bit) - 1u));
                for (uint32_t q = 0; q < wq; ++q) j += (uint32_t)__popc(L.mask[x][q]);
                L.pcol[x] = pstart[j];
            }
            L.target[x] = tg ? 1 : 0;
        }
        // bucket ss is in order; (x, ss) = the rotations i-1 of it with
        // T[i-1] = x, in that order, for every later x.  Chunks of FW *
        // kCopyR * 64 rotations: every wave loads its kCopyR * 64 at once,
        // counts its targets per x, a scan over the waves gives each wave its
        // first slot per x (carried from chunk to chunk in pcol), then the
        // stable placement from registers.  A flagged source gives a flagged
        // target.
        if (__syncthreads_or(tg ? 1 : 0)) {
            uint32_t* C = &L.w[0][0] + w * 256;
            const uint32_t cs = L.cstart[ss], ce = L.cstart[ss + 1];
            for (uint32_t c0 = cs; c0 < ce; c0 += FW * kCopyR * 64) {
                const uint32_t w0 = c0 + (uint32_t)w * (kCopyR * 64);
                uint32_t jv[kCopyR], xv[kCopyR];
#pragma unroll
                for (int j = 0; j < 4; ++j) C[lane * 4 + j] = 0;
#pragma unroll
                for (int r = 0; r < kCopyR; ++r) {
                    const uint32_t k = w0 + (uint32_t)(r * 64 + lane);
                    jv[r] = k < ce ? ld_fresh(sa + k) : 0xffffffffu;
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int r = 0; r < kCopyR; ++r) {
                    const bool v = jv[r] != 0xffffffffu;
                    const uint32_t i = jv[r];
                    const uint32_t j = i ? i - 1 : (uint32_t)n - 1;
                    const uint32_t x = v ? (uint32_t)Tl[j] : 0u;
                    const bool tgt = v && L.target[x];
                    jv[r] = j;
                    xv[r] = tgt ? x : 0x100u;
                    if (tgt) atomicAdd(&C[x], 1u);
                }
                __syncthreads();
                if (t < 256) {
                    uint32_t run = L.pcol[t];
                    uint32_t* c0p = &L.w[0][0] + t;
                    for (int q = 0; q < FW; ++q) {
                        const uint32_t v = c0p[q * 256];
                        c0p[q * 256] = run;
                        run += v;
                    }
                    L.pcol[t] = run;
                }
                __syncthreads();
#pragma unroll
                for (int r = 0; r < kCopyR; ++r) {
                    const uint32_t x = xv[r];
                    const bool tgt = x != 0x100u;
                    const uint64_t peers = wave_match8(x, tgt);
                    const uint32_t bs = tgt ? C[x & 255u] : 0u;
                    if (tgt) {
                        const uint32_t below = (uint32_t)__popcll(peers & __lanemask_lt());
                        const uint32_t pos = bs + below;
                        sa[pos] = jv[r];
                        text_final(Tl, n, pos, jv[r], bw, orig);
                        if (below == 0) C[x] = bs + (uint32_t)__popcll(peers);
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        __threadfence_block();
        __syncthreads();
#ifdef BZ2MI_PHASES
        tkc += wall_clock64() - tk1;
#endif
    }
    __syncthreads();
#if BZ2MI_TEXT_FINALPASS
    if (!uniform(L.fail)) {
        // BWT bytes and origPtr from the finished SA, 4 positions per thread:
        // a 16-byte SA load and a 4-byte store
        for (uint32_t k0 = 4u * (uint32_t)t; k0 < (uint32_t)n; k0 += 4u * FT) {
            if (k0 + 4u <= (uint32_t)n) {
                const uint4 v = *reinterpret_cast<const uint4*>(sa + k0);
                const uint32_t ii[4] = {v.x & 0x1ffffu, v.y & 0x1ffffu, v.z & 0x1ffffu, v.w & 0x1ffffu};
                uint32_t word = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    word |= (uint32_t)bwt_byte(Tl, n, ii[j]) << (8 * j);
                    if (ii[j] == 0) *orig = k0 + (uint32_t)j;
                }
                *reinterpret_cast<uint32_t*>(out + k0) = word;
            } else {
                for (uint32_t k = k0; k < (uint32_t)n; ++k) {
                    const uint32_t i = ld_fresh(sa + k) & 0x1ffffu;
                    out[k] = bwt_byte(Tl, n, i);
                    if (i == 0) *orig = k;
                }
            }
        }
    }
#endif
    if (t == 0 && L.fail) redo[b] = 2u;
    TBK_T(6, L.fail);
#ifdef BZ2MI_PHASES
    if (t == 0) {
        atomicAdd(&g_tbk_stat[1], tks);
        atomicAdd(&g_tbk_stat[2], tkc);
        atomicAdd(&g_tbk_stat[8], 1ull);
        atomicAdd(&g_tbk_stat[9], wall_clock64() - tk0);
        atomicAdd(&g_tbk_stat[11], (unsigned long long)L.nflag);
        atomicAdd(&g_tbk_stat[14], tkr);
        if (ndef) {
            atomicAdd(&g_tbk_res[8], 1ull);
            atomicAdd(&g_tbk_res[2], (unsigned long long)ndef);
            atomicMax(&g_tbk_res[9], (unsigned long long)ndef);
        }
        atomicMax(&g_tbk_stat[15], wall_clock64() - tk0);
        for (int k = 3; k < 8; ++k) atomicAdd(&g_tbk_stat[k], (unsigned long long)L.stat[k]);
        atomicAdd(&g_tbk_x[0], (unsigned long long)L.stat[14]);
        atomicMax(&g_tbk_x[6], tkr);
        atomicMax(&g_tbk_x[7], tks);
        atomicAdd(&g_tbk_x[1], (unsigned long long)L.stat[15]);
        for (int k = 10; k < 14; ++k)
            if (k != 11) atomicAdd(&g_tbk_stat[k], (unsigned long long)L.stat[k]);
    }
#endif
}

// BZ2MI_TEXTBWT=0 (A/B): the text-like blocks go through the general path
__global__ void redo_all_kernel(uint32_t* redo, int nblocks) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nblocks && redo[b] == 1u) redo[b] = 2u;
}

// ---- kernel 4 (one launch per round, gridDim.y workgroups per block, each
// a slice of its list): the block's tie groups sorted by their next 8 bytes
// -- groups of <= kTieThread rotations one per thread, larger ones one per
// wave.  New ties go to the next round's list (tout_count zeroed before the
// launch); the last round hands them to the block's group list for prefix
// doubling.
__global__ __launch_bounds__(256) void bwt_tie_kernel(const uint8_t* __restrict__ blocks, size_t stride,
                                                      const uint32_t* __restrict__ lens,
                                                      uint32_t* __restrict__ sa_all, uint8_t* __restrict__ bwt_out,
                                                      uint32_t* __restrict__ orig_out,
                                                      const uint64_t* __restrict__ tin,
                                                      const uint32_t* __restrict__ tin_count,
                                                      uint64_t* __restrict__ tout, uint32_t* __restrict__ tout_count,
                                                      size_t tcap, Seg* __restrict__ grp_all,
                                                      uint32_t* __restrict__ ngroups, uint32_t* __restrict__ p2list,
                                                      uint32_t* __restrict__ p2count, int last, int nblocks,
                                                      int xcd_map) {
    __shared__ TieLds L;
    // xcd_map (900 KB blocks): a 1-D grid of 64 x ceil(blocks / 8) where XCD
    // x (workgroup w -> XCD w mod 8) takes the blocks b = x (mod 8), the 8
    // slices of one block after another, so the blocks in flight (whose text
    // the members gather from) are a few per XCD instead of every block of
    // the batch; else grid (blocks, slices)
    uint32_t b, ysl, nsl;
    if (xcd_map) {
        const uint32_t xcd = blockIdx.x & 7u, sl = blockIdx.x >> 3;
        b = (sl / (uint32_t)kTieSlices) * 8u + xcd;
        ysl = sl % (uint32_t)kTieSlices;
        nsl = (uint32_t)kTieSlices;
        if (b >= (uint32_t)nblocks) return;
    } else {
        b = blockIdx.x;
        ysl = blockIdx.y;
        nsl = gridDim.y;
    }
    const uint32_t nq = uniform(tin_count[b]);
    const uint32_t y0 = ysl * NT, ystep = nsl * NT;
    if (y0 >= nq) return;
    const int n = (int)uniform(lens[b]);
    const uint8_t* T = blocks + (size_t)b * stride;
    uint32_t* sa = sa_all + (size_t)b * stride;
    uint8_t* bw = bwt_out + (size_t)b * stride;
    const uint64_t* in = tin + (size_t)b * tcap;
    const GroupSink sink = last ? GroupSink{grp_all + (size_t)b * bwt_group_stride(stride), &ngroups[b], 0xffffffffu,
                                            p2list, p2count, b, nullptr, nullptr}
                                : GroupSink{nullptr, nullptr, 0, nullptr, nullptr, b, tout + (size_t)b * tcap,
                                            &tout_count[b]};
    auto unpack = [](uint64_t e, Seg& seg, uint32_t& d) {
        seg = Seg{(uint32_t)(e >> 22) & 0xfffffu, ((uint32_t)(e >> 13) & 511u) + 1u};
        d = (uint32_t)e & 0x1fffu;
    };
    // small groups: one per thread, 256 at a time; their members are loaded
    // by all threads at once (flattened) into LDS, then every thread ranks
    // its own group there
    for (uint32_t q0 = y0; q0 < nq; q0 += ystep) {
        const uint32_t q = q0 + threadIdx.x;
        uint32_t d = 0;
        Seg seg{0, 0};
        if (q < nq) unpack(in[q], seg, d);
        const uint32_t len = seg.len <= (uint32_t)kTieThread ? seg.len : 0u;
        uint32_t total;
        const uint32_t off = wg_excl_sum<NT>(len, L.tmp, &total);
        L.off[threadIdx.x] = off;
        L.gst[threadIdx.x] = seg.start;
        L.gdp[threadIdx.x] = d;
        __syncthreads();
        // 4 members per thread and step, their loads in flight together
        for (uint32_t m0 = 0; m0 < total; m0 += 4 * NT) {
            uint32_t pos[4], dep[4], iv[4];
            uint64_t kv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t m = m0 + j * NT + threadIdx.x;
                // owner group: the last g with off[g] <= m
                uint32_t lo = 0, hi = NT;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (L.off[mid] <= m) lo = mid;
                    else hi = mid;
                }
                pos[j] = L.gst[lo] + (m - L.off[lo]);
                dep[j] = L.gdp[lo];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) iv[j] = m0 + j * NT + threadIdx.x < total ? sa[pos[j]] : 0u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t p = iv[j] + dep[j];
                if (p >= (uint32_t)n) p %= (uint32_t)n;
                kv[j] = m0 + j * NT + threadIdx.x < total ? load8(T, n, p) : 0ull;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t m = m0 + j * NT + threadIdx.x;
                if (m < total) {
                    L.key[m] = kv[j];
                    L.idx[m] = iv[j];
                }
            }
        }
        __syncthreads();
        if (len) thread_rank_ties(T, n, sa, seg, d, off, sink, bw, orig_out + b, L);
        __syncthreads();
    }
    // large groups: one per wave (the list is scanned for them)
    for (uint32_t q0 = y0 + wave_id() * 64; q0 < nq; q0 += ystep) {
        const uint32_t q = q0 + lane_id();
        uint32_t d = 0;
        Seg seg{0, 0};
        if (q < nq) unpack(in[q], seg, d);
        uint64_t big = __ballot(q < nq && seg.len > (uint32_t)kTieThread);
        while (big) {
            const int l = __builtin_ctzll(big);
            big &= big - 1;
            const Seg sg{uniform(__shfl(seg.start, l)), uniform(__shfl(seg.len, l))};
            const uint32_t dd = uniform(__shfl(d, l));
            Scratch s{};
            s.sa = sa;
            wave_sort_any<0>(T, n, s, sg, dd, sink, bw, orig_out + b);
        }
    }
}

// ---- kernel 5: blocks with groups left: labels, prefix doubling, BWT bytes
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

// ==== prefix doubling over the whole grid (blocks beyond kBwtLdsText) ====
// Every group of every enlisted block sits in one flat list; each round is a
// few launches over all of them, so a block's doubling is spread over the
// chip instead of one workgroup (a 900 KB block of text with long repeated
// passages keeps ~50,000 groups for ~10 rounds: one workgroup per block left
// the double stage latency-bound at ~0.1-0.3 s per block).  Round r, h = 9 << r:
//   pairset / runend / decide  the repeat pairs of resolve_pairs, grid-wide
//                              (partner offsets tagged with the round, so the
//                              array is never cleared between rounds);
//   snap                       key[i] = label[i + h] << 20 | i for every member
//                              of every group (all reads before any relabel);
//   sort                       groups of 2 and <= 8 by one thread (ranks by
//                              counting), <= 512 by one wave (register bitonic),
//   large                      larger ones by one workgroup (LSD radix);
// subgroups go to the next round's lists.  Then the BWT bytes of the enlisted
// blocks.  Launches with nothing to do return at once (counters in G.ctr).
struct DblSlot {
    uint64_t* ka;
    uint64_t* kb;
    uint32_t* rank;
    uint32_t* pd;
    uint32_t* ne;
    uint32_t* va;  // radix values of large groups
    uint32_t* vb;
    uint32_t* cf;
};

__device__ __forceinline__ DblSlot dbl_slot(const DblGrid& G, uint32_t k) {
    const size_t S = (size_t)G.S;
    uint8_t* p = G.scratch + (size_t)k * G.per_slot;
    DblSlot d;
    d.ka = (uint64_t*)p; p += 8 * S;
    d.kb = (uint64_t*)p; p += 8 * S;
    d.rank = (uint32_t*)p; p += 4 * S;
    d.pd = (uint32_t*)p; p += 4 * S;
    d.ne = (uint32_t*)p; p += 4 * S;
    d.va = (uint32_t*)p; p += 4 * S;
    d.vb = (uint32_t*)p; p += 4 * S;
    d.cf = (uint32_t*)p;
    return d;
}

__device__ __forceinline__ void dbl_unpack(uint64_t e, uint32_t& k, uint32_t& start, uint32_t& len) {
    k = (uint32_t)(e >> 42);
    start = (uint32_t)(e >> 22) & 0xfffffu;
    len = ((uint32_t)(e >> 13) & 511u) + 1u;
}
__device__ __forceinline__ uint64_t dbl_large_pack(uint32_t k, uint32_t start, uint32_t len) {
    return ((uint64_t)k << 40) | ((uint64_t)start << 20) | len;
}

// wave-aggregated append (every lane of the wave that reaches it calls it)
__device__ __forceinline__ void dbl_append(bool want, uint64_t e, uint64_t* list, uint32_t* cnt) {
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(cnt, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, leader);
    if (want) list[base + (uint32_t)__popcll(m & __lanemask_lt())] = e;
}

// list appends staged in LDS and written with one global atomic per workgroup
// and step (the chip-wide list counters are single addresses)
constexpr int kDblStage = 2048;
struct DblOut {
    uint64_t buf[kDblStage];
    uint32_t n, nn, base;
    uint32_t cnt[2];
};
__device__ __forceinline__ void stage_push(DblOut& o, bool want, uint64_t e) {
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(&o.n, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, leader);
    if (want) o.buf[base + (uint32_t)__popcll(m & __lanemask_lt())] = e;
}
// every thread of the workgroup calls it
__device__ __forceinline__ void stage_flush(DblOut& o, uint64_t* list, uint32_t* cnt) {
    __syncthreads();
    if (threadIdx.x == 0) {
        o.nn = o.n;
        o.base = o.n ? atomicAdd(cnt, o.n) : 0u;
        o.n = 0;
    }
    __syncthreads();
    const uint32_t nn = o.nn, bb = o.base;
    for (uint32_t j = threadIdx.x; j < nn; j += NT) list[bb + j] = o.buf[j];
    __syncthreads();
}

// partner offsets and run ends recomputed in round r (c[6]): round 0 always;
// later while the last recomputation decided at least a ninth of its pairs.
// c[7] = 1 + the round they were last recomputed in (their tag); pairs still
// undecided keep their run end (a fact about the text), so every round
// re-checks the two rotations after it as the labels refine.
__device__ __forceinline__ bool dbl_pairs_on(const uint32_t* ctr, int r) {
    if (r == 0) return true;
    const uint32_t* c = ctr + kDblCtr * (r - 1);
    return c[6] != 0 && c[4] > 0 && c[3] >= c[4] / 8;
}

// the wave's first list index and the stride of a grid-wide wave loop
__device__ __forceinline__ uint32_t dbl_wave_base() { return (blockIdx.x * NW + (uint32_t)wave_id()) * 64u; }
__device__ __forceinline__ uint32_t dbl_wave_stride() { return gridDim.x * NW * 64u; }

// labels: every position its SA index (group members get their group's start
// next); partner offsets cleared
__global__ __launch_bounds__(256) void dbl_init_rank_kernel(DblGrid G) {
    const uint32_t P = *G.p2count;
    const uint32_t C = ((uint32_t)G.S + 4095u) / 4096u;
    for (uint32_t it = blockIdx.x; it < P * C; it += gridDim.x) {
        const uint32_t k = it / C, c = it - k * C;
        const uint32_t b = G.p2list[k];
        const uint32_t n = G.lens[b];
        const uint32_t lo = c * 4096u;
        if (lo >= n) continue;
        const uint32_t hi = min(n, lo + 4096u);
        const uint32_t* sa = G.sa_all + (size_t)b * G.stride;
        const DblSlot d = dbl_slot(G, k);
        uint32_t iv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t p = lo + (uint32_t)j * NT + threadIdx.x;
            iv[j] = p < hi ? sa[p] : 0u;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t p = lo + (uint32_t)j * NT + threadIdx.x;
            if (p < hi) {
                d.rank[iv[j]] = p;
                d.pd[p] = 0;
            }
        }
    }
}

// group labels; the phase-1 group lists become the round-0 lists
__global__ __launch_bounds__(256) void dbl_init_groups_kernel(DblGrid G) {
    __shared__ DblOut o;
    if (threadIdx.x == 0) o.n = 0;
    __syncthreads();
    const uint32_t P = *G.p2count;
    for (uint32_t k = blockIdx.x; k < P; k += gridDim.x) {
        const uint32_t b = G.p2list[k];
        const uint32_t ng = G.ngroups[b];
        const Seg* grp = G.grp_all + (size_t)b * bwt_group_stride(G.stride);
        const uint32_t* sa = G.sa_all + (size_t)b * G.stride;
        const DblSlot d = dbl_slot(G, k);
        for (uint32_t q0 = 0; q0 < ng; q0 += NT) {
            const uint32_t q = q0 + threadIdx.x;
            Seg sg{0, 0};
            if (q < ng) sg = grp[q];
            if (sg.len <= 64)
                for (uint32_t j = 0; j < sg.len; ++j) d.rank[sa[sg.start + j]] = sg.start;
            uint64_t big = __ballot(sg.len > 64);
            while (big) {
                const int l = __builtin_ctzll(big);
                big &= big - 1;
                const uint32_t st = uniform((uint32_t)__shfl((int)sg.start, l));
                const uint32_t ln = uniform((uint32_t)__shfl((int)sg.len, l));
                for (uint32_t j = lane_id(); j < ln; j += 64) d.rank[sa[st + j]] = st;
            }
            stage_push(o, q < ng && sg.len <= (uint32_t)kSmall, sq_pack(k, sg.start, max(sg.len, 1u), 0));
            stage_flush(o, G.list[0], &G.ctr[0]);
            dbl_append(q < ng && sg.len > (uint32_t)kSmall, dbl_large_pack(k, sg.start, sg.len), G.large[0],
                       &G.ctr[2]);
        }
    }
}

// partner offsets of the round's pairs, tagged with the round
__global__ __launch_bounds__(256) void dbl_pairset_kernel(DblGrid G, int r) {
    const bool on = dbl_pairs_on(G.ctr, r);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        G.ctr[kDblCtr * r + 6] = on ? 1u : 0u;
        G.ctr[kDblCtr * r + 7] = on ? (uint32_t)(r + 1) : r ? G.ctr[kDblCtr * (r - 1) + 7] : 0u;
    }
    if (!on) return;
    const uint32_t cin = G.ctr[kDblCtr * r];
    const uint32_t tag = (uint32_t)(r + 1) << 20;
    const uint64_t* list = G.list[0];
    for (uint32_t q = blockIdx.x * NT + threadIdx.x; q < cin; q += gridDim.x * NT) {
        uint32_t k, start, len;
        dbl_unpack(list[q], k, start, len);
        if (len != 2) continue;
        const uint32_t b = G.p2list[k];
        const uint32_t n = G.lens[b];
        const uint32_t* sa = G.sa_all + (size_t)b * G.stride;
        const uint32_t a = sa[start], c = sa[start + 1];
        const DblSlot d = dbl_slot(G, k);
        d.pd[a] = tag | (c > a ? c - a : c + n - a);
        d.pd[c] = tag | (a > c ? a - c : a + n - c);
    }
}

// run ends of equal partner offsets: wave w of chunk c scans the 1024
// positions of sub-range 4c + w from the right (cf = its first run end)
__global__ __launch_bounds__(256) void dbl_runend_kernel(DblGrid G, int r) {
    if (G.ctr[kDblCtr * r + 6] == 0) return;
    const uint32_t P = *G.p2count;
    const uint32_t C = ((uint32_t)G.S + 4095u) / 4096u;
    const int w = wave_id(), lane = lane_id();
    for (uint32_t it = blockIdx.x; it < P * C; it += gridDim.x) {
        const uint32_t k = it / C, c = it - k * C;
        const uint32_t b = G.p2list[k];
        const uint32_t n = G.lens[b];
        const uint32_t lo = c * 4096u + (uint32_t)w * 1024u;
        const DblSlot d = dbl_slot(G, k);
        if (lo >= n) {
            if (lane == 0) d.cf[c * 4 + w] = kNoEnd;
            continue;
        }
        const uint32_t hi = min(n, lo + 1024u);
        uint32_t carry = kNoEnd;
        for (uint32_t ts = lo + ((hi - 1 - lo) & ~63u);; ts -= 64) {
            const uint32_t p = ts + (uint32_t)lane;
            const bool valid = p < hi;
            bool bnd = false;
            if (valid) bnd = d.pd[p] != d.pd[p + 1 == n ? 0u : p + 1];
            const uint64_t B = __ballot(bnd);
            const uint64_t above = B & (~0ull << lane);
            if (valid) d.ne[p] = above ? ts + (uint32_t)__builtin_ctzll(above) : carry;
            if (B) carry = ts + (uint32_t)__builtin_ctzll(B);
            if (ts == lo) break;
        }
        if (lane == 0) d.cf[c * 4 + w] = carry;
    }
}

// pairs decided by the rotations after their run (resolve_pairs); the rest of
// the round's groups (blocks with h < n) go on to the other list
__global__ __launch_bounds__(256) void dbl_decide_kernel(DblGrid G, int r) {
    __shared__ DblOut o;
    uint32_t* cnt = G.ctr + kDblCtr * r;
    const uint32_t tag = cnt[7] << 20;  // the last recomputation's tag (0: none)
    const uint32_t cin = cnt[0];
    const uint32_t h = 9u << r;
    const int t = threadIdx.x;
    if (t == 0) {
        o.n = 0;
        o.cnt[0] = o.cnt[1] = 0;
    }
    __syncthreads();
    const uint64_t* lin = G.list[0];
    uint64_t* lout = G.list[1];
    uint32_t ndec = 0, nund = 0;
    for (uint32_t q0 = blockIdx.x * NT; q0 < cin; q0 += gridDim.x * NT) {
        const uint32_t q = q0 + (uint32_t)t;
        bool keep = false;
        uint64_t e = 0;
        if (q < cin) {
            e = lin[q];
            uint32_t k, start, len;
            dbl_unpack(e, k, start, len);
            const uint32_t b = G.p2list[k];
            const uint32_t n = G.lens[b];
            keep = h < n;
            uint32_t* sa = G.sa_all + (size_t)b * G.stride;
            const DblSlot d = dbl_slot(G, k);
            uint32_t a = 0, c = 0, off = 0;
            if (keep && len == 2 && tag) {
                a = sa[start];
                c = sa[start + 1];
                off = c > a ? c - a : c + n - a;
            }
            // a run end only where the pair was a pair at the last recomputation
            if (keep && len == 2 && tag && d.pd[a] == (tag | off)) {
                uint32_t end = d.ne[a];
                if (end == kNoEnd) {  // the run leaves a's sub-range: the next sub-range's first end (cyclic)
                    const uint32_t nsub = (n + 1023u) / 1024u;
                    uint32_t sj = a / 1024u;
                    for (uint32_t j = 0; j < nsub && end == kNoEnd; ++j) {
                        sj = sj + 1 == nsub ? 0u : sj + 1;
                        end = d.cf[sj];
                    }
                }
                bool a_first = a < c;  // no end anywhere: every position pairs at n / 2, equal rotations
                bool dec = true;
                if (end != kNoEnd) {
                    const uint32_t x = end + 1 == n ? 0u : end + 1;
                    const uint32_t y = x + off >= n ? x + off - n : x + off;
                    const uint32_t la = d.rank[x], lb = d.rank[y];
                    dec = la != lb;
                    a_first = la < lb;
                }
                if (dec) {
                    const uint32_t f = a_first ? a : c, l = a_first ? c : a;
                    sa[start] = f;
                    sa[start + 1] = l;
                    d.rank[f] = start;
                    d.rank[l] = start + 1;
                    keep = false;
                    ndec++;
                } else {
                    nund++;
                }
            }
        }
        stage_push(o, keep, e);
        stage_flush(o, lout, &cnt[1]);
    }
    atomicAdd(&o.cnt[0], ndec);
    atomicAdd(&o.cnt[1], nund);
    __syncthreads();
    if (t == 0) {
        if (o.cnt[0]) atomicAdd(&cnt[3], o.cnt[0]);
        if (o.cnt[1]) atomicAdd(&cnt[4], o.cnt[1]);
    }
}

// keys of every member of the round's groups, before any relabelling
__global__ __launch_bounds__(256) void dbl_snap_kernel(DblGrid G, int r) {
    const uint32_t* cnt = G.ctr + kDblCtr * r;
    const uint32_t c1 = cnt[1];
    const uint64_t* lmid = G.list[1];
    const uint32_t cl = cnt[2];
    const uint32_t h = 9u << r;
    const int lane = lane_id();
    for (uint32_t q0 = dbl_wave_base(); q0 < c1; q0 += dbl_wave_stride()) {
        const uint32_t q = q0 + (uint32_t)lane;
        uint32_t k = 0, start = 0, len = 0;
        if (q < c1) {
            dbl_unpack(lmid[q], k, start, len);
            if (h >= G.lens[G.p2list[k]]) len = 0;
        }
        if (len > 0 && len <= 32) {
            const uint32_t b = G.p2list[k];
            const uint32_t n = G.lens[b];
            const uint32_t* sa = G.sa_all + (size_t)b * G.stride;
            const DblSlot d = dbl_slot(G, k);
            for (uint32_t j = 0; j < len; ++j) {
                const uint32_t i = sa[start + j];
                const uint32_t ih = i + h >= n ? i + h - n : i + h;
                d.ka[start + j] = ((uint64_t)d.rank[ih] << kIdxBits) | i;
            }
        }
        uint64_t big = __ballot(len > 32);
        while (big) {
            const int l = __builtin_ctzll(big);
            big &= big - 1;
            const uint32_t kk = uniform((uint32_t)__shfl((int)k, l));
            const uint32_t st = uniform((uint32_t)__shfl((int)start, l));
            const uint32_t ln = uniform((uint32_t)__shfl((int)len, l));
            const uint32_t b = G.p2list[kk];
            const uint32_t n = G.lens[b];
            const uint32_t* sa = G.sa_all + (size_t)b * G.stride;
            const DblSlot d = dbl_slot(G, kk);
            for (uint32_t j = (uint32_t)lane; j < ln; j += 64) {
                const uint32_t i = sa[st + j];
                const uint32_t ih = i + h >= n ? i + h - n : i + h;
                d.ka[st + j] = ((uint64_t)d.rank[ih] << kIdxBits) | i;
            }
        }
    }
    for (uint32_t q = blockIdx.x; q < cl; q += gridDim.x) {
        const uint64_t e = G.large[r & 1][q];
        const uint32_t k = (uint32_t)(e >> 40), st = (uint32_t)(e >> 20) & 0xfffffu, ln = (uint32_t)e & 0xfffffu;
        const uint32_t b = G.p2list[k];
        const uint32_t n = G.lens[b];
        if (h >= n) continue;
        const uint32_t* sa = G.sa_all + (size_t)b * G.stride;
        const DblSlot d = dbl_slot(G, k);
        for (uint32_t j = threadIdx.x; j < ln; j += NT) {
            const uint32_t i = sa[st + j];
            const uint32_t ih = i + h >= n ? i + h - n : i + h;
            d.ka[st + j] = ((uint64_t)d.rank[ih] << kIdxBits) | i;
        }
    }
}

constexpr int kDblThread = 8;  // groups a thread sorts by counting

// groups of <= 512: sorted on their keys, relabelled, subgroups to the next
// round's list
__global__ __launch_bounds__(256) void dbl_sort_kernel(DblGrid G, int r) {
    __shared__ DblOut o;
    const uint32_t c1 = G.ctr[kDblCtr * r + 1];
    const uint64_t* lmid = G.list[1];
    uint64_t* lnext = G.list[0];
    uint32_t* nxt = G.ctr + kDblCtr * (r + 1);
    const uint32_t h = 9u << r;
    const int t = threadIdx.x;
    if (t == 0) o.n = 0;
    __syncthreads();
    for (uint32_t q0 = blockIdx.x * NT; q0 < c1; q0 += gridDim.x * NT) {
        const uint32_t q = q0 + (uint32_t)t;
        uint32_t k = 0, start = 0, len = 0;
        if (q < c1) {
            dbl_unpack(lmid[q], k, start, len);
            if (h >= G.lens[G.p2list[k]]) len = 0;
        }
        const bool thr = len > 0 && len <= (uint32_t)kDblThread;
        uint32_t* sa = nullptr;
        DblSlot d{};
        if (thr) {
            sa = G.sa_all + (size_t)G.p2list[k] * G.stride;
            d = dbl_slot(G, k);
        }
        bool pair_tie = false;
        if (thr && len == 2) {
            const uint64_t x = d.ka[start], y = d.ka[start + 1];
            const uint64_t f = x < y ? x : y, l = x < y ? y : x;
            const uint32_t fi = (uint32_t)f & ((1u << kIdxBits) - 1u), li = (uint32_t)l & ((1u << kIdxBits) - 1u);
            pair_tie = (f >> kIdxBits) == (l >> kIdxBits);
            sa[start] = fi;
            sa[start + 1] = li;
            d.rank[fi] = start;
            d.rank[li] = pair_tie ? start : start + 1;
        }
        stage_push(o, pair_tie, sq_pack(k, start, 2, 0));
        const bool cnt_sort = thr && len > 2;
        if (__ballot(cnt_sort)) {
            uint64_t kk[kDblThread];
#pragma unroll
            for (int j = 0; j < kDblThread; ++j) kk[j] = cnt_sort && (uint32_t)j < len ? d.ka[start + j] : ~0ull;
#pragma unroll
            for (int j = 0; j < kDblThread; ++j) {
                bool want = false;
                uint64_t ent = 0;
                if (cnt_sort && (uint32_t)j < len) {
                    const uint64_t kj = kk[j], gj = kj >> kIdxBits;
                    uint32_t pos = 0, lbl = 0, eq = 0;
#pragma unroll
                    for (int m = 0; m < kDblThread; ++m) {
                        pos += kk[m] < kj;
                        lbl += (kk[m] >> kIdxBits) < gj;
                        eq += (kk[m] >> kIdxBits) == gj;
                    }
                    const uint32_t i = (uint32_t)kj & ((1u << kIdxBits) - 1u);
                    sa[start + pos] = i;
                    d.rank[i] = start + lbl;
                    want = eq >= 2 && pos == lbl;
                    ent = sq_pack(k, start + lbl, max(eq, 1u), 0);
                }
                stage_push(o, want, ent);
            }
        }
        uint64_t big = __ballot(len > (uint32_t)kDblThread);
        while (big) {
            const int l = __builtin_ctzll(big);
            big &= big - 1;
            const uint32_t kw = uniform((uint32_t)__shfl((int)k, l));
            const uint32_t st = uniform((uint32_t)__shfl((int)start, l));
            const uint32_t ln = uniform((uint32_t)__shfl((int)len, l));
            const uint32_t b = G.p2list[kw];
            const DblSlot dw = dbl_slot(G, kw);
            Scratch s{};
            s.sa = G.sa_all + (size_t)b * G.stride;
            s.rank = dw.rank;
            s.ka = dw.ka;
            const GroupSink sink{nullptr, nullptr, 0, nullptr, nullptr, kw, lnext, &nxt[0], nullptr};
            wave_sort_any<1>(nullptr, (int)G.lens[b], s, Seg{st, ln}, 0, sink, nullptr, nullptr);
        }
        stage_flush(o, lnext, &nxt[0]);
    }
}

// groups of > 512: one workgroup each
__global__ __launch_bounds__(256) void dbl_large_kernel(DblGrid G, int r) {
    __shared__ BwtShared sh;
    const uint32_t cl = G.ctr[kDblCtr * r + 2];
    uint32_t* nxt = G.ctr + kDblCtr * (r + 1);
    const uint32_t h = 9u << r;
    for (uint32_t q = blockIdx.x; q < cl; q += gridDim.x) {
        const uint64_t e = G.large[r & 1][q];
        const uint32_t k = (uint32_t)(e >> 40), st = (uint32_t)(e >> 20) & 0xfffffu, ln = (uint32_t)e & 0xfffffu;
        const uint32_t b = G.p2list[k];
        if (h >= G.lens[b]) continue;
        const DblSlot d = dbl_slot(G, k);
        Scratch s{};
        s.sa = G.sa_all + (size_t)b * G.stride;
        s.rank = d.rank;
        s.ka = d.ka;
        s.kb = d.kb;
        s.va = d.va;
        s.vb = d.vb;
        uint64_t* lnext = G.large[(r + 1) & 1];
        uint64_t* list0 = G.list[0];
        wg_sort_group(s, Seg{st, ln}, sh, [&](Seg o) {
            if (o.len <= (uint32_t)kSmall) list0[atomicAdd(&nxt[0], 1u)] = sq_pack(k, o.start, o.len, 0);
            else lnext[atomicAdd(&nxt[2], 1u)] = dbl_large_pack(k, o.start, o.len);
        });
        __syncthreads();
    }
}

// BWT bytes and origPtr of the positions the doubling may have moved: the
// members of the phase-1 groups (phase 1 wrote every other position's byte)
__device__ __forceinline__ void dbl_emit_one(const uint8_t* T, uint32_t n, const uint32_t* sa, uint8_t* out,
                                             uint32_t* orig, uint32_t p) {
    const uint32_t i = sa[p];
    out[p] = bwt_byte(T, (int)n, i);
    if (i == 0) *orig = p;
}
__global__ __launch_bounds__(256) void dbl_emit_kernel(DblGrid G) {
    const uint32_t P = *G.p2count;
    for (uint32_t k = blockIdx.x; k < P; k += gridDim.x) {
        const uint32_t b = G.p2list[k];
        const uint32_t n = G.lens[b];
        const uint32_t ng = G.ngroups[b];
        const Seg* grp = G.grp_all + (size_t)b * bwt_group_stride(G.stride);
        const uint32_t* sa = G.sa_all + (size_t)b * G.stride;
        const uint8_t* T = G.blocks + (size_t)b * G.stride;
        uint8_t* out = G.bwt_out + (size_t)b * G.stride;
        uint32_t* orig = G.orig_out + b;
        for (uint32_t q0 = 0; q0 < ng; q0 += NT) {
            const uint32_t q = q0 + threadIdx.x;
            Seg sg{0, 0};
            if (q < ng) sg = grp[q];
            if (sg.len <= 64)
                for (uint32_t j = 0; j < sg.len; ++j) dbl_emit_one(T, n, sa, out, orig, sg.start + j);
            uint64_t big = __ballot(sg.len > 64);
            while (big) {
                const int l = __builtin_ctzll(big);
                big &= big - 1;
                const uint32_t st = uniform((uint32_t)__shfl((int)sg.start, l));
                const uint32_t ln = uniform((uint32_t)__shfl((int)sg.len, l));
                for (uint32_t j = lane_id(); j < ln; j += 64) dbl_emit_one(T, n, sa, out, orig, st + j);
            }
        }
    }
}

}  // namespace bz2mi
