// Multi-table Huffman coding and bit packing of one block per workgroup.
//
// Restates HuffmanStageEncoder (reference kernel.cpp:3064-3096) and the
// symbol map / origPtr writes of close_block (kernel.cpp:3116-3118):
//   seeds      generateHuffmanOptimisationSeeds  kernel.cpp:2859-2893
//   4x refine  optimiseSelectorsAndHuffmanTables kernel.cpp:2895-2951
//   lengths    generateHuffmanCodeLengths        kernel.cpp:2835-2857
//              + the in-place length-limited allocator kernel.cpp:2652-2806
//   codes      assignHuffmanCodeSymbols          kernel.cpp:2953-2989
//   tables     writeSelectorsAndHuffmanTables    kernel.cpp:2991-3041
//   data       writeBlockData                    kernel.cpp:3043-3062
//
// Work split (256 threads = 4 waves):
//  * the two inherently serial pieces -- seed boundaries and the allocator --
//    run with their array spread over one wave's registers (WaveList): every
//    access is a readlane (or a lane-select write) with a uniform index
//    instead of a dependent LDS round trip; tables run on different waves;
//  * a refinement pass reads each group's 50 symbols once (dword loads),
//    adds the six packed 10-bit costs per symbol, picks the table and counts
//    the symbols into that table's frequencies;
//  * canonical codes, selector MTF positions (from per-table last-use scans)
//    and table deltas are computed in parallel;
//  * the data is packed in tiles of 2048 symbols: a workgroup scan of the
//    code lengths places every thread's 8 codes into an LDS window of the
//    output, which is flushed as whole words (the partial word carried on).
// The payload is a byte-swapped 32-bit word image of the MSB-first stream.
#include "common.hpp"
#include "kernels.hpp"

namespace bz2mi {

BZ2MI_PHASE_TABLE(g_huf_phase)

namespace {

// BZ2MI_HUF_NT: threads per workgroup (a multiple of 64); with 6 or more
// waves every table's code lengths are built on a wave of its own
#ifndef BZ2MI_HUF_NT
#define BZ2MI_HUF_NT 256
#endif
constexpr int NT = BZ2MI_HUF_NT;
constexpr int NW = NT / 64;
// BZ2MI_HUF_TS: symbols per thread of a data tile (8 or 4; 4 halves the
// output window, so the workgroup fits 8 per CU)
#ifndef BZ2MI_HUF_TS
#define BZ2MI_HUF_TS 8
#endif
constexpr int TS = BZ2MI_HUF_TS;
static_assert(TS == 8 || TS == 4, "tile symbols per thread");
constexpr int kTileSyms = TS * NT;                   // symbols per data tile
constexpr int kWinWords = kTileSyms * kMaxCodeLen / 32 + 2;

struct HufShared {
    uint8_t lens[kMaxTables][kMaxAlpha + 2];
    uint64_t pack[kMaxAlpha];
    union {
        struct {
            int tf[kMaxTables][kMaxAlpha];
            int work[kMaxTables][kMaxAlpha];
        } opt;
        struct {
            uint32_t codes[kMaxTables][kMaxAlpha];
            uint32_t win[2][kWinWords];
        } out;
    } u;
    uint32_t run[kMaxTables][kMaxCodeLen + 2];
    uint32_t tbits[kMaxTables];
    int lo[kMaxTables], hi[kMaxTables];
    int last[NW][kMaxTables];
    uint32_t tmp[NW];
};

// ---- an int array of up to 320 entries held in one wave's registers: entry
// i is lane i%64 of register i/64.  Indices must be wave-uniform.
struct WaveList {
    int r0, r1, r2, r3, r4;

    __device__ __forceinline__ void load(const int* src, int n) {
        const int l = lane_id();
        r0 = l < n ? src[l] : 0;
        r1 = l + 64 < n ? src[l + 64] : 0;
        r2 = l + 128 < n ? src[l + 128] : 0;
        r3 = l + 192 < n ? src[l + 192] : 0;
        r4 = l + 256 < n ? src[l + 256] : 0;
    }
    // branch-free: read the lane of all five registers, pick with scalar selects
    __device__ __forceinline__ int get(int i) const {
        const int k = i >> 6, l = i & 63;
        const int v0 = __builtin_amdgcn_readlane(r0, l), v1 = __builtin_amdgcn_readlane(r1, l);
        const int v2 = __builtin_amdgcn_readlane(r2, l), v3 = __builtin_amdgcn_readlane(r3, l);
        const int v4 = __builtin_amdgcn_readlane(r4, l);
        return k == 0 ? v0 : k == 1 ? v1 : k == 2 ? v2 : k == 3 ? v3 : v4;
    }
    __device__ __forceinline__ void set(int i, int v) {
        const int k = i >> 6;
        const bool me = lane_id() == (i & 63);
        r0 = (me && k == 0) ? v : r0;
        r1 = (me && k == 1) ? v : r1;
        r2 = (me && k == 2) ? v : r2;
        r3 = (me && k == 3) ? v : r3;
        r4 = (me && k == 4) ? v : r4;
    }
    // entries (lo, hi] = v
    __device__ __forceinline__ void fill(int lo, int hi, int v) {
        const int l = lane_id();
        r0 = (l > lo && l <= hi) ? v : r0;
        r1 = (l + 64 > lo && l + 64 <= hi) ? v : r1;
        r2 = (l + 128 > lo && l + 128 <= hi) ? v : r2;
        r3 = (l + 192 > lo && l + 192 <= hi) ? v : r3;
        r4 = (l + 256 > lo && l + 256 <= hi) ? v : r4;
    }
};

// ---- length-limited code length allocator (kernel.cpp:2652-2806), restated
// over a WaveList.  All values are wave-uniform.
__device__ __forceinline__ int sig_bits(int x) { return x > 0 ? 32 - __clz(x) : 0; }

// x % len for the entries the allocator takes it of: parent pointers (< 2 len)
// and depths (< 64); anything else takes the general path.
__device__ __forceinline__ int mod_len(int x, int len) {
    if ((unsigned)x < 2u * (unsigned)len) return x >= len ? x - len : x;
    return x % len;
}

// first() (kernel.cpp:2661-2686) with every probe of its exponential and
// binary searches answered from bit masks: am holds mod_len of every entry,
// one compare per register gives the predicate "parent above limit" for all
// 320 entries at once (five 64-bit masks in SGPRs), and the searches run on
// the scalar unit with the reference's exact probe sequence -- no readlane
// round trips per probe, and no assumption that the predicate is monotone.
__device__ __forceinline__ int ha_first(const WaveList& am, int len, int i, int nodesToMove) {
    (void)len;
    const int limit = i;
    const uint64_t p0 = __ballot(am.r0 > limit), p1 = __ballot(am.r1 > limit), p2 = __ballot(am.r2 > limit);
    const uint64_t p3 = __ballot(am.r3 > limit), p4 = __ballot(am.r4 > limit);
    auto P = [&](int j) -> bool {
        const int q = j >> 6;
        const uint64_t m = q == 0 ? p0 : q == 1 ? p1 : q == 2 ? p2 : q == 3 ? p3 : p4;
        return (m >> (j & 63)) & 1ull;
    };
    // Fast path: when the predicate over [lo, limit] is true on a suffix that
    // reaches `limit` (the parent pointers are nondecreasing, so it is, bar
    // ~3% of calls), the searches end at the suffix's first index.  Checked
    // against first() on 47M calls of random allocations; anything else
    // takes the probe sequence below.
    const int lo = nodesToMove > 0 ? nodesToMove : 0;
    if (lo <= limit && P(limit)) {
        int hf = -1, lt = 1 << 30;
#pragma unroll
        for (int w = 4; w >= 0; --w) {
            const uint64_t pw = w == 0 ? p0 : w == 1 ? p1 : w == 2 ? p2 : w == 3 ? p3 : p4;
            const int a = lo - 64 * w, b = limit - 64 * w;
            uint64_t rng = 0;
            if (b >= 0 && a <= 63) rng = (b >= 63 ? ~0ull : ((2ull << b) - 1ull)) & (a <= 0 ? ~0ull : (~0ull << a));
            const uint64_t f = ~pw & rng, tr = pw & rng;
            if (hf < 0 && f) hf = 64 * w + 63 - __clzll((long long)f);
            if (tr) lt = 64 * w + __builtin_ctzll(tr);
        }
        if (hf < lt) return hf < 0 ? lo : hf + 1;
    }
    int k = len - 2;
    while (i >= nodesToMove && P(i)) {
        k = i;
        i -= (limit - i + 1);
    }
    if (i < nodesToMove - 1) i = nodesToMove - 1;
    while (k > i + 1) {
        const int t = (i + k) >> 1;
        if (P(t)) k = t;
        else i = t;
    }
    return k;
}

// the entries' values mod len (first()'s `array[i] % length`), lane-parallel
__device__ __forceinline__ WaveList mod_list(const WaveList& a, int len) {
    WaveList m;
    m.r0 = mod_len(a.r0, len);
    m.r1 = mod_len(a.r1, len);
    m.r2 = mod_len(a.r2, len);
    m.r3 = mod_len(a.r3, len);
    m.r4 = mod_len(a.r4, len);
    return m;
}

// Phase 1 of the allocator: the extended parent pointers of the in-place
// two-queue Huffman construction (kernel.cpp:2686-2712).  The sequential
// loop picks items (sorted leaves A[top..], internal nodes IW[head..tail))
// smallest first -- leaf on ties -- and pairs consecutive picks into the next
// internal node.  Every internal node made from items >= x weighs >= 2x, so
// all known items <= 2x are picked, in merged order, before any new one: a
// wave merges up to 64 of them per step (ranks by binary search across
// lanes) and forms their pairs at once.  The result is the reference's array:
// A[k] = parent of internal node k (+len when it was the second pick) for
// k < len-2, A[len-2] = root weight, A[len-1] = largest leaf.
// 64-bit compare-exchange step of a bitonic half-cleaner at lane distance J:
// the lower lane of each pair keeps the smaller key
template <int J>
__device__ __forceinline__ uint64_t half_clean(uint64_t k) {
    const uint32_t lo = xor_lanes<J>((uint32_t)k), hi = xor_lanes<J>((uint32_t)(k >> 32));
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    const bool lower = (lane_id() & J) == 0;
    return lower ? (k < o ? k : o) : (k > o ? k : o);
}

// lane l gets lane 63 - l
__device__ __forceinline__ uint32_t lane_reverse(uint32_t v) {
    constexpr int kRowMirror = 0x140;  // row_mirror: lane 15 - l inside each row of 16
    return xor_lanes<16>(xor_lanes<32>(dpp_mov<kRowMirror>(v)));
}

__device__ void ha_parents(int* A, int* IW, int len) {
    const int lane = lane_id();
    constexpr int INF = 0x7fffffff;
    if (lane == 0) IW[0] = A[0] + A[1];
    int top = 2, head = 0, tail = 1;
    while (tail < len - 1) {
        const int li = top + lane, ii = head + lane;
        const int lw = li < len ? A[li] : INF;
        const int iw = ii < tail ? IW[ii] : INF;
        const int x = min(__builtin_amdgcn_readlane(lw, 0), __builtin_amdgcn_readlane(iw, 0));
        const int limit = 2 * x;  // weights sum to <= 900,001
        uint64_t bL = __ballot(lw <= limit), bI = __ballot(iw <= limit);
        int E = (__popcll(bL) + __popcll(bI)) & ~1;
        if (E > 64) E = 64;
        if (E == 0) {
            // only x itself is <= 2x: it pairs with the next smallest known item
            bL = __ballot(lw != INF);
            bI = __ballot(iw != INF);
            E = 2;
        }
        const int cL = __popcll(bL), cI = __popcll(bI);
        // merged order of the candidates: keys weight << 8 | internal << 7 |
        // queue position (leaves before internal nodes of equal weight, each
        // list in its own order), the leaves ascending in lanes, the internal
        // nodes reversed behind them -- a bitonic sequence whose 64 smallest
        // one min step and six half-cleaners (DPP / permlane) put in order
        const uint64_t kl = lane < cL ? ((uint64_t)(uint32_t)lw << 8) | (uint64_t)lane : ~0ull;
        const uint64_t ki = lane < cI ? ((uint64_t)(uint32_t)iw << 8) | 0x80u | (uint64_t)lane : ~0ull;
        const uint64_t kr = ((uint64_t)lane_reverse((uint32_t)(ki >> 32)) << 32) | lane_reverse((uint32_t)ki);
        uint64_t k = kl < kr ? kl : kr;
        k = half_clean<32>(k);
        k = half_clean<16>(k);
        k = half_clean<8>(k);
        k = half_clean<4>(k);
        k = half_clean<2>(k);
        k = half_clean<1>(k);
        // lane p holds merged position p; positions < E are picked, pairs
        // (2q, 2q+1) form internal node tail + q
        const bool take = lane < E;
        const bool isI = (k >> 7) & 1u;
        const int w = (int)(uint32_t)(k >> 8);
        if (take && isI) A[head + (int)(k & 63u)] = tail + (lane >> 1) + ((lane & 1) ? len : 0);
        const int uI = __popcll(__ballot(take && isI));
        const int uL = (E - uI);
        const int wn = (int)xor_lanes<1>((uint32_t)w);
        if (take && (lane & 1) == 0) IW[tail + (lane >> 1)] = w + wn;
        top += uL;
        head += uI;
        tail += E >> 1;
    }
    if (lane == 0) A[len - 2] = IW[len - 2];
}

// Phase 2 (kernel.cpp:2714-2806): depths from the parent pointers, limited to
// kMaxCodeLen, written from the top of the array.
__device__ void ha_depths(WaveList& a, int len) {
    WaveList am = mod_list(a, len);  // kept equal to mod_len of every entry of a
    int r = len - 2;
    for (int d = 1; d < kMaxCodeLen - 1 && r > 1; d++) r = ha_first(am, len, r - 1, 0);
    if (mod_len(a.get(0), len) >= r) {
        int firstNode = len - 2, nextNode = len - 1;
        for (int d = 1, avail = 2; avail > 0 && d < 64; d++) {
            const int lastNode = firstNode;
            firstNode = ha_first(am, len, lastNode - 1, 0);
            const int cnt = avail - (lastNode - firstNode);
            if (cnt > 0) {
                a.fill(nextNode - cnt, nextNode, d);
                am.fill(nextNode - cnt, nextNode, mod_len(d, len));
                nextNode -= cnt;
            }
            avail = (lastNode - firstNode) << 1;
        }
    } else {
        const int insertDepth = kMaxCodeLen - sig_bits(r - 1);
        int firstNode = len - 2, nextNode = len - 1;
        int d = (insertDepth == 1) ? 2 : 1;
        int left = (insertDepth == 1) ? r - 2 : r;
        for (int avail = d << 1; avail > 0 && d < 64; d++) {
            const int lastNode = firstNode;
            if (firstNode > r) firstNode = ha_first(am, len, lastNode - 1, r);
            int off = 0;
            if (d >= insertDepth) {
                const int cap = 1 << (d - insertDepth);
                off = left < cap ? left : cap;
            } else if (d == insertDepth - 1) {
                off = 1;
                if (a.get(firstNode) == lastNode) firstNode++;
            }
            const int cnt = avail - (lastNode - firstNode + off);
            if (cnt > 0) {
                a.fill(nextNode - cnt, nextNode, d);
                am.fill(nextNode - cnt, nextNode, mod_len(d, len));
                nextNode -= cnt;
            }
            left -= off;
            avail = (lastNode - firstNode + off) << 1;
        }
    }
}

// Phase 2 without the serial level walk when no length limit applies: the
// depth of every internal node by pointer jumping over the parent pointers
// (P, Dd: two LDS arrays of >= len ints, free after ha_parents), the internal
// nodes per depth I_d by ballots, and the leaves per depth L_d = 2 I_(d-1) -
// I_d assigned from the top of the sorted array, as allocateNodeLengths
// (kernel.cpp:2722-2739) assigns them level by level.  Returns false (and
// leaves `a` untouched) when the deepest leaf would pass kMaxCodeLen, the
// reference's relocation case (findNodesToRelocate's test, :2714-2720 /
// :2807-2811), which ha_depths then runs.
__device__ bool ha_depths_fast(WaveList& a, int len, int* P, int* Dd) {
    const int lane = lane_id();
    const int root = len - 2;
    int dep[5];
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        const int k = r * 64 + lane;
        const int v = r == 0 ? a.r0 : r == 1 ? a.r1 : r == 2 ? a.r2 : r == 3 ? a.r3 : a.r4;
        dep[r] = k < root ? 1 : 0;
        if (k < len) {
            P[k] = k < root ? mod_len(v, len) : k;
            Dd[k] = dep[r];
        }
    }
    __builtin_amdgcn_wave_barrier();
    // jumps register by register: a node read later in a round may already
    // have jumped, which only speeds it up -- each (P, Dd) pair is read
    // between the two writes of another register's update, never across them
    for (int round = 0; round < 12; ++round) {
        bool moved = false;
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            const int k = r * 64 + lane;
            if (k < len) {
                const int p = P[k];
                const int pp = P[p], dp = Dd[p];
                moved |= pp != p;
                dep[r] += dp;
                Dd[k] = dep[r];
                P[k] = pp;
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (!__ballot(moved)) break;
    }
    // deepest internal node (node 0 in a Huffman tree; the maximum for safety)
    int dmax = 0;
#pragma unroll
    for (int r = 0; r < 5; ++r)
        if (r * 64 + lane < len - 1) dmax = max(dmax, dep[r]);
    dmax = (int)__builtin_amdgcn_readlane((int)wave_incl_max((uint32_t)dmax), 63);
    if (dmax + 1 > kMaxCodeLen) return false;
    // internal nodes per depth: lane d holds I_d
    int icnt = 0;
    for (int d = 1; d <= dmax; ++d) {
        int id = 0;
#pragma unroll
        for (int r = 0; r < 5; ++r) id += __popcll(__ballot(r * 64 + lane < len - 1 && dep[r] == d));
        icnt = lane == d ? id : icnt;
    }
    // leaves: depth 1 + #{d : cum_d <= rank from the top}, cum_d = sum of
    // L_e = 2 I_(e-1) - I_e over e <= d (I_0 = 1, the root)
#pragma unroll
    for (int r = 0; r < 5; ++r) dep[r] = 1;
    int iprev = 1, cum = 0;
    for (int d = 1; d <= dmax; ++d) {
        const int id = __builtin_amdgcn_readlane(icnt, d);
        cum += 2 * iprev - id;
        iprev = id;
#pragma unroll
        for (int r = 0; r < 5; ++r) dep[r] += (len - 1 - (r * 64 + lane)) >= cum ? 1 : 0;
    }
    a.r0 = lane < len ? dep[0] : a.r0;
    a.r1 = lane + 64 < len ? dep[1] : a.r1;
    a.r2 = lane + 128 < len ? dep[2] : a.r2;
    a.r3 = lane + 192 < len ? dep[3] : a.r3;
    a.r4 = lane + 256 < len ? dep[4] : a.r4;
    return true;
}

// BZ2MI_HUF_FASTDEPTHS (default): ha_depths_fast before the serial walk
#ifndef BZ2MI_HUF_FASTDEPTHS
#define BZ2MI_HUF_FASTDEPTHS 1
#endif
constexpr bool kHufFastDepths = BZ2MI_HUF_FASTDEPTHS != 0;
__device__ __forceinline__ int table_count(int m) {
    return m >= 2400 ? 6 : m >= 1200 ? 5 : m >= 600 ? 4 : m >= 200 ? 3 : 2;
}

// table q is handled by wave q % NW
__device__ __forceinline__ bool my_table(int q) { return q % NW == wave_id(); }

// ascending register bitonic sort of 64*E keys over one wave, striped
// (element e of lane l is item e*64 + l)
template <int E>
__device__ __forceinline__ void wave_bitonic32(uint32_t (&key)[8]) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= 64 * E; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j >= 1; j >>= 1) {
            if (j >= 64) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
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
                for (int e = 0; e < E; ++e) {
                    const uint32_t o = xor_lanes_rt(key[e], j);  // DPP / permlane (j folds to a constant)
                    const bool asc = ((e * 64 + lane) & k) == 0;
                    const bool lower = (lane & j) == 0;
                    key[e] = (lower == asc) ? min(key[e], o) : max(key[e], o);
                }
            }
        }
    }
}

// code lengths of table q from sh.u.opt.tf[q] (generateHuffmanCodeLengths,
// kernel.cpp:2835-2857) on one wave: sort the unique keys (freq << 9) | symbol,
// run the allocator on the sorted frequencies, scatter depths to symbols
__device__ void build_table(HufShared& sh, int q, int alpha, bool stamp = false) {
    const int lane = lane_id();
    int* tf = sh.u.opt.tf[q];
    int* A = sh.u.opt.work[q];
    uint32_t key[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int j = e * 64 + lane;
        key[e] = j < alpha ? ((uint32_t)tf[j] << 9) | (uint32_t)j : 0xffffffffu;
    }
    if (alpha <= 64) wave_bitonic32<1>(key);
    else if (alpha <= 128) wave_bitonic32<2>(key);
    else if (alpha <= 256) wave_bitonic32<4>(key);
    else wave_bitonic32<8>(key);
    BZ2MI_PHASE(g_huf_phase, 13, stamp);
#pragma unroll
    for (int e = 0; e < 5; ++e)
        if (e * 64 + lane < alpha) A[e * 64 + lane] = (int)(key[e] >> 9);
    WaveList a;
    if (alpha > 2) {
        ha_parents(A, tf, alpha);  // (tf[q] is free: keys are in registers)
        BZ2MI_PHASE(g_huf_phase, 14, stamp);
        a.load(A, alpha);
        // (A and tf are free again: the pointers are in registers)
        if (!kHufFastDepths || !ha_depths_fast(a, alpha, A, tf)) ha_depths(a, alpha);
        BZ2MI_PHASE(g_huf_phase, 15, stamp);
    } else {
        a.load(A, alpha);
        a.fill(-1, alpha - 1, 1);  // (alpha >= 3 in practice: RUNA, RUNB, EOB)
    }
    const int v[5] = {a.r0, a.r1, a.r2, a.r3, a.r4};
#pragma unroll
    for (int e = 0; e < 5; ++e)
        if (e * 64 + lane < alpha) sh.lens[q][key[e] & 511u] = (uint8_t)v[e];
}

// code lengths of every table, table q on wave q%NW
__device__ void build_lengths(HufShared& sh, int T, int alpha, bool stamp = false) {
    for (int q = 0; q < T; ++q)
        if (my_table(q)) build_table(sh, q, alpha, stamp && q == 0);
    __syncthreads();
}

// exclusive max-scan over the workgroup of six per-thread values (-1 = none)
__device__ __forceinline__ void wg_excl_max6(int (&v)[kMaxTables], HufShared& sh) {
    const int lane = lane_id(), w = wave_id();
    int inc[kMaxTables];
#pragma unroll
    for (int u = 0; u < kMaxTables; ++u) {
        int x = v[u];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, d);
            if (lane >= d) x = max(x, y);
        }
        inc[u] = x;
        if (lane == 63) sh.last[w][u] = x;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kMaxTables; ++u) {
        int base = -1;
        for (int k = 0; k < w; ++k) base = max(base, sh.last[k][u]);
        const int prev = __shfl_up(inc[u], 1);
        v[u] = max(base, lane ? prev : -1);
    }
    __syncthreads();
}

// MTF position of selector value v given each table's last use (-1: unused)
// before it: the list holds the used tables most recent first, then the
// unused ones ascending (valueToFront, kernel.cpp:3009-3013).
__device__ __forceinline__ int selector_pos(const int (&last)[kMaxTables], int v) {
    int lv = last[0];
#pragma unroll
    for (int u = 1; u < kMaxTables; ++u) lv = (v == u) ? last[u] : lv;
    int pos = 0;
    if (lv >= 0) {
#pragma unroll
        for (int u = 0; u < kMaxTables; ++u) pos += last[u] > lv;
    } else {
#pragma unroll
        for (int u = 0; u < kMaxTables; ++u) pos += (last[u] >= 0) | (u < v);
    }
    return pos;
}

__device__ __forceinline__ void note_use(int (&last)[kMaxTables], int v, int g) {
#pragma unroll
    for (int u = 0; u < kMaxTables; ++u) last[u] = (v == u) ? g : last[u];
}

// index of the best (cheapest, first on ties) of T packed 10-bit costs
__device__ __forceinline__ int best_table(uint64_t c, int T) {
    int best = 0;
    uint32_t bestCost = (uint32_t)(c & 1023u);
    for (int q = 1; q < T; ++q) {
        const uint32_t cq = (uint32_t)((c >> (10 * q)) & 1023u);
        if (cq < bestCost) {
            bestCost = cq;
            best = q;
        }
    }
    return best;
}

}  // namespace

int huffman_phases(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_huf_phase), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

// 7 workgroups per CU (22.6 KB of LDS each): the length builds are serial, latency-bound wave code,
// so more resident blocks pay for a few spilled registers
#ifndef BZ2MI_HUF_WGS
#define BZ2MI_HUF_WGS 7
#endif
int huffman_threads() { return NT; }

__global__ __launch_bounds__(NT, BZ2MI_HUF_WGS) void huffman_kernel(
    const uint16_t* __restrict__ mtf, size_t mtf_stride, const uint32_t* __restrict__ mtf_len,
    const uint32_t* __restrict__ alpha_in, const uint32_t* __restrict__ seed,
    const uint32_t* __restrict__ present, const uint32_t* __restrict__ orig, int nblocks,
    uint32_t* __restrict__ payload, size_t payload_words, uint64_t* __restrict__ payload_bits) {
    __shared__ HufShared sh;
    // selectors: dynamic LDS sized by the launcher for its block size
    // (ceil((S + 1) / 50) bytes: 1.8 KB at S = 90,000, 18 KB at 900,000)
    extern __shared__ uint8_t sel[];
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    const int t = threadIdx.x, lane = lane_id();
    const int m = (int)uniform(mtf_len[b]);
    const int alpha = (int)uniform(alpha_in[b]);
    const int T = table_count(m);
    const int nsel = (m + kGroupRun - 1) / kGroupRun;
    const uint16_t* X = mtf + (size_t)b * mtf_stride;
    uint32_t* out = payload + (size_t)b * payload_words;
    [[maybe_unused]] const bool stamp = b == nblocks / 2;
    BZ2MI_PHASE(g_huf_phase, 0, stamp);

    // ---- seeds: symbol ranges of roughly equal frequency per table (wave 0,
    // frequencies in registers; int32 wrap-around like the reference's int array)
    if (wave_id() == 0) {
        WaveList F;
        F.load(reinterpret_cast<const int*>(seed + (size_t)b * kMaxAlpha), alpha);
        int32_t remaining = m;
        int lowEnd = -1;
        for (int i = 0; i < T; i++) {
            const int32_t target = remaining / (T - i);
            const int lowStart = lowEnd + 1;
            int32_t actual = 0;
            while (actual < target && lowEnd < alpha - 1)
                actual = (int32_t)((uint32_t)actual + (uint32_t)F.get(++lowEnd));
            if (lowEnd > lowStart && i != 0 && i != T - 1 && ((T - i) % 2) == 0)
                actual = (int32_t)((uint32_t)actual - (uint32_t)F.get(lowEnd--));
            if (lane == 0) {
                sh.lo[i] = lowStart;
                sh.hi[i] = lowEnd;
            }
            remaining = (int32_t)((uint32_t)remaining - (uint32_t)actual);
        }
    }
    __syncthreads();
    for (int e = t; e < T * alpha; e += NT) {
        const int q = e / alpha, j = e - q * alpha;
        sh.lens[q][j] = (j < sh.lo[q] || j > sh.hi[q]) ? kHighCost : 0;
    }
    __syncthreads();
    BZ2MI_PHASE(g_huf_phase, 1, stamp);

    // ---- 4 refinement passes: choose tables, count, rebuild lengths
    for (int it = 3; it >= 0; --it) {
        for (int s = t; s < alpha; s += NT) {
            uint64_t p = 0;
            for (int q = 0; q < T; ++q) p |= (uint64_t)sh.lens[q][s] << (10 * q);
            sh.pack[s] = p;
        }
        for (int e = t; e < kMaxTables * kMaxAlpha; e += NT) (&sh.u.opt.tf[0][0])[e] = 0;
        __syncthreads();
        for (int g = t; g < nsel; g += NT) {
            const int g0 = g * kGroupRun;
            if (g0 + kGroupRun <= m) {
                // 50 symbols = 25 dwords (g0 * 2 bytes is a multiple of 4)
                const uint32_t* W = reinterpret_cast<const uint32_t*>(X + g0);
                uint32_t w[kGroupRun / 2];
#pragma unroll
                for (int k = 0; k < kGroupRun / 2; ++k) w[k] = W[k];
                uint64_t c = 0;
#pragma unroll
                for (int k = 0; k < kGroupRun / 2; ++k) c += sh.pack[w[k] & 0xffffu] + sh.pack[w[k] >> 16];
                const int best = best_table(c, T);
                sel[g] = (uint8_t)best;
                int* tf = sh.u.opt.tf[best];
#pragma unroll
                for (int k = 0; k < kGroupRun / 2; ++k) {
                    atomicAdd(&tf[w[k] & 0xffffu], 1);
                    atomicAdd(&tf[w[k] >> 16], 1);
                }
            } else {
                uint64_t c = 0;
                for (int i = g0; i < m; ++i) c += sh.pack[X[i]];
                const int best = best_table(c, T);
                sel[g] = (uint8_t)best;
                for (int i = g0; i < m; ++i) atomicAdd(&sh.u.opt.tf[best][X[i]], 1);
            }
        }
        __syncthreads();
        BZ2MI_PHASE(g_huf_phase, 2 + 2 * (3 - it), stamp);
        build_lengths(sh, T, alpha, stamp && it == 0);
        BZ2MI_PHASE(g_huf_phase, 3 + 2 * (3 - it), stamp);
    }

    // ---- canonical codes (assignHuffmanCodeSymbols): codes of length L start
    // at first[L] = (first[L-1] + count[L-1]) << 1 and go up in symbol order.
    // Table q on wave q%4; table bit size 5 + sum(2|delta| + 1).
    for (int q = 0; q < T; ++q) {
        if (!my_table(q)) continue;
        const uint8_t* Lq = sh.lens[q];
        uint32_t cnt = 0, dbits = 0;  // lane L: number of codes of length L
        for (int j0 = 0; j0 < alpha; j0 += 64) {
            const int j = j0 + lane;
            const bool valid = j < alpha;
            const int L = valid ? Lq[j] : 0;
            const int d = (valid && j) ? L - Lq[j - 1] : 0;
            dbits += valid ? 2u * (uint32_t)(d < 0 ? -d : d) + 1u : 0u;
#pragma unroll
            for (int k = 1; k <= kMaxCodeLen; ++k) {
                const uint32_t c = (uint32_t)__popcll(__ballot(valid && L == k));
                if (lane == k) cnt += c;
            }
        }
        dbits = wave_sum(dbits);
        const uint64_t nz = __ballot(cnt != 0);
        const int mn = nz ? __ffsll((long long)nz) - 1 : kMaxCodeLen + 1;
        uint32_t code = 0, myfirst = 0;
        for (int L = 0; L <= kMaxCodeLen; ++L) {
            if (lane == L) myfirst = code;
            if (L >= mn) code = (code + (uint32_t)__builtin_amdgcn_readlane((int)cnt, L)) << 1;
        }
        if (lane < kMaxCodeLen + 2) sh.run[q][lane] = myfirst;
        if (lane == 0) sh.tbits[q] = 5u + dbits;
        for (int j0 = 0; j0 < alpha; j0 += 64) {
            const int j = j0 + lane;
            const bool valid = j < alpha;
            const int L = valid ? Lq[j] : 0;
            const uint64_t peers = wave_match8((uint32_t)L, valid);
            const uint32_t rank = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
            const uint32_t base = valid ? sh.run[q][L] : 0u;
            if (valid) sh.u.out.codes[q][j] = ((uint32_t)L << 24) | (base + rank);
            if (valid && (peers >> lane) == 1ull) sh.run[q][L] = base + rank + 1u;  // highest peer
        }
    }

    // ---- selector MTF positions: every thread walks its contiguous range
    // knowing, per table, the last use before the range (max-scan)
    const int sper = (nsel + NT - 1) / NT;
    const int s0 = min(t * sper, nsel), s1 = min(s0 + sper, nsel);
    int last0[kMaxTables];
#pragma unroll
    for (int u = 0; u < kMaxTables; ++u) last0[u] = -1;
    for (int g = s0; g < s1; ++g) note_use(last0, sel[g], g);
    wg_excl_max6(last0, sh);  // (its barriers also complete the codes)
    uint32_t mysel = 0;
    {
        int last[kMaxTables];
#pragma unroll
        for (int u = 0; u < kMaxTables; ++u) last[u] = last0[u];
        for (int g = s0; g < s1; ++g) {
            const int v = sel[g];
            mysel += (uint32_t)selector_pos(last, v) + 1u;
            note_use(last, v, g);
        }
    }
    BZ2MI_PHASE(g_huf_phase, 10, stamp);
    uint32_t selbits;
    const uint32_t seloff = wg_excl_sum<NT>(mysel, sh.tmp, &selbits);
    // symbol map size
    const uint32_t* P = present + (size_t)b * 8;
    uint32_t used16 = 0;
    for (int q = 0; q < 16; ++q) {
        const uint32_t half = (P[q >> 1] >> ((q & 1) * 16)) & 0xffffu;
        if (half) used16 |= 1u << q;
    }
    const uint64_t mapbits = 16 + 16 * (uint64_t)__popc(used16);
    uint64_t tabbits = 0;
    for (int q = 0; q < T; ++q) tabbits += sh.tbits[q];
    const uint64_t sel0 = 24 + mapbits + 3 + 15;
    const uint64_t tab0 = sel0 + selbits;
    const uint64_t data0 = tab0 + tabbits;
    const uint64_t dword0 = data0 >> 5;
    // zero the words before the data (written with atomicOr on shared edges)
    for (uint64_t w = t; w <= dword0; w += NT) out[w] = 0;
    __syncthreads();

    // ---- header (thread 0): origPtr, symbol map, T, nsel
    if (t == 0) {
        BitSink s;
        s.init(out, 0);
        s.put(24, orig[b]);
        s.put(16, __brev(used16) >> 16);
        for (int q = 0; q < 16; ++q)
            if (used16 & (1u << q)) {
                const uint32_t half = (P[q >> 1] >> ((q & 1) * 16)) & 0xffffu;
                s.put(16, __brev(half) >> 16);  // symbol 16q+j at bit j from the front
            }
        s.put(3, (uint32_t)T);
        s.put(15, (uint32_t)nsel);
        s.finish();
    }
    // ---- selectors (writeUnary: pos ones, then a zero), every thread its range
    {
        BitSink s;
        s.init(out, sel0 + seloff);
        int last[kMaxTables];
#pragma unroll
        for (int u = 0; u < kMaxTables; ++u) last[u] = last0[u];
        for (int g = s0; g < s1; ++g) {
            const int v = sel[g];
            const int pos = selector_pos(last, v);
            s.put(pos + 1, ((1u << pos) - 1u) << 1);
            note_use(last, v, g);
        }
        s.finish();
    }
    // ---- tables (delta-coded lengths): table q on wave q%4, one symbol per
    // lane -- its |delta| pairs (10 = +1, 11 = -1) and the closing 0 -- placed
    // by a wave scan of the piece lengths
    for (int q = 0; q < T; ++q) {
        if (!my_table(q)) continue;
        uint64_t at = tab0;
        for (int r = 0; r < q; ++r) at += sh.tbits[r];
        const uint8_t* Lq = sh.lens[q];
        if (lane == 0) put_bits_or(out, at, 5, Lq[0]);
        at += 5;
        for (int j0 = 0; j0 < alpha; j0 += 64) {
            const int j = j0 + lane;
            const bool valid = j < alpha;
            const int d = (valid && j) ? (int)Lq[j] - (int)Lq[j - 1] : 0;
            const int ad = d < 0 ? -d : d;
            const uint32_t nb = valid ? 2u * (uint32_t)ad + 1u : 0u;
            const uint32_t inc = wave_incl_sum(nb);
            const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            if (valid) {
                const uint64_t pat = d > 0 ? 0xaaaaaaaaaaaaaaaaull : ~0ull;
                const uint64_t v = (pat & ((1ull << (2 * ad)) - 1ull)) << 1;
                const uint64_t p = at + inc - nb;
                if (nb > 32) {
                    put_bits_or(out, p, (int)nb - 32, (uint32_t)(v >> 32));
                    put_bits_or(out, p + nb - 32, 32, (uint32_t)v);
                } else {
                    put_bits_or(out, p, (int)nb, (uint32_t)v);
                }
            }
            at += total;
        }
    }
    BZ2MI_PHASE(g_huf_phase, 11, stamp);

    // ---- data (writeBlockData): tiles of 2048 symbols, 8 per thread, packed
    // into an LDS window of the stream and flushed as whole words
    for (int k = t; k < 2 * kWinWords; k += NT) (&sh.u.out.win[0][0])[k] = 0;
    __syncthreads();
    uint64_t bit0 = data0;  // stream position of the current tile
    int cur = 0;
    for (int base = 0; base < m; base += kTileSyms) {
        const int i0 = base + TS * t;
        uint32_t sym[TS];
        if (i0 + TS <= m) {
            if constexpr (TS == 8) {
                const uint4 v = *reinterpret_cast<const uint4*>(X + i0);
                const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    sym[2 * k] = vv[k] & 0xffffu;
                    sym[2 * k + 1] = vv[k] >> 16;
                }
            } else {
                const uint2 v = *reinterpret_cast<const uint2*>(X + i0);
                sym[0] = v.x & 0xffffu;
                sym[1] = v.x >> 16;
                sym[2] = v.y & 0xffffu;
                sym[3] = v.y >> 16;
            }
        } else {
#pragma unroll
            for (int k = 0; k < TS; ++k) sym[k] = i0 + k < m ? X[i0 + k] : 0u;
        }
        uint32_t cs[TS];
        uint32_t mybits = 0;
#pragma unroll
        for (int k = 0; k < TS; ++k) {
            const int i = i0 + k;
            cs[k] = i < m ? sh.u.out.codes[sel[(unsigned)i / kGroupRun]][sym[k]] : 0u;
            mybits += cs[k] >> 24;
        }
        uint32_t tilebits;
        const uint32_t off = wg_excl_sum<NT>(mybits, sh.tmp, &tilebits);
        uint32_t* win = sh.u.out.win[cur];
        const uint64_t w0 = bit0 >> 5;
        {
            const uint32_t p = (uint32_t)(bit0 & 31) + off;
            uint32_t wi = p >> 5;
            int nacc = (int)(p & 31);
            uint64_t acc = 0;
#pragma unroll
            for (int k = 0; k < TS; ++k) {
                const int L = (int)(cs[k] >> 24);
                acc |= ((uint64_t)(cs[k] & 0xffffffu) << (63 - L) << 1) >> nacc;
                nacc += L;
                if (nacc >= 32) {
                    atomicOr(&win[wi], (uint32_t)(acc >> 32));
                    acc <<= 32;
                    nacc -= 32;
                    wi++;
                }
            }
            if (nacc > 0) atomicOr(&win[wi], (uint32_t)(acc >> 32));
        }
        __syncthreads();
        const uint64_t bit1 = bit0 + tilebits;
        const int nfull = (int)((bit1 >> 5) - w0);
        uint32_t* nxt = sh.u.out.win[cur ^ 1];
        for (int k = t; k <= nfull; k += NT) {
            const uint32_t v = win[k];
            win[k] = 0;
            if (k == nfull) nxt[0] = v;  // partial word carried into the next tile
            else if (w0 + k == dword0) atomicOr(&out[w0 + k], bswap32(v));
            else out[w0 + k] = bswap32(v);
        }
        bit0 = bit1;
        cur ^= 1;
        // (the next tile's scan barriers order these window writes)
    }
    __syncthreads();
    // last partial word, and a zero word after the stream
    if (t == 0) {
        const uint64_t wl = bit0 >> 5;
        const uint32_t v = sh.u.out.win[cur][0];
        if (wl == dword0) atomicOr(&out[wl], bswap32(v));
        else out[wl] = bswap32(v);
        if (bit0 & 31) out[wl + 1] = 0;
        payload_bits[b] = bit0;
    }
#ifdef BZ2MI_PHASES
    __syncthreads();
    BZ2MI_PHASE(g_huf_phase, 12, stamp);
#endif
}

}  // namespace bz2mi
