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
// Group costs use the six 5-bit code lengths packed into 10-bit lanes of one
// 64-bit word, so a group's six costs are one add per symbol.  The payload is
// written MSB-first into a zeroed, byte-swapped 32-bit word image: every
// thread owns a contiguous bit range (plain stores inside, atomicOr on the two
// shared end words).
#include "common.hpp"
#include "kernels.hpp"

namespace bz2mi {

namespace {

constexpr int NT = 256;
constexpr int kMaxSel = 18432;  // >= ceil(900001/50): the 900 KB block mode

struct HufShared {
    int lens[kMaxTables][kMaxAlpha];
    int tf[kMaxTables][kMaxAlpha];
    int work[kMaxTables][kMaxAlpha];
    short idx[kMaxTables][kMaxAlpha];
    uint32_t codes[kMaxTables][kMaxAlpha];
    uint64_t pack[kMaxAlpha];
    uint8_t sel[kMaxSel];
    uint32_t tbits[kMaxTables];
    uint32_t tmp[NT / 64];
    uint64_t tmp64[NT / 64];
    uint64_t bc[4];
};

// ---- length-limited code length allocator (kernel.cpp:2652-2806), restated
__device__ int sig_bits(int x) {
    int n = 0;
    while (x > 0) {
        x >>= 1;
        n++;
    }
    return n;
}

__device__ int ha_first(const int* a, int len, int i, int nodesToMove) {
    const int limit = i;
    int k = len - 2;
    while (i >= nodesToMove && (a[i] % len) > limit) {
        k = i;
        i -= (limit - i + 1);
    }
    if (i < nodesToMove - 1) i = nodesToMove - 1;
    while (k > i + 1) {
        const int t = (i + k) >> 1;
        if ((a[t] % len) > limit) k = t;
        else i = t;
    }
    return k;
}

__device__ void ha_allocate(int* a, int len) {
    if (len <= 2) {
        if (len == 2) a[1] = 1;
        a[0] = 1;
        return;
    }
    // extended parent pointers
    a[0] += a[1];
    for (int head = 0, tail = 1, top = 2; tail < len - 1; tail++) {
        int t;
        if (top >= len || a[head] < a[top]) {
            t = a[head];
            a[head++] = tail;
        } else {
            t = a[top++];
        }
        if (top >= len || (head < tail && a[head] < a[top])) {
            t += a[head];
            a[head++] = tail + len;
        } else {
            t += a[top++];
        }
        a[tail] = t;
    }
    // nodes to relocate for the maximum length
    int r = len - 2;
    for (int d = 1; d < kMaxCodeLen - 1 && r > 1; d++) r = ha_first(a, len, r - 1, 0);
    if ((a[0] % len) >= r) {
        int firstNode = len - 2, nextNode = len - 1;
        for (int d = 1, avail = 2; avail > 0 && d < 64; d++) {
            const int lastNode = firstNode;
            firstNode = ha_first(a, len, lastNode - 1, 0);
            for (int i = avail - (lastNode - firstNode); i > 0; i--) a[nextNode--] = d;
            avail = (lastNode - firstNode) << 1;
        }
    } else {
        const int insertDepth = kMaxCodeLen - sig_bits(r - 1);
        int firstNode = len - 2, nextNode = len - 1;
        int d = (insertDepth == 1) ? 2 : 1;
        int left = (insertDepth == 1) ? r - 2 : r;
        for (int avail = d << 1; avail > 0 && d < 64; d++) {
            const int lastNode = firstNode;
            if (firstNode > r) firstNode = ha_first(a, len, lastNode - 1, r);
            int off = 0;
            if (d >= insertDepth) {
                const int cap = 1 << (d - insertDepth);
                off = left < cap ? left : cap;
            } else if (d == insertDepth - 1) {
                off = 1;
                if (a[firstNode] == lastNode) firstNode++;
            }
            for (int i = avail - (lastNode - firstNode + off); i > 0; i--) a[nextNode--] = d;
            left -= off;
            avail = (lastNode - firstNode + off) << 1;
        }
    }
}

__device__ __forceinline__ int table_count(int m) {
    return m >= 2400 ? 6 : m >= 1200 ? 5 : m >= 600 ? 4 : m >= 200 ? 3 : 2;
}

// code lengths of every table from sh.tf (generateHuffmanCodeLengths)
__device__ void build_lengths(HufShared& sh, int T, int alpha) {
    const int t = threadIdx.x;
    // rank sort of the unique keys (freq << 9) | symbol, all tables at once
    for (int e = t; e < T * alpha; e += NT) {
        const int q = e / alpha, s = e % alpha;
        const int key = (sh.tf[q][s] << 9) | s;
        int r = 0;
        for (int j = 0; j < alpha; ++j) r += ((sh.tf[q][j] << 9) | j) < key;
        sh.work[q][r] = key >> 9;
        sh.idx[q][r] = (short)s;
    }
    __syncthreads();
    if (t < T) ha_allocate(sh.work[t], alpha);
    __syncthreads();
    for (int e = t; e < T * alpha; e += NT) {
        const int q = e / alpha, r = e % alpha;
        sh.lens[q][sh.idx[q][r]] = sh.work[q][r];
    }
    __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(256) void huffman_kernel(
    const uint16_t* __restrict__ mtf, size_t mtf_stride, const uint32_t* __restrict__ mtf_len,
    const uint32_t* __restrict__ alpha_in, const uint32_t* __restrict__ seed,
    const uint32_t* __restrict__ present, const uint32_t* __restrict__ orig, int nblocks,
    uint32_t* __restrict__ payload, size_t payload_words, uint64_t* __restrict__ payload_bits) {
    __shared__ HufShared sh;
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    const int t = threadIdx.x;
    const int m = (int)uniform(mtf_len[b]);
    const int alpha = (int)uniform(alpha_in[b]);
    const int T = table_count(m);
    const int nsel = (m + kGroupRun - 1) / kGroupRun;
    const uint16_t* X = mtf + (size_t)b * mtf_stride;
    const uint32_t* F = seed + (size_t)b * kMaxAlpha;
    uint32_t* out = payload + (size_t)b * payload_words;

    for (int e = t; e < kMaxTables * kMaxAlpha; e += NT) (&sh.lens[0][0])[e] = 0;
    __syncthreads();
    // ---- seeds (serial; int32 wrap-around like the reference's int array)
    if (t == 0) {
        int32_t remaining = m;
        int lowEnd = -1;
        for (int i = 0; i < T; i++) {
            const int32_t target = remaining / (T - i);
            const int lowStart = lowEnd + 1;
            int32_t actual = 0;
            while (actual < target && lowEnd < alpha - 1) actual = (int32_t)((uint32_t)actual + F[++lowEnd]);
            if (lowEnd > lowStart && i != 0 && i != T - 1 && ((T - i) % 2) == 0)
                actual = (int32_t)((uint32_t)actual - F[lowEnd--]);
            for (int j = 0; j < alpha; j++)
                if (j < lowStart || j > lowEnd) sh.lens[i][j] = kHighCost;
            remaining = (int32_t)((uint32_t)remaining - (uint32_t)actual);
        }
    }
    __syncthreads();
    // ---- 4 refinement passes
    for (int it = 3; it >= 0; --it) {
        for (int s = t; s < alpha; s += NT) {
            uint64_t p = 0;
            for (int q = 0; q < T; ++q) p |= (uint64_t)sh.lens[q][s] << (10 * q);
            sh.pack[s] = p;
        }
        for (int e = t; e < kMaxTables * kMaxAlpha; e += NT) (&sh.tf[0][0])[e] = 0;
        __syncthreads();
        for (int g = t; g < nsel; g += NT) {
            const int g0 = g * kGroupRun, g1 = min(g0 + kGroupRun, m);
            uint64_t c = 0;
            for (int i = g0; i < g1; ++i) c += sh.pack[X[i]];
            int best = 0;
            uint32_t bestCost = (uint32_t)(c & 1023u);
            for (int q = 1; q < T; ++q) {
                const uint32_t cq = (uint32_t)((c >> (10 * q)) & 1023u);
                if (cq < bestCost) {
                    bestCost = cq;
                    best = q;
                }
            }
            sh.sel[g] = (uint8_t)best;
        }
        __syncthreads();
        for (int i = t; i < m; i += NT) atomicAdd(&sh.tf[sh.sel[i / kGroupRun]][X[i]], 1);
        __syncthreads();
        build_lengths(sh, T, alpha);
    }
    // ---- canonical codes per table (thread q), table bit sizes
    if (t < T) {
        const int* Lq = sh.lens[t];
        int mn = 32, mx = 0;
        for (int j = 0; j < alpha; ++j) {
            mn = Lq[j] < mn ? Lq[j] : mn;
            mx = Lq[j] > mx ? Lq[j] : mx;
        }
        uint32_t code = 0;
        for (int Ln = mn; Ln <= mx; Ln++) {
            for (int j = 0; j < alpha; j++)
                if ((Lq[j] & 0xff) == Ln) sh.codes[t][j] = ((uint32_t)Ln << 24) | code++;
            code <<= 1;
        }
        uint32_t bits = 5;
        int cur = Lq[0];
        for (int j = 0; j < alpha; ++j) {
            const int d = Lq[j] - cur;
            bits += 2u * (uint32_t)(d < 0 ? -d : d) + 1u;
            cur = Lq[j];
        }
        sh.tbits[t] = bits;
    }
    // ---- selector MTF positions (serial), header size
    if (t == NT - 1) {
        uint8_t lst[kMaxTables] = {0, 1, 2, 3, 4, 5};
        uint64_t sb = 0;
        for (int g = 0; g < nsel; ++g) {
            const int v = sh.sel[g];
            int pos = 0;
            while (pos < kMaxTables - 1 && lst[pos] != v) pos++;
            for (int q = pos; q > 0; q--) lst[q] = lst[q - 1];
            lst[0] = (uint8_t)v;
            sb += (uint64_t)pos + 1;
        }
        sh.bc[0] = sb;
    }
    __syncthreads();
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
    const uint64_t selbits = uniform64(sh.bc[0]);
    const uint64_t data0 = 24 + mapbits + 3 + 15 + selbits + tabbits;
    // data size: per-thread contiguous symbol ranges
    const int per = (m + NT - 1) / NT;
    const int i0 = min(t * per, m), i1 = min(i0 + per, m);
    uint64_t mybits = 0;
    for (int i = i0; i < i1; ++i) mybits += sh.codes[sh.sel[i / kGroupRun]][X[i]] >> 24;
    uint64_t allbits;
    const uint64_t myoff = data0 + wg_excl_sum64<NT>(mybits, sh.tmp64, &allbits);
    const uint64_t total = data0 + allbits;
    // zero the payload image
    const uint64_t nwords = (total + 31) / 32 + 1;
    for (uint64_t w = t; w < nwords; w += NT) out[w] = 0;
    __syncthreads();
    // ---- header parts (thread 0): origPtr, symbol map, T, nsel, selectors
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
        uint8_t lst[kMaxTables] = {0, 1, 2, 3, 4, 5};
        for (int g = 0; g < nsel; ++g) {
            const int v = sh.sel[g];
            int pos = 0;
            while (pos < kMaxTables - 1 && lst[pos] != v) pos++;
            for (int q = pos; q > 0; q--) lst[q] = lst[q - 1];
            lst[0] = (uint8_t)v;
            s.put(pos + 1, ((1u << pos) - 1u) << 1);  // writeUnary: pos ones, then a zero
        }
        s.finish();
    }
    // tables: thread 64+q writes table q
    if (t >= 64 && t < 64 + T) {
        const int q = t - 64;
        uint64_t at = 24 + mapbits + 18 + selbits;
        for (int r = 0; r < q; ++r) at += sh.tbits[r];
        BitSink s;
        s.init(out, at);
        const int* Lq = sh.lens[q];
        int cur = Lq[0];
        s.put(5, (uint32_t)cur);
        for (int j = 0; j < alpha; ++j) {
            const int L = Lq[j];
            int d = L - cur;
            const uint32_t v = d > 0 ? 2u : 3u;  // 10 = +1, 11 = -1
            if (d < 0) d = -d;
            while (d-- > 0) s.put(2, v);
            s.put(1, 0);
            cur = L;
        }
        s.finish();
    }
    // data: every thread its range
    {
        BitSink s;
        s.init(out, myoff);
        for (int i = i0; i < i1; ++i) {
            const uint32_t cs = sh.codes[sh.sel[i / kGroupRun]][X[i]];
            s.put((int)(cs >> 24), cs & 0xffffffu);
        }
        s.finish();
    }
    if (t == 0) payload_bits[b] = total;
}

}  // namespace bz2mi
