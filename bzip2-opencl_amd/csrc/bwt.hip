// Per-block cyclic BWT on the device: one 256-thread workgroup per block,
// prefix doubling over the block's rotations with a workgroup LSD radix sort.
//
// Replaces DivSufSortBWT (reference kernel.cpp:2429-2456, with the wrap byte
// of close_block kernel.cpp:3113).  The rotation order of an aperiodic block is
// unique, so any correct sort reproduces the reference; equal rotations of a
// periodic block stay in index order (SURVEY H2/H8 decision), which every
// stable pass below preserves.
//
// Data layout (HBM): blocks at `stride` bytes apart; per workgroup slot a
// scratch region of 40*S bytes (SA, rank, two key/value ping-pong buffers and
// two active-slot lists).  Blocks are pulled from a device work counter, so
// the grid is sized to the chip, not to the batch.
#include "common.hpp"
#include "kernels.hpp"

namespace bz2mi {

namespace {

constexpr int NT = 256;
constexpr int NW = NT / 64;
constexpr int kRankBits = 20;  // S <= 2^20

struct BwtShared {
    uint32_t hist[256];
    uint32_t base[256];
    uint32_t wcnt[NW][256];
    uint32_t tmp[NW * 2];
    uint64_t tmp64[NW];
    uint64_t tmp64b[NW];
    uint32_t bcast[4];
};

struct Scratch {
    uint32_t* sa;
    uint32_t* rank;
    uint64_t* ka;
    uint64_t* kb;
    uint32_t* va;
    uint32_t* vb;
    uint32_t* slot;
    uint32_t* slot2;
};

__device__ Scratch carve(uint8_t* base, int S) {
    Scratch s;
    uint8_t* p = base;
    s.ka = (uint64_t*)p; p += 8ull * S;
    s.kb = (uint64_t*)p; p += 8ull * S;
    s.sa = (uint32_t*)p; p += 4ull * S;
    s.rank = (uint32_t*)p; p += 4ull * S;
    s.va = (uint32_t*)p; p += 4ull * S;
    s.vb = (uint32_t*)p; p += 4ull * S;
    s.slot = (uint32_t*)p; p += 4ull * S;
    s.slot2 = (uint32_t*)p; p += 4ull * S;
    return s;
}

// OR ^ AND over all keys: the bits that vary, so constant digits are skipped.
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

// One stable counting pass on digit (key >> shift) & 255.
__device__ void radix_pass(const uint64_t* kin, const uint32_t* vin, uint64_t* kout, uint32_t* vout,
                           int m, int shift, BwtShared& sh) {
    const int t = threadIdx.x;
    sh.hist[t] = 0;
    for (int w = 0; w < NW; ++w) sh.wcnt[w][t] = 0;
    __syncthreads();
    for (int i = t; i < m; i += NT) atomicAdd(&sh.hist[(kin[i] >> shift) & 255u], 1u);
    __syncthreads();
    uint32_t total;
    uint32_t ex = wg_excl_sum<NT>(sh.hist[t], sh.tmp, &total);
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

// Sort (k,v)[0..m) by key bits [0, bits); returns true if the result is in
// the second buffers (kb, vb).
__device__ bool radix_sort(uint64_t* ka, uint32_t* va, uint64_t* kb, uint32_t* vb, int m, int bits,
                           BwtShared& sh) {
    uint64_t vary;
    key_span(ka, m, sh, &vary);
    bool flip = false;
    for (int shift = 0; shift < bits; shift += 8) {
        if (((vary >> shift) & 255u) == 0) continue;
        if (!flip) radix_pass(ka, va, kb, vb, m, shift, sh);
        else radix_pass(kb, vb, ka, va, m, shift, sh);
        flip = !flip;
    }
    return flip;
}

// After sorting the active list: place values in SA, relabel groups by the SA
// index of their first element, and compact the non-singleton entries into
// `nslot`.  `slot` == nullptr means the identity list (round 0).
__device__ int regroup(const uint64_t* key, const uint32_t* val, const uint32_t* slot, uint32_t* nslot,
                       int m, Scratch& s, BwtShared& sh) {
    const int t = threadIdx.x;
    uint32_t carry_start = 0;
    uint32_t kept = 0;
    for (int tile = 0; tile < m; tile += NT) {
        const int k = tile + t;
        const bool valid = k < m;
        bool start = false, next_start = true;
        uint32_t sl = 0;
        if (valid) {
            const uint64_t me = key[k];
            start = (k == 0) || key[k - 1] != me;
            next_start = (k + 1 == m) || key[k + 1] != me;
            sl = slot ? slot[k] : (uint32_t)k;
            s.sa[sl] = val[k];
        }
        uint32_t tot;
        uint32_t gstart = wg_incl_max<NT>(start ? (uint32_t)k : 0u, sh.tmp, &tot);
        if (gstart < carry_start) gstart = carry_start;
        // the group's label is the SA index of its first element
        const bool keep = valid && !(start && next_start);
        uint32_t cnt;
        const uint32_t off = wg_excl_sum<NT>(keep ? 1u : 0u, sh.tmp, &cnt);
        if (valid) {
            const uint32_t gslot = slot ? slot[gstart] : gstart;
            s.rank[val[k]] = gslot;
            if (keep) nslot[kept + off] = sl;
        }
        kept += cnt;
        carry_start = carry_start > tot ? carry_start : tot;
        __syncthreads();
    }
    return (int)kept;
}

__device__ void bwt_block(const uint8_t* __restrict__ T, int n, uint8_t* __restrict__ out,
                          uint32_t* __restrict__ orig, Scratch& s, BwtShared& sh) {
    const int t = threadIdx.x;
    // round 0: 4-byte cyclic prefixes
    for (int i = t; i < n; i += NT) {
        uint32_t k = 0;
        int j = i;
        for (int q = 0; q < 4; ++q) {
            k = (k << 8) | T[j];
            j = (j + 1 == n) ? 0 : j + 1;
        }
        s.ka[i] = k;
        s.va[i] = (uint32_t)i;
    }
    __syncthreads();
    bool flip = radix_sort(s.ka, s.va, s.kb, s.vb, n, 32, sh);
    int m = regroup(flip ? s.kb : s.ka, flip ? s.vb : s.va, nullptr, s.slot, n, s, sh);
    __syncthreads();
    uint32_t* cur = s.slot;
    uint32_t* nxt = s.slot2;
    for (long long h = 4; m > 0 && h < n; h <<= 1) {
        // snapshot keys: (label of i, label of i+h) -- all reads before any relabel
        for (int k = t; k < m; k += NT) {
            const uint32_t i = s.sa[cur[k]];
            uint32_t ih = (uint32_t)((i + h) % n);
            s.ka[k] = ((uint64_t)s.rank[i] << kRankBits) | s.rank[ih];
            s.va[k] = i;
        }
        __syncthreads();
        flip = radix_sort(s.ka, s.va, s.kb, s.vb, m, 2 * kRankBits, sh);
        m = regroup(flip ? s.kb : s.ka, flip ? s.vb : s.va, cur, nxt, m, s, sh);
        __syncthreads();
        uint32_t* tmp = cur;
        cur = nxt;
        nxt = tmp;
    }
    for (int k = t; k < n; k += NT) {
        const uint32_t i = s.sa[k];
        out[k] = T[i == 0 ? n - 1 : i - 1];
        if (i == 0) *orig = (uint32_t)k;
    }
    __syncthreads();
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
            bwt_block(T, n, out, orig_out + b, s, sh);
        } else if (t == 0) {
            if (n == 1) out[0] = T[0];
            orig_out[b] = 0;
        }
        __syncthreads();
    }
}

}  // namespace bz2mi
