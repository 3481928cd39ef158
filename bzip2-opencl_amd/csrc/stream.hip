// Cross-block kernels: the per-slot seed carry-over and the bit-level stream
// assembly.
//
// seed_kernel restates the reference's never-cleared per-slot MTF frequency
// array (OutputStream.hpp:93 allocated once, kernel.cpp:2613/2641-2643 adding
// into it, kernel.cpp:2859-2893 reading it): block b of the stream seeds its
// Huffman tables from the running sum of the histograms of every earlier block
// that used the same slot (b mod p), itself included.
//
// offsets_kernel / assemble_kernel replace the host bit stitching of
// OutputStream::closeBlocks (OutputStream.hpp:192-239) and
// BitOutputStream.hpp:30-99: blocks are concatenated at bit granularity, each
// as 81 header bits (0x314159265359, block CRC, randomised=0) followed by its
// payload; an optional prefix (stream header and/or carried bits) and the
// end-of-stream trailer (0x177245385090, stream CRC, zero pad) frame them.
#include "common.hpp"
#include "kernels.hpp"

namespace bz2mi {

// One workgroup per (slot, 64 symbols): a slot's chain of blocks b, b+p, ...
// is cut into kSeedWaves contiguous pieces, one per wave (lane = symbol); the
// pieces' sums are scanned in LDS and every wave then writes its running sums.
// (The serial walk of the whole chain per thread took 0.45 ms per GiB: ~1200
// dependent iterations of a global load.)
__global__ __launch_bounds__(kSeedWaves * 64) void seed_kernel(const uint32_t* __restrict__ hist,
                                                              uint32_t* __restrict__ seed,
                                                              uint32_t* __restrict__ state, int nblocks, int p,
                                                              uint64_t first_block) {
    __shared__ uint32_t part[kSeedWaves][64];
    constexpr int nsg = (kMaxAlpha + 63) / 64;
    const int slot = (int)blockIdx.x / nsg, lane = lane_id(), w = wave_id();
    const int sym = ((int)blockIdx.x % nsg) * 64 + lane;
    const bool ok = sym < kMaxAlpha;
    // first batch-local block that maps to `slot`, and the chain's length
    const int r = (int)(first_block % (uint64_t)p);
    int b0 = slot - r;
    if (b0 < 0) b0 += p;
    const int m = b0 < nblocks ? (nblocks - 1 - b0) / p + 1 : 0;
    const int per = (m + kSeedWaves - 1) / kSeedWaves;
    const int i0 = min(m, w * per), i1 = min(m, i0 + per);
    const uint32_t* H = hist + sym;
    uint32_t s = 0;
#pragma unroll 8
    for (int i = i0; i < i1; ++i) s += ok ? H[(size_t)(b0 + i * p) * kMaxAlpha] : 0u;
    part[w][lane] = s;
    uint32_t acc = ok ? state[slot * kMaxAlpha + sym] : 0u;  // read before the last wave rewrites it
    __syncthreads();
    for (int v = 0; v < w; ++v) acc += part[v][lane];
#pragma unroll 8
    for (int i = i0; i < i1; ++i) {
        const size_t at = (size_t)(b0 + i * p) * kMaxAlpha + sym;
        if (ok) {
            acc += hist[at];
            seed[at] = acc;
        }
    }
    // the last wave's sum covers every piece
    if (w == kSeedWaves - 1 && ok) state[slot * kMaxAlpha + sym] = acc;
}

// offs[b] = prefix_bits + sum_{b'<b} (81 + bits[b']); offs[nblocks] = end.
__global__ __launch_bounds__(256) void offsets_kernel(const uint64_t* __restrict__ bits, int nblocks,
                                                      uint64_t prefix_bits, uint64_t* __restrict__ offs) {
    __shared__ uint64_t tmp[4];
    uint64_t carry = prefix_bits;
    for (int base = 0; base < nblocks; base += 256) {
        const int b = base + threadIdx.x;
        const uint64_t v = b < nblocks ? bits[b] + (uint64_t)kHeaderBits : 0;
        uint64_t tot;
        const uint64_t ex = wg_excl_sum64<256>(v, tmp, &tot);
        if (b < nblocks) offs[b] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) offs[nblocks] = carry;
}

namespace {

struct Frame {
    const uint32_t* payload;
    size_t payload_words;
    const uint64_t* offs;
    const uint32_t* crc;
    int nblocks;
    uint64_t prefix;       // MSB-aligned prefix bits
    int prefix_bits;
    int final_;
    uint32_t stream_crc;
};

// Up to `want` (<=32) bits starting at absolute position `pos`, taken from the
// segment `seg` (-1 prefix, 0..nblocks-1 blocks, nblocks trailer) that holds
// `pos`; returns the number of bits taken (stops at the segment's end).
__device__ int seg_bits(const Frame& f, int seg, uint64_t pos, int want, uint32_t* out) {
    uint64_t s0, s1;
    if (seg < 0) {
        s0 = 0;
        s1 = (uint64_t)f.prefix_bits;
    } else if (seg < f.nblocks) {
        s0 = f.offs[seg];
        s1 = f.offs[seg + 1];
    } else {
        s0 = f.offs[f.nblocks];
        s1 = s0 + (f.final_ ? 80u : 0u);
    }
    const uint64_t local = pos - s0;
    int take = (int)((s1 - pos) < (uint64_t)want ? (s1 - pos) : (uint64_t)want);
    if (take <= 0) {
        *out = 0;
        return 0;
    }
    uint64_t win;  // 64-bit MSB-first window starting at `local`
    if (seg < 0) {
        win = f.prefix << local;
    } else if (seg == f.nblocks) {
        const uint32_t c = f.stream_crc;
        const uint32_t w[3] = {0x17724538u, 0x50900000u | (c >> 16), c << 16};
        const int wi = (int)(local >> 5), sh = (int)(local & 31);
        const uint64_t hi = ((uint64_t)w[wi] << 32) | (wi + 1 < 3 ? w[wi + 1] : 0u);
        win = hi << sh;
    } else if (local < (uint64_t)kHeaderBits) {
        const uint32_t c = f.crc[seg];
        const uint32_t w[3] = {0x31415926u, 0x53590000u | (c >> 16), c << 16};
        const int wi = (int)(local >> 5), sh = (int)(local & 31);
        const uint64_t hi = ((uint64_t)w[wi] << 32) | (wi + 1 < 3 ? w[wi + 1] : 0u);
        win = hi << sh;
        const int left = kHeaderBits - (int)local;
        take = take < left ? take : left;
    } else {
        const uint64_t q = local - kHeaderBits;
        const uint32_t* W = f.payload + (size_t)seg * f.payload_words;
        const size_t wi = q >> 5;
        const int sh = (int)(q & 31);
        const uint64_t hi = ((uint64_t)bswap32(W[wi]) << 32) | bswap32(W[wi + 1]);
        win = hi << sh;
    }
    *out = (uint32_t)(win >> 32) >> (32 - take) << (32 - take);  // top `take` bits, MSB-aligned
    return take;
}

}  // namespace

namespace {

// One output word built from the segments its bits lie in, starting at seg
// (header bits, segment edges, prefix and trailer).
__device__ uint32_t general_word(const Frame& f, int seg, uint64_t w, uint64_t end) {
    uint64_t pos = w << 5;
    uint32_t word = 0;
    int got = 0;
    while (got < 32 && pos < end) {
        // advance to the segment holding pos
        for (;;) {
            const uint64_t s1 = seg < 0 ? (uint64_t)f.prefix_bits : (seg < f.nblocks ? f.offs[seg + 1] : end);
            if (pos < s1) break;
            seg++;
        }
        uint32_t bitsv;
        const int take = seg_bits(f, seg, pos, 32 - got, &bitsv);
        if (take == 0) break;
        word |= bitsv >> got;
        got += take;
        pos += take;
    }
    return bswap32(word);
}

// Every output word is built by the segment that holds its first bit, so no
// word is written twice and no atomics are needed.  Workgroup g handles
// segment g-1 (workgroup 0: the prefix).  Words at or past cap_words are not
// written (the caller detects the overflow from the final length).  The words
// whose 32 bits all lie in a block's payload are one funnel shift of two
// payload words (the shift is the same for the whole block); they go four per
// thread as 16-byte stores, the rest (header, block edges) word by word.
__device__ void assemble_body(const Frame& f, uint32_t* __restrict__ out, uint64_t cap_words) {
    const uint64_t end = f.offs[f.nblocks] + (f.final_ ? 80u : 0u);
    const int nblocks = f.nblocks;
    const int seg0 = (int)blockIdx.x - 1;
    if (seg0 > nblocks) return;
    uint64_t lo, hi;
    if (seg0 < 0) {
        lo = 0;
        hi = (uint64_t)f.prefix_bits;
    } else if (seg0 < nblocks) {
        lo = f.offs[seg0];
        hi = f.offs[seg0 + 1];
    } else {
        lo = f.offs[nblocks];
        hi = end;
    }
    // words whose first bit lies in [lo, hi)
    const uint64_t w0 = (lo + 31) >> 5, w1 = min((hi + 31) >> 5, cap_words);
    // payload words [f0, f1) of a block (empty otherwise)
    uint64_t f0 = w1, f1 = w1, pbit = 0;
    if (seg0 >= 0 && seg0 < nblocks) {
        pbit = lo + (uint64_t)kHeaderBits;
        f0 = max((pbit + 31) >> 5, w0);
        f1 = min(hi >> 5, w1);
        if (f0 > f1) f0 = f1 = w1;
    }
    for (uint64_t w = w0 + threadIdx.x; w < f0; w += blockDim.x) out[w] = general_word(f, seg0, w, end);
    for (uint64_t w = f1 + threadIdx.x; w < w1; w += blockDim.x) out[w] = general_word(f, seg0, w, end);
    if (f0 >= f1) return;
    const uint32_t* W = f.payload + (size_t)seg0 * f.payload_words;
    const uint32_t sh = (uint32_t)(((f0 << 5) - pbit) & 31u);
    const uint64_t i0 = ((f0 << 5) - pbit) >> 5;  // payload word under output word f0
    auto word_at = [&](uint64_t w) -> uint32_t {
        const uint64_t i = i0 + (w - f0);
        const uint32_t a = bswap32(W[i]);
        const uint32_t v = sh ? (a << sh) | (bswap32(W[i + 1]) >> (32u - sh)) : a;
        return bswap32(v);
    };
    // 16-byte aligned quads of output words inside [f0, f1)
    const uint64_t mis = ((uint64_t)(uintptr_t)out >> 2) & 3u;  // out is 4-byte aligned
    uint64_t a0 = ((f0 + mis + 3) & ~3ull) - mis;
    if (a0 > f1) a0 = f1;
    uint64_t a1 = ((f1 + mis) & ~3ull) - mis;
    if (a1 < a0) a1 = a0;
    for (uint64_t w = f0 + threadIdx.x; w < a0; w += blockDim.x) out[w] = word_at(w);
    for (uint64_t w = a1 + threadIdx.x; w < f1; w += blockDim.x) out[w] = word_at(w);
    for (uint64_t w = a0 + 4 * (uint64_t)threadIdx.x; w < a1; w += 4 * (uint64_t)blockDim.x) {
        const uint64_t i = i0 + (w - f0);
        uint32_t x[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) x[k] = bswap32(W[i + k]);
        uint32_t y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = bswap32(sh ? (x[k] << sh) | (x[k + 1] >> (32u - sh)) : x[k]);
        *reinterpret_cast<uint4*>(out + w) = make_uint4(y[0], y[1], y[2], y[3]);
    }
}

}  // namespace

// Host-driven form: prefix bits and stream CRC from the host.
__global__ __launch_bounds__(256) void assemble_kernel(const uint32_t* __restrict__ payload, size_t payload_words,
                                                       const uint64_t* __restrict__ offs,
                                                       const uint32_t* __restrict__ crc, int nblocks,
                                                       uint64_t prefix, int prefix_bits, int final_,
                                                       uint32_t stream_crc, uint32_t* __restrict__ out) {
    const Frame f{payload, payload_words, offs, crc, nblocks, prefix, prefix_bits, final_, stream_crc};
    assemble_body(f, out, ~0ull);
}

// ---- device-resident stream state (pipelined compress_device): batches are
// assembled one after another on one stream without host round trips.

// offs[b] = carry_bits + sum_{b'<b} (81 + bits[b']); folds the batch's block
// CRCs into the stream CRC: crc' = rotl(crc, nb) ^ XOR_b rotl(crc_b, nb-1-b)
// (the sequential crc = rotl(crc, 1) ^ crc_b of OutputStream.hpp:233).
__global__ __launch_bounds__(256) void offsets_dev_kernel(const uint64_t* __restrict__ bits,
                                                          const uint32_t* __restrict__ crcs, int nblocks,
                                                          StreamDev* __restrict__ st, uint64_t* __restrict__ offs) {
    __shared__ uint64_t tmp[4];
    __shared__ uint32_t xr[4];
    uint64_t carry = (uint64_t)st->carry_bits;
    uint32_t x = 0;
    for (int base = 0; base < nblocks; base += 256) {
        const int b = base + threadIdx.x;
        const uint64_t v = b < nblocks ? bits[b] + (uint64_t)kHeaderBits : 0;
        uint64_t tot;
        const uint64_t ex = wg_excl_sum64<256>(v, tmp, &tot);
        if (b < nblocks) {
            offs[b] = carry + ex;
            const uint32_t r = (uint32_t)(nblocks - 1 - b) & 31u;
            const uint32_t cb = crcs[b];
            x ^= r ? (cb << r) | (cb >> (32 - r)) : cb;
        }
        carry += tot;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x ^= (uint32_t)__shfl_xor((int)x, d);
    if (lane_id() == 0) xr[wave_id()] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        offs[nblocks] = carry;
        const uint32_t r = (uint32_t)nblocks & 31u, c0 = st->crc;
        st->crc = (r ? (c0 << r) | (c0 >> (32 - r)) : c0) ^ xr[0] ^ xr[1] ^ xr[2] ^ xr[3];
    }
}

__global__ __launch_bounds__(256) void assemble_dev_kernel(const uint32_t* __restrict__ payload, size_t payload_words,
                                                           const uint64_t* __restrict__ offs,
                                                           const uint32_t* __restrict__ crc, int nblocks, int final_,
                                                           const StreamDev* __restrict__ st,
                                                           uint32_t* __restrict__ out, uint64_t cap_words) {
    const uint64_t base = st->word_base;
    const Frame f{payload, payload_words, offs, crc, nblocks, (uint64_t)st->carry << 32, (int)st->carry_bits,
                  final_, st->crc};
    assemble_body(f, out + base, cap_words > base ? cap_words - base : 0);
}

// Volumes of a batch (RLE1 bytes, MTF symbols, payload bits) added into acc[0..2].
__global__ __launch_bounds__(256) void volume_kernel(const uint32_t* __restrict__ lens,
                                                     const uint32_t* __restrict__ mtflen,
                                                     const uint64_t* __restrict__ pbits, int nblocks,
                                                     unsigned long long* __restrict__ acc) {
    unsigned long long a = 0, m = 0, p = 0;
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < nblocks; b += gridDim.x * blockDim.x) {
        a += lens[b];
        m += mtflen[b];
        p += pbits[b];
    }
    if (a) atomicAdd(&acc[0], a);
    if (m) atomicAdd(&acc[1], m);
    if (p) atomicAdd(&acc[2], p);
}

// Move the state past the batch: whole words are final, the partial last
// word is carried (read back from the output); the final batch records the
// stream length instead.
__global__ void advance_kernel(const uint64_t* __restrict__ offs, int nblocks, int final_, StreamDev* __restrict__ st,
                               const uint32_t* __restrict__ out, uint64_t cap_words) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t end = offs[nblocks] + (final_ ? 80u : 0u);
    const uint64_t base = st->word_base;
    if (final_) {
        st->final_bits = base * 32 + end;
        return;
    }
    const uint64_t nb = base + (end >> 5);
    const uint32_t cb = (uint32_t)(end & 31);
    uint32_t carry = 0;
    if (cb && nb < cap_words) carry = bswap32(out[nb]) & (0xffffffffu << (32 - cb));
    st->word_base = nb;
    st->carry = carry;
    st->carry_bits = cb;
}

}  // namespace bz2mi
