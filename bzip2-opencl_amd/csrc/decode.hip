// bzip2 decompression on the device.
//
// Replaces the reference's host decoder: InputStream (include/InputStream.hpp:
// 36-159: stream header, block / end-of-stream markers, stream CRC),
// BlockDecompressor (BlockDecompressor.hpp:37-282: block header, symbol map,
// selectors, table code lengths, Huffman + MTF + RLE2 decode, inverse BWT,
// RLE1 expansion with the block CRC) and HuffmanStageDecoder
// (HuffmanStageDecoder.hpp:30-136: canonical code tables, 50-symbol groups).
// The reference decodes one byte at a time on one thread; here every block of
// the stream is decoded at once:
//
//   K1 dec_scan_kernel     every bit position is tested for the 48-bit block
//                          and end-of-stream magics (candidates; the 32 bits
//                          after a magic are the stored CRC)
//   K2 dec_huff_kernel     one wave per candidate block: header, tables, then
//                          the Huffman symbols (scalar bit reader, LDS lookup
//                          tables) with the move-to-front list held across
//                          the wave (4 entries per lane) and RLE2 runs, giving
//                          the BWT bytes, their histogram and the end bit
//   (host)                 the chain stream header -> blocks -> end marker is
//                          walked over the candidates' end bits, which drops
//                          magics that occur inside compressed data
//   K3 dec_ibwt_kernel     one workgroup per block: stable counting sort into
//                          the merged pointer vector (BlockDecompressor.hpp:
//                          238-262), then 1024 walkers split the LF cycle into
//                          segments, a chain pass orders them, and the walkers
//                          write the RLE1 bytes
//   K4 dec_rle1_kernel     one workgroup per block, 256 chunks: the RLE1 state
//                          machine (BlockDecompressor.hpp:55-88) is run from
//                          all 5 entry states per chunk, chained, then run
//                          again writing the output; the block CRC is
//                          combined from the chunk CRCs with x^(8L) mod P.
#include "common.hpp"
#include "decode.hpp"

namespace bz2mi {

// x^(8 * 2^k) mod P (CRC32 polynomial 0x04c11db7, MSB-first register)
__constant__ uint32_t c_xpow8[64];

namespace {

__device__ __forceinline__ uint32_t gf_mulmod(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll 4
    for (int i = 31; i >= 0; --i) {
        r = (r << 1) ^ ((r >> 31) ? 0x04c11db7u : 0u);
        if ((b >> i) & 1u) r ^= a;
    }
    return r;
}

// v * x^(8 L) mod P: the CRC register after L more zero bytes
__device__ __forceinline__ uint32_t crc_shift(uint32_t v, uint64_t L) {
    for (int k = 0; L; ++k, L >>= 1)
        if (L & 1) v = gf_mulmod(v, c_xpow8[k]);
    return v;
}

// ---- big-endian bit reader over the compressed stream, all-uniform (one
// reader per wave; the state lives in SGPRs)
struct BitReader {
    const uint32_t* w;  // stream as 32-bit words (byte-swapped on use)
    uint64_t nbits;     // stream length in bits
    uint64_t pos;       // next bit (absolute)
    uint64_t buf;       // MSB-aligned pending bits
    int nb;             // valid bits in buf
    uint64_t res;       // next 64 bits (reserve), MSB first
    int rb;             // valid bits in res (0, 32 or 64)
    uint64_t pf;        // the 64 bits after res, loaded ahead (prefetch)
    uint64_t wnext;     // word index of the next prefetch
    bool over;          // read past the end

    __device__ __forceinline__ uint32_t word(uint64_t i) const {
        // big-endian word i; bytes past the end read as zero (no over-read)
        const uint64_t nbytes = nbits >> 3;
        if ((i + 1) * 4 <= nbytes) return __builtin_bswap32(w[i]);
        uint32_t x = 0;
        const uint8_t* b = reinterpret_cast<const uint8_t*>(w);
        for (int q = 0; q < 4; ++q) x = (x << 8) | ((i * 4 + q < nbytes) ? b[i * 4 + q] : 0u);
        return x;
    }
    __device__ __forceinline__ uint64_t load64(uint64_t i) const {
        if ((i + 2) * 4 <= (nbits >> 3))
            return ((uint64_t)__builtin_bswap32(w[i]) << 32) | __builtin_bswap32(w[i + 1]);
        return ((uint64_t)word(i) << 32) | word(i + 1);
    }
    __device__ void init(const uint8_t* base, uint64_t nbytes, uint64_t bitpos) {
        // `base` is 4-byte aligned
        w = reinterpret_cast<const uint32_t*>(base);
        nbits = nbytes * 8;
        pos = bitpos;
        const uint64_t w0 = bitpos >> 5;
        const int off = (int)(bitpos & 31);
        buf = load64(w0) << off;
        nb = 64 - off;
        res = load64(w0 + 2);
        rb = 64;
        pf = load64(w0 + 4);
        wnext = w0 + 6;
        over = false;
    }
    // keep > 32 bits in buf: 32 bits move from the reserve; an empty reserve
    // takes the prefetched 64 bits and the next prefetch is issued (its
    // latency is covered by the ~64 bits decoded meanwhile)
    __device__ __forceinline__ void refill() {
        if (nb <= 32) {
            buf |= (res >> 32) << (32 - nb);
            res <<= 32;
            rb -= 32;
            nb += 32;
            if (rb == 0) {
                res = pf;
                rb = 64;
                pf = load64(wnext);
                wnext += 2;
            }
        }
    }
    __device__ __forceinline__ uint32_t peek(int k) const { return (uint32_t)(buf >> (64 - k)); }
    __device__ __forceinline__ void skip(int k) {  // k <= 32
        buf <<= k;
        nb -= k;
        pos += k;
        refill();
    }
    // skip without keeping `pos` (the symbol loop): position() recovers it
    // from the reader state -- bits loaded up to word wnext minus the unread
    // ones (pf, res, buf)
    __device__ __forceinline__ void skip_fast(int k) {  // k <= 32
        buf <<= k;
        nb -= k;
        refill();
    }
    __device__ __forceinline__ uint64_t position() const { return wnext * 32 - 64 - (uint64_t)rb - (uint64_t)nb; }
    __device__ __forceinline__ void check() {
        if (pos > nbits) over = true;
    }
    __device__ __forceinline__ uint32_t bits(int k) {  // 1..32
        const uint32_t v = peek(k);
        skip(k);
        check();
        return v;
    }
    __device__ __forceinline__ uint32_t bit() { return bits(1); }
};

// BZ2MI_HUF_WORDPARSE (default): selectors and delta-coded lengths parsed a
// word at a time (leading-ones count, pair flags) instead of bit by bit
#ifndef BZ2MI_HUF_WORDPARSE
#define BZ2MI_HUF_WORDPARSE 1
#endif
constexpr int kLutBits = 9;
constexpr uint16_t kLong = 0xffff;
constexpr int kMaxDecLen = 23;  // HUFFMAN_DECODE_MAXIMUM_CODE_LENGTH (Config.hpp:38)
constexpr int kDecMaxSel = 18002; // 900 KB blocks (bzip2's BZ_MAX_SELECTORS)

struct HuffLds {
    uint16_t lut[kMaxTables][1 << kLutBits];  // sym | len << 12, or kLong
    int32_t limit[kMaxTables][kMaxDecLen + 2];
    int32_t base[kMaxTables][kMaxDecLen + 2];  // rank of the first code of a length minus that code
    uint16_t perm[kMaxTables][kMaxAlpha];       // symbols by (length, symbol)
    uint8_t len[kMaxTables][kMaxAlpha];
    uint8_t symmap[256];
};

__device__ __forceinline__ void fail(DecBlockInfo* info, uint32_t code) {
    if (threadIdx.x == 0) info->status = code;
}

}  // namespace

// ---- K1: candidates.  Thread per 8-byte word of the stream: the 64 bit
// positions starting in it, the 48-bit window read from 16 bytes.
// BZ2MI_SCAN_HASH (default): a magic that starts in byte B of the thread's
// word covers bytes B+1..B+4 completely, and those 32 bits are one of 16
// values (2 magics x 8 bit offsets); a perfect hash of them ((w * K) >> 27,
// 32 slots) tests each B with one LDS lookup, and only a hit runs the exact
// test of its 8 bit positions (instead of 64 exact tests per thread).
#ifndef BZ2MI_SCAN_HASH
#define BZ2MI_SCAN_HASH 1
#endif
constexpr uint32_t kScanK = 0xcd447e35u;
__constant__ uint32_t c_scan_tab[32] = {
    // slot -> bytes 1..4 of a magic at bit offset s (blk s = 0..7, eos s = 0..7);
    // empty slots hold a value that hashes elsewhere (never matches)
    0x41592653u, 0x41592653u, 0x282b24cau, 0x5dc914e1u, 0xa0ac9329u, 0x50564994u, 0xbb9229c2u, 0x77245385u,
    0x41592653u, 0x41592653u, 0x41592653u, 0x8a0ac932u, 0x41592653u, 0x41592653u, 0xee48a70au, 0x41592653u,
    0x41592653u, 0x14159265u, 0x41592653u, 0x41592653u, 0x2ee48a70u, 0xc5056499u, 0x41592653u, 0x72453850u,
    0x41592653u, 0x41592653u, 0x41592653u, 0xb9229c28u, 0x41592653u, 0xdc914e14u, 0x6282b24cu, 0x41592653u,
};

__global__ __launch_bounds__(256) void dec_scan_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                       DecCand* __restrict__ cand, uint32_t* __restrict__ ncand,
                                                       uint32_t cap) {
#if BZ2MI_SCAN_HASH
    __shared__ uint32_t htab[32];
    if (threadIdx.x < 32) htab[threadIdx.x] = c_scan_tab[threadIdx.x];
    __syncthreads();
#endif
    const uint64_t wi = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t b0 = wi * 8;
    if (b0 >= n) return;
    uint64_t hi = 0, lo = 0, t2 = 0;
    if (((reinterpret_cast<uintptr_t>(in) & 3u) == 0) && b0 + 20 <= n) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(in + b0);
        const uint32_t a0 = __builtin_bswap32(w[0]), a1 = __builtin_bswap32(w[1]), a2 = __builtin_bswap32(w[2]),
                       a3 = __builtin_bswap32(w[3]), a4 = __builtin_bswap32(w[4]);
        hi = ((uint64_t)a0 << 32) | a1;
        lo = ((uint64_t)a2 << 32) | a3;
        t2 = (uint64_t)a4 << 32;
    } else {
        uint8_t by[20];
#pragma unroll
        for (int k = 0; k < 20; ++k) by[k] = (b0 + k < n) ? in[b0 + k] : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) hi = (hi << 8) | by[k];
#pragma unroll
        for (int k = 8; k < 16; ++k) lo = (lo << 8) | by[k];
#pragma unroll
        for (int k = 16; k < 20; ++k) t2 = (t2 << 8) | by[k];
        t2 <<= 32;
    }
    // bits [q, q+64) of the 192-bit window hi:lo:t2 (q < 128)
    auto get64 = [&](int q) -> uint64_t {
        if (q == 0) return hi;
        if (q < 64) return (hi << q) | (lo >> (64 - q));
        if (q == 64) return lo;
        return (lo << (q - 64)) | (t2 >> (128 - q));
    };
    constexpr uint64_t kBlk = 0x314159265359ull, kEos = 0x177245385090ull;
    auto exact = [&](int o) {
        const uint64_t p = b0 * 8 + (uint64_t)o;
        if (p + 48 > n * 8) return;
        const uint64_t win = get64(o) >> 16;
        if (win == kBlk || win == kEos) {
            const uint32_t nx = (uint32_t)(get64(o + 48) >> 32);  // the 32 bits after the magic
            const uint32_t slot = atomicAdd(ncand, 1u);
            if (slot < cap) cand[slot] = DecCand{p, win == kEos ? 1u : 0u, nx};
        }
    };
#if BZ2MI_SCAN_HASH
    uint32_t hits = 0;
#pragma unroll
    for (int B = 0; B < 8; ++B) {
        const uint32_t v = (uint32_t)(get64(8 * (B + 1)) >> 32);  // bytes B+1..B+4
        hits |= (htab[(v * kScanK) >> 27] == v ? 1u : 0u) << B;
    }
    while (hits) {
        const int B = __builtin_ctz(hits);
        hits &= hits - 1;
        for (int s2 = 0; s2 < 8; ++s2) exact(8 * B + s2);
    }
#else
    for (int o = 0; o < 64; ++o) exact(o);
#endif
}

// ---- K2: one wave per candidate block: header, symbol map, selectors, code
// lengths and the decoding tables (HuffmanStageDecoder::
// createHuffmanDecodingTables :86-135), handed to dec_sym_kernel in `tabs`.
__global__ __launch_bounds__(64) void dec_huff_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                      const DecCand* __restrict__ cand, const uint32_t* __restrict__ ids,
                                                      uint32_t nids, uint32_t max_sel, uint8_t* __restrict__ tabs,
                                                      uint8_t* __restrict__ symmap_out,
                                                      DecBlockInfo* __restrict__ infos) {
    __shared__ HuffLds L;
    extern __shared__ uint32_t sel_lds[];  // selectors, 4 bits each ((max_sel + 7) / 8 words)
    const uint32_t k = blockIdx.x;
    if (k >= nids) return;
    const int lane = lane_id();
    const uint32_t c = uniform(ids[k]);
    DecBlockInfo* info = infos + k;
    BitReader br;
    br.init(in, n, cand[c].bitpos + 48);
    if (lane == 0) {
        info->status = 0;
        info->end_bit = 0;
        info->len = 0;
        info->nsym = 0;
        info->data_bit = 0;
        info->nsel = 0;
    }
    const uint32_t crc = br.bits(16) << 16;
    const uint32_t crc2 = crc | br.bits(16);
    const uint32_t rnd = br.bit();
    const uint32_t orig = br.bits(24);
    if (lane == 0) {
        info->crc = crc2;
        info->orig = orig;
    }
    // symbol map (BlockDecompressor.hpp:134-152)
    const uint32_t used = br.bits(16);
    uint32_t nsym = 0;
    for (int i = 0; i < 16; ++i) {
        if (used & (0x8000u >> i)) {
            const uint32_t m = br.bits(16);
            for (int j = 0; j < 16; ++j)
                if (m & (0x8000u >> j)) {
                    if (lane == 0) L.symmap[nsym] = (uint8_t)(i * 16 + j);
                    nsym++;
                }
        }
    }
    const uint32_t alpha = nsym + 2;  // symbols 0 (RUNA) .. nsym + 1 (end of block)
    const uint32_t ntab = br.bits(3), nsel = br.bits(15);
    if (ntab < 2 || ntab > (uint32_t)kMaxTables || nsel < 1 || nsel > max_sel || nsel > (uint32_t)kDecMaxSel) {
        fail(info, kDecTables);
        return;
    }
    // selectors, MTF-coded in unary (:156-161)
    {
        uint32_t mtf = 0x543210u;  // 4-bit entries, front = lowest nibble
        for (uint32_t i = 0; i < nsel; ++i) {
            uint32_t u = 0;
#if BZ2MI_HUF_WORDPARSE
            // the unary code's ones counted at once (ntab <= 6 < 8 peeked bits)
            u = (uint32_t)__builtin_clz(~(br.peek(8) << 24) | 0x00800000u);
            if (u < ntab) {
                br.skip((int)u + 1);
                br.check();
            }
#else
            while (br.bit()) {
                if (++u >= ntab) break;
            }
#endif
            if (u >= ntab || br.over) {
                fail(info, kDecTables);
                return;
            }
            const uint32_t v = (mtf >> (4 * u)) & 15u;
            const uint32_t below = mtf & ((1u << (4 * u)) - 1u);
            const uint32_t above = u == 5 ? 0u : (mtf >> (4 * (u + 1))) << (4 * (u + 1));
            mtf = above | (below << 4) | v;
            if (lane == 0) {
                uint32_t& wv = sel_lds[i >> 3];
                wv = (i & 7) ? (wv | (v << (4 * (i & 7)))) : v;
            }
        }
    }
    // code lengths, delta-coded (:163-174)
    for (uint32_t t = 0; t < ntab; ++t) {
        int cur = (int)br.bits(5);
        for (uint32_t j = 0; j < alpha; ++j) {
#if BZ2MI_HUF_WORDPARSE
            // "1x" pairs then a 0, read from one 32-bit peek: the first 0
            // among the pair flags (even offsets) ends the code; each x = 1
            // is -1, each x = 0 is +1 (more than 15 pairs: bit by bit)
            const uint32_t w = br.peek(32);
            const uint32_t stop = ~w & 0xAAAAAAAAu;
            if (stop) {
                const uint32_t kp = (uint32_t)__builtin_clz(stop) >> 1;  // pairs before the 0
                const uint32_t top = kp ? ~0u << (32 - 2 * kp) : 0u;
                const int xs = __popc(w & 0x55555555u & top);
                cur += (int)kp - 2 * xs;
                br.skip((int)(2 * kp + 1));
                br.check();
            } else
#endif
            {
                int guard = 0;
                while (br.bit()) {
                    cur += br.bit() ? -1 : 1;
                    if (++guard > 40) break;
                }
            }
            if (cur < 1 || cur > kMaxDecLen || br.over) {
                fail(info, kDecTables);
                return;
            }
            if (lane == 0) L.len[t][j] = (uint8_t)cur;
        }
    }
    __syncthreads();
    // decoding tables (HuffmanStageDecoder.hpp:86-135): lane t < ntab builds
    // table t's limits, bases and symbol permutation; then all lanes fill the
    // 9-bit lookup tables
    if ((uint32_t)lane < ntab) {
        const int t = lane;
        uint32_t cnt[kMaxDecLen + 1];
        for (int l = 0; l <= kMaxDecLen; ++l) cnt[l] = 0;
        for (uint32_t j = 0; j < alpha; ++j) cnt[L.len[t][j]]++;
        int32_t code = 0, rank = 0;
        for (int l = 1; l <= kMaxDecLen; ++l) {
            if (cnt[l]) {
                L.base[t][l] = rank - code;
                L.limit[t][l] = code + (int32_t)cnt[l] - 1;
            } else {
                L.base[t][l] = 0;
                L.limit[t][l] = -1;
            }
            rank += (int32_t)cnt[l];
            code = (code + (int32_t)cnt[l]) << 1;
        }
        // permutation: ranks in (length, symbol) order
        uint32_t next[kMaxDecLen + 1];
        uint32_t r0 = 0;
        for (int l = 1; l <= kMaxDecLen; ++l) {
            next[l] = r0;
            r0 += cnt[l];
        }
        for (uint32_t j = 0; j < alpha; ++j) L.perm[t][next[L.len[t][j]]++] = (uint16_t)j;
    }
    for (int i = lane; i < kMaxTables * (1 << kLutBits); i += 64) (&L.lut[0][0])[i] = kLong;
    __syncthreads();
    // lookup tables: the symbol of rank R (in (length, symbol) order) has the
    // code R - base[length]; codes of <= kLutBits bits fill their entries
    for (uint32_t t = 0; t < ntab; ++t) {
        for (uint32_t R = lane; R < alpha; R += 64) {
            const uint32_t j = L.perm[t][R];
            const uint32_t l = L.len[t][j];
            if (l > (uint32_t)kLutBits) continue;
            const uint32_t cj = (uint32_t)((int32_t)R - L.base[t][l]);
            const uint32_t lo = cj << (kLutBits - l), hi = (cj + 1) << (kLutBits - l);
            for (uint32_t e = lo; e < hi && e < (1u << kLutBits); ++e) L.lut[t][e] = (uint16_t)(j | (l << 12));
        }
    }
    __syncthreads();
    if (rnd) {  // BlockDecompressor.hpp:270-273
        fail(info, kDecRandomised);
        return;
    }
    // ---- hand the tables to dec_sym_kernel: lookup tables, limits, bases,
    // permutations and the selectors, and where the data starts
    uint8_t* tb = tabs + (size_t)k * kTabBytes;
    {
        uint32_t* d32 = reinterpret_cast<uint32_t*>(tb);
        const uint32_t* l32 = reinterpret_cast<const uint32_t*>(&L.lut[0][0]);
        for (int i = lane; i < kMaxTables * (1 << kLutBits) / 2; i += 64) d32[i] = l32[i];
        int32_t* lim = reinterpret_cast<int32_t*>(tb + kTabLimit);
        int32_t* bas = reinterpret_cast<int32_t*>(tb + kTabBase);
        for (int i = lane; i < kMaxTables * (kMaxDecLen + 2); i += 64) {
            lim[i] = (&L.limit[0][0])[i];
            bas[i] = (&L.base[0][0])[i];
        }
        uint16_t* per = reinterpret_cast<uint16_t*>(tb + kTabPerm);
        for (int i = lane; i < kMaxTables * kMaxAlpha; i += 64) per[i] = (&L.perm[0][0])[i];
        uint8_t* sg = tb + kTabSel;
        for (uint32_t i = lane; i < nsel; i += 64) sg[i] = (uint8_t)((sel_lds[i >> 3] >> (4 * (i & 7))) & 15u);
    }
    if (lane == 0) {
        info->status = 0;
        info->data_bit = br.pos;
        info->nsel = nsel;
        info->alpha = nsym;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) symmap_out[(size_t)k * 256 + lane * 4 + j] = L.symmap[lane * 4 + j];
}

// ---- K2s: the Huffman symbols (HuffmanStageDecoder::nextSymbol :48-71), the
// one serial chain of a block: lanes 0..kSymBlocks-1 of a wave each decode
// their own block, with its lookup tables in LDS (one gather per symbol) and
// a private bit reader; the other lanes only stage the tables.  Vector code:
// the chains of 8 blocks per wave share the instruction stream instead of
// queueing on the CU's one scalar unit.
#ifndef BZ2MI_SYM_BLOCKS
#define BZ2MI_SYM_BLOCKS 2
#endif
constexpr int kSymBlocks = BZ2MI_SYM_BLOCKS;  // blocks per wave (LDS: 6 KB of tables each); measured
                                              // 1/2/4/8 blocks: 91 / 73 / 94 / 90 ms per GiB

// codes longer than the lookup table (the reference's limit / base walk)
__device__ __forceinline__ uint32_t long_code(const BitReader& br, const int32_t* lim, const int32_t* bas,
                                           const uint16_t* per, uint32_t* len_out) {
    for (uint32_t len = kLutBits + 1; len <= (uint32_t)kMaxDecLen; ++len) {
        const int32_t cv = (int32_t)br.peek((int)len);
        if (cv <= lim[len]) {
            *len_out = len;
            return per[(uint32_t)(cv + bas[len])];
        }
    }
    *len_out = 0;
    return 0xffffffffu;
}

// work item j decodes candidate sel[j] (its tables and info) into symbol row j
__global__ __launch_bounds__(64) void dec_sym_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                     const uint8_t* __restrict__ tabs, const uint32_t* __restrict__ sel,
                                                     uint32_t nids, uint32_t smax,
                                                     uint16_t* __restrict__ syms, size_t sym_stride,
                                                     DecBlockInfo* __restrict__ infos) {
    // the lookup tables (the table layout's first kTabLimit bytes) of the
    // wave's blocks; the long-code limit / base arrays stay in global memory
    // (staged too they cost occupancy: measured 80 -> 104 ms per GiB)
    static_assert(kTabLimit == kMaxTables * (1 << kLutBits) * 2, "table layout");
    __shared__ uint32_t tabl[kSymBlocks][kTabLimit / 4];
    const int lane = lane_id();
    const uint32_t k0 = blockIdx.x * kSymBlocks;
    // stage the tables of this wave's blocks
    for (int b = 0; b < kSymBlocks; ++b) {
        if (k0 + b >= nids) break;
        const uint32_t id = uniform(sel[k0 + b]);
        const uint32_t st = uniform(infos[id].status);
        if (st) continue;
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(tabs + (size_t)id * kTabBytes);
        for (int i = lane; i < (int)(kTabLimit / 4); i += 64) tabl[b][i] = s32[i];
    }
    __syncthreads();
    const uint32_t k = k0 + (uint32_t)lane;
    if (lane >= kSymBlocks || k >= nids) return;
    const uint32_t id = sel[k];
    DecBlockInfo* info = infos + id;
    if (info->status) return;
    const uint8_t* tb = tabs + (size_t)id * kTabBytes;
    const uint8_t* tl = reinterpret_cast<const uint8_t*>(&tabl[lane][0]);
    const int32_t* lim = reinterpret_cast<const int32_t*>(tb + kTabLimit);
    const int32_t* bas = reinterpret_cast<const int32_t*>(tb + kTabBase);
    const uint16_t* per = reinterpret_cast<const uint16_t*>(tb + kTabPerm);
    const uint8_t* sg = tb + kTabSel;
    const uint32_t nsel = info->nsel, eob = info->alpha + 1;
    const uint16_t* L = reinterpret_cast<const uint16_t*>(tl);
    BitReader br;
    br.init(in, n, info->data_bit);
    uint16_t* so = syms + (size_t)k * sym_stride;
    const uint32_t ns_max = smax + 2;
    uint32_t g = 0, gleft = kGroupRun, ns = 0, status = 0;
    uint32_t tbase = (uint32_t)sg[0] << kLutBits;
    uint32_t nsel1 = nsel > 1 ? sg[1] : 0u;  // next group's table, loaded ahead
    // symbols leave in 16-byte stores of 8: a 128-bit shift register (the
    // newest symbol enters at the top), stored when 8 have entered -- one
    // store per 8 symbols instead of a 2-byte store per symbol
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    auto push = [&](uint32_t v) {
        a0 = __builtin_amdgcn_alignbit(a1, a0, 16);
        a1 = __builtin_amdgcn_alignbit(a2, a1, 16);
        a2 = __builtin_amdgcn_alignbit(a3, a2, 16);
        a3 = (a3 >> 16) | (v << 16);
    };
    for (;;) {
        const uint32_t e = L[tbase + br.peek(kLutBits)];
        uint32_t sym, len;
        if (e != kLong) {
            sym = e & 0xfffu;
            len = e >> 12;
        } else {
            const uint32_t t = tbase >> kLutBits;
            sym = long_code(br, lim + t * (kMaxDecLen + 2), bas + t * (kMaxDecLen + 2), per + t * kMaxAlpha, &len);
            if (sym == 0xffffffffu) {
                status = kDecData;
                break;
            }
        }
        br.skip_fast((int)len);
        // (reading past the end is checked once, after the loop: the reader
        // returns zero bits there, and a block that ran past the end fails
        // with kDecData whatever it decoded meanwhile)
        push(sym);
        if ((++ns & 7u) == 0) *reinterpret_cast<uint4*>(so + ns - 8) = make_uint4(a0, a1, a2, a3);
        if (sym == eob || ns >= ns_max) {
            if (sym != eob) status = kDecSize;
            break;
        }
        if (--gleft == 0) {  // next group of 50 (HuffmanStageDecoder.hpp:50-57)
            if (++g >= nsel) {
                status = kDecData;
                break;
            }
            tbase = nsel1 << kLutBits;
            nsel1 = g + 1 < nsel ? sg[g + 1] : 0u;
            gleft = kGroupRun;
        }
    }
    br.pos = br.position();
    if (br.pos > br.nbits) status = kDecData;
    if (ns & 7u) {  // the last partial 8 (zeros after it: the stride is a multiple of 64 symbols)
        for (uint32_t q = ns & 7u; q < 8; ++q) push(0u);
        *reinterpret_cast<uint4*>(so + (ns & ~7u)) = make_uint4(a0, a1, a2, a3);
    }
    info->status = status;
    info->nsym = ns;
    info->end_bit = br.pos;
}

// ---- K2s, windowed (BZ2MI_SYM_WINDOW, the default): one block per wave.
// The wave's 64 lanes look up the codes that would start at bit offsets
// 0..63 of the reader's 128-bit window at once (one LDS gather), and the
// block's serial chain then hops through those lookups -- offset o, its
// entry (a lane read), o += the code length -- on the scalar unit, a few
// instructions per symbol instead of a dependent LDS lookup and shift each.
// A window ends past offset 63, at a group boundary (the next group's table)
// or at a code longer than the lookup (the reference's limit / base walk on
// the window's bits).  Symbols collect one per lane and leave 64 at a time.
__global__ __launch_bounds__(64) void dec_symw_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                      const uint8_t* __restrict__ tabs, const uint32_t* __restrict__ sel,
                                                      uint32_t nids, uint32_t smax, uint16_t* __restrict__ syms,
                                                      size_t sym_stride, DecBlockInfo* __restrict__ infos) {
    static_assert(kTabLimit == kMaxTables * (1 << kLutBits) * 2, "table layout");
    static_assert(kTabSel % 4 == 0 && kTabBytes - kTabSel >= (kDecMaxSel / 4 + 2) * 4, "selector words");
    __shared__ uint32_t lut32[kTabLimit / 4];
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t k = blockIdx.x;
    if (k >= nids) return;
    const uint32_t id = uniform(sel[k]);
    DecBlockInfo* info = infos + id;
    if (uniform(info->status)) return;
    const uint8_t* tb = tabs + (size_t)id * kTabBytes;
    {
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(tb);
        for (uint32_t i = lane; i < (uint32_t)(kTabLimit / 4); i += 64) lut32[i] = s32[i];
    }
    __syncthreads();
    const uint16_t* lut = reinterpret_cast<const uint16_t*>(lut32);
    const int32_t* lim = reinterpret_cast<const int32_t*>(tb + kTabLimit);
    const int32_t* bas = reinterpret_cast<const int32_t*>(tb + kTabBase);
    const uint16_t* per = reinterpret_cast<const uint16_t*>(tb + kTabPerm);
    const uint8_t* sg = tb + kTabSel;
    const uint32_t nsel = uniform(info->nsel), eob = uniform(info->alpha) + 1;
    // the reader: the stream's words wb..wb+127 one per lane in two vector
    // registers (ra: the current 64, byte-swapped; rb: the next 64 as loaded,
    // a ring ahead -- vector loads, untouched until the window reaches them,
    // so no wait on them stalls the chain), the position `bo` bits into ra.
    // Indices are clamped to the last whole word and the words from there
    // on fixed up when a window reaches them.
    const uint32_t* w32 = reinterpret_cast<const uint32_t*>(in);  // (4-byte aligned)
    const uint64_t nfull = n >> 2;
    uint32_t tailw = 0;  // the last partial word, zero-padded
    for (uint32_t q = 0; q < (uint32_t)(n & 3u); ++q) tailw |= (uint32_t)in[nfull * 4 + q] << (24 - 8 * q);
    // (a block candidate needs more than 4 bytes: nfull >= 1)
    auto raw_word = [&](uint64_t w0) -> uint32_t { return w32[min(w0 + lane, nfull - 1)]; };
    const uint64_t p0 = uniform64(info->data_bit);
    uint64_t wb = p0 >> 5;
    uint32_t bo = (uint32_t)(p0 & 31u);
    uint32_t ra = raw_word(wb), rb = raw_word(wb + 64);
    uint16_t* so = syms + (size_t)k * sym_stride;
    const uint32_t ns_max = smax + 2;
    uint32_t g = 0, gleft = kGroupRun, ns = 0, status = 0;
    // selectors four to a word, the next word loaded ahead (the words past
    // nsel are inside the table area: kTabBytes holds the maximum + padding)
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sg);
    uint32_t swc = sw[0], swn = sw[1];
    uint32_t tsel = swc & 255u;
    bool done = false;
    // one ring of 64 words: windows while the position is in `cur`; then the
    // ring after `nxt` is loaded into `cur`'s register (the two swap roles,
    // so a load is only waited for a whole ring later)
    auto run_ring = [&](uint32_t& cur, const uint32_t& nxt) {
      const uint32_t cs = __builtin_bswap32(cur);
      while (!done && bo < 64 * 32) {
        // words wi..wi+4 (the window: 128 bits from bit `off` of word wi)
        const uint32_t wi = bo >> 5, off = bo & 31u;
        uint32_t a[5];
        if (wi + 4 < 64) {
#pragma unroll
            for (int q = 0; q < 5; ++q) a[q] = (uint32_t)__builtin_amdgcn_readlane((int)cs, (int)(wi + q));
        } else {
            const uint32_t ns2 = __builtin_bswap32(nxt);
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                const uint32_t j = wi + q;
                const uint32_t xa = (uint32_t)__builtin_amdgcn_readlane((int)cs, (int)(j & 63u));
                const uint32_t xb = (uint32_t)__builtin_amdgcn_readlane((int)ns2, (int)(j & 63u));
                a[q] = j < 64 ? xa : xb;
            }
        }
        if (wb + wi + 4 >= nfull) {  // the stream's end: its partial word, zeros after
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                const uint64_t j = wb + wi + q;
                a[q] = j < nfull ? a[q] : j == nfull ? tailw : 0u;
            }
        }
        const uint64_t x0 = ((uint64_t)a[0] << 32) | a[1], x1 = ((uint64_t)a[2] << 32) | a[3];
        const uint64_t x2 = (uint64_t)a[4] << 32;
        const uint64_t whi = off ? (x0 << off) | (x1 >> (64 - off)) : x0;
        const uint64_t wlo = off ? (x1 << off) | (x2 >> (64 - off)) : x1;
        const uint64_t vj = lane ? (whi << lane) | (wlo >> (64 - lane)) : whi;
        const uint32_t ev = lut[(tsel << kLutBits) + (uint32_t)(vj >> (64 - kLutBits))];
        // chain words: the entry, or 0 (length 0) where the chain must stop
        // for the per-symbol path -- a code longer than the lookup, or the
        // end-of-block symbol
        const uint32_t cw = (ev == kLong || (ev & 0xfffu) == eob) ? 0u : ev;
        // the fast hops: up to `budget` ordinary symbols (the group's rest,
        // the size limit), visited offsets marked in `vis`
        const uint32_t budget = min(gleft, ns_max - ns);
        uint64_t vis = 0;
        uint32_t o = 0, cnt = 0;
        bool special = false;
#if BZ2MI_SYM_JUMP
        // the chain by pointer jumping over the lanes: lane j's successor is
        // j + its code length (64: past the window or a special lane, where
        // the chain ends), R_j the offsets reachable from j; doubling until
        // lane 0's jump leaves the window gives the whole chain from 0
        {
            const uint32_t l1 = cw >> 12;
            const uint32_t nxu = lane + l1;
            const bool spc = l1 == 0;
            uint32_t J = spc ? 64u : min(nxu, 64u);
            uint64_t R = 1ull << lane;
            for (int k = 0; k < 6; ++k) {
                if ((uint32_t)__builtin_amdgcn_readlane((int)J, 0) >= 64u) break;
                const int src = (int)(J & 63u);
                const uint32_t rlo = (uint32_t)__shfl((int)(uint32_t)R, src);
                const uint32_t rhi = (uint32_t)__shfl((int)(uint32_t)(R >> 32), src);
                const uint32_t jn = (uint32_t)__shfl((int)J, src);
                const bool in = J < 64u;
                R |= in ? (((uint64_t)rhi << 32) | rlo) : 0ull;
                J = in ? jn : 64u;
            }
            const uint64_t orbit = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(R >> 32), 0) << 32) |
                                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)R, 0);
            const uint64_t spm = __ballot(spc);
            const uint64_t ord = orbit & ~spm;  // ordinary codes on the chain, in order
            const uint32_t rk = (uint32_t)__popcll(ord & ((1ull << lane) - 1ull));
            vis = __ballot(((ord >> lane) & 1u) && rk < budget);  // the first `budget` of them
            cnt = (uint32_t)__popcll(vis);
            if (cnt == budget) {  // stopped by the budget (even before a special code): after the last taken
                o = (uint32_t)__builtin_amdgcn_readlane((int)nxu, 63 - __builtin_clzll(vis));
            } else if (orbit & spm) {  // ended at a special code
                o = (uint32_t)__builtin_ctzll(orbit & spm);
                special = true;
            } else {  // ran past the window
                o = (uint32_t)__builtin_amdgcn_readlane((int)nxu, 63 - __builtin_clzll(ord));
            }
        }
#elif BZ2MI_SYM_PAIRS
        // two hops at a time: lane j also holds the length of the code that
        // follows its own (0: special or past the window)
        uint32_t pw;
        {
            const uint32_t l1 = cw >> 12, j2 = lane + l1;
            const uint32_t c2 = (uint32_t)__shfl((int)cw, (int)(j2 & 63u));
            const uint32_t l2 = (l1 && j2 < 64) ? (c2 >> 12) : 0u;
            pw = l1 | (l2 << 8);
        }
        for (;;) {
            const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)pw, (int)o);
            const uint32_t l1 = c & 0xffu, l2 = c >> 8;
            if (l1 == 0) {
                special = true;
                break;
            }
            // (branch-free: t = 1 takes both)
            const uint32_t t = (uint32_t)(l2 != 0) & (uint32_t)(cnt + 2 <= budget);
            vis |= (1ull | ((uint64_t)t << l1)) << o;
            o += l1 + (l2 & (0u - t));
            cnt += 1 + t;
            if (cnt == budget || o >= 64) break;
        }
#else
        for (;;) {
            const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cw, (int)o);
            const uint32_t len = c >> 12;
            if (len == 0) {
                special = true;
                break;
            }
            vis |= 1ull << o;
            o += len;
            if (++cnt == budget || o >= 64) break;
        }
#endif
        // the window's symbols: the visited lanes in order (offsets increase)
        if ((vis >> lane) & 1u) {
            const uint32_t rk = (uint32_t)__popcll(vis & ((1ull << lane) - 1ull));
            so[ns + rk] = (uint16_t)(ev & 0xfffu);
        }
        ns += cnt;
        gleft -= cnt;
        if (!special) {
            if (ns >= ns_max) {  // (an ordinary symbol: not the end of block)
                status = kDecSize;
                done = true;
            }
        } else {
            // one symbol the slow way: a long code (the reference's limit /
            // base walk on the window's bits) or the end of block
            const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)ev, (int)o);
            uint32_t sym = e & 0xfffu, len = e >> 12;
            if (e == kLong) {
                const uint64_t x = o ? (whi << o) | (wlo >> (64 - o)) : whi;
                const int32_t* lt = lim + tsel * (kMaxDecLen + 2);
                const int32_t* bt = bas + tsel * (kMaxDecLen + 2);
                sym = 0xffffffffu;
                len = 0;
                for (uint32_t l2 = kLutBits + 1; l2 <= (uint32_t)kMaxDecLen; ++l2) {
                    const int32_t cv = (int32_t)(x >> (64 - l2));
                    if (cv <= lt[l2]) {
                        len = l2;
                        sym = per[tsel * kMaxAlpha + (uint32_t)(cv + bt[l2])];
                        break;
                    }
                }
            }
            if (sym == 0xffffffffu) {
                status = kDecData;
                done = true;
            } else {
                if (lane == 0) so[ns] = (uint16_t)sym;
                ++ns;
                o += len;
                --gleft;
                if (sym == eob || ns >= ns_max) {
                    if (sym != eob) status = kDecSize;
                    done = true;
                }
            }
        }
        if (!done && gleft == 0) {  // next group of 50 (HuffmanStageDecoder.hpp:50-57): its table
            if (++g >= nsel) {
                status = kDecData;
                done = true;
            } else {
                if ((g & 3u) == 0) {
                    swc = swn;
                    swn = sw[(g >> 2) + 1];
                }
                tsel = (swc >> (8 * (g & 3u))) & 255u;
                gleft = kGroupRun;
            }
        }
        bo += o;
      }
      if (!done) {
          bo -= 64 * 32;
          wb += 64;
          cur = raw_word(wb + 64);
      }
    };
    while (!done) {
        run_ring(ra, rb);
        if (done) break;
        run_ring(rb, ra);
    }
    // zeros up to the next multiple of 64 symbols (inside the stride)
    {
        const uint32_t z = (ns & ~63u) + lane;
        if (z >= ns && (ns & 63u)) so[z] = 0;
    }
    const uint64_t pos = wb * 32 + bo;
    if (pos > n * 8) status = kDecData;
    if (lane == 0) {
        info->status = status;
        info->nsym = ns;
        info->end_bit = pos;
    }
}

// ---- K2b: data, part 2 (BlockDecompressor::decodeHuffmanData :177-231):
// RUNA/RUNB runs and inverse move-to-front, one wave per block of the chain.
// Lane c takes the c-th 64th of the block's symbols (its start moved past run
// digits, so no run is split), and the serial list is broken up:
//   pass A  every lane decodes its chunk against a *symbolic* start list
//           (entries = indices into the list at its chunk start): its own
//           recency list (LDS, 4 entries per word, [word][lane]) and the set
//           of start indices it took (LDS bit set).  Rank r < D picks recency
//           entry r; r >= D picks the (r-D)-th untaken start index.  Every
//           symbol leaves (symbolic value | byte count << 8) in a scratch word;
//   pass B  the start lists are composed left to right (entries = output
//           bytes, list 0 = the symbol map):
//           list_{c+1} = list_c[recency_c] ++ list_c[untaken_c ascending],
//   pass C  and, with list_c known, the wave writes chunk c's bytes (lanes on
//           consecutive symbols, offsets by a wave scan of the byte counts).
// A symbol costs its lane ~rank/4 LDS word shifts instead of a serial pass
// of the whole wave.
// BZ2MI_MTF_QUAD (default): the recency list as 16-byte quads ([quad][lane],
// entry 16q + 4j + i in byte i of word j), so a move to front shifts 16
// entries per LDS read/write pair instead of 4.
#ifndef BZ2MI_MTF_QUAD
#define BZ2MI_MTF_QUAD 1
#endif
// BZ2MI_MTF_BFI: every quad blended with its mask, only the write predicated
#ifndef BZ2MI_MTF_BFI
#define BZ2MI_MTF_BFI 1
#endif
#ifndef BZ2MI_MTF_QGROUP
#define BZ2MI_MTF_QGROUP 4
#endif
#ifndef BZ2MI_MTF_PREFETCH
#define BZ2MI_MTF_PREFETCH 16
#endif
// BZ2MI_DMTF_WAVES (decode.hpp): waves per block in pass A (chunks = 64 x
// waves); passes B + C run on wave 0.
constexpr uint32_t kMW = BZ2MI_DMTF_WAVES;
constexpr uint32_t kMC = 64 * kMW;  // chunks per block
struct MtfLds {
#if BZ2MI_MTF_QUAD
    uint4 rec4[16][kMC];     // [quad][chunk] recency list
#else
    uint32_t rec[64][kMC];   // [word][chunk] recency list, entry 4w+j in byte j
#endif
    uint32_t used[8][kMC];   // [word][chunk] start indices taken
    uint32_t ca[kMC];        // chunk starts
    uint32_t cnt[kMC];       // chunk byte counts -> output offsets
    uint8_t lists[2][256];   // start lists of chunk c and c+1, as output bytes
};

// word w (entries 4w..4w+3) of lane `lane`'s recency list
__device__ __forceinline__ uint32_t& rec_word(MtfLds& L, uint32_t w, uint32_t lane) {
#if BZ2MI_MTF_QUAD
    return reinterpret_cast<uint32_t*>(&L.rec4[w >> 2][lane])[w & 3];
#else
    return L.rec[w][lane];
#endif
}

__device__ __forceinline__ uint32_t select_zero(uint32_t u, uint32_t k) {
    // index of the k-th (0-based) zero bit of u, LSB first (k < popc(~u))
    uint32_t x = ~u, pos = 0;
#pragma unroll
    for (int sh = 16; sh; sh >>= 1) {
        const uint32_t c = (uint32_t)__popc(x & ((1u << sh) - 1u));
        if (k >= c) {
            k -= c;
            x >>= sh;
            pos += sh;
        }
    }
    return pos;
}

__global__ __launch_bounds__(kDecMtfThreads) void dec_mtf_kernel(const uint16_t* __restrict__ syms, size_t sym_stride,
                                                     const uint8_t* __restrict__ symmaps,
                                                     const uint32_t* __restrict__ blocks,
                                                     const uint32_t* __restrict__ sym_row, uint32_t nblocks,
                                                     uint32_t smax, uint32_t* __restrict__ scratch, size_t sstride,
                                                     uint8_t* __restrict__ bwt, size_t stride,
                                                     DecBlockInfo* __restrict__ infos) {
    __shared__ MtfLds L;
    const uint32_t bi = blockIdx.x;
    if (bi >= nblocks) return;
    const int lane = lane_id();
    const uint32_t ch = threadIdx.x;  // this thread's chunk
    const uint32_t k = uniform(blocks[bi]);
    DecBlockInfo* info = infos + k;
    const uint32_t ns = uniform(info->nsym), eob = uniform(info->alpha) + 1, orig = uniform(info->orig);
    const uint16_t* so = syms + (size_t)sym_row[bi] * sym_stride;
    uint32_t* tv = scratch + (size_t)bi * sstride;
    uint8_t* out = bwt + (size_t)bi * stride;  // (rows by chain position)
    // chunk [a, b): nominal kMC-th, start moved past run digits
    uint32_t a = (uint32_t)((uint64_t)ns * ch / kMC);
    if (ch)
        while (a < ns && so[a] <= 1) ++a;
    L.ca[ch] = a;
    __syncthreads();
    const uint32_t b = ch == kMC - 1 ? ns : L.ca[ch + 1];
    // ---- pass A
#pragma unroll
    for (int w = 0; w < 8; ++w) L.used[w][ch] = 0;
    uint32_t D = 0, run = 0, inc = 1, runpos = 0, cnt = 0;
    bool inrun = false;
    auto flush_run = [&]() {
        const uint32_t front = D ? (rec_word(L, 0, ch) & 255u) : 0u;
        tv[runpos] = front | (run << 8);
        cnt += run;
        inrun = false;
    };
    // the chunk's symbols arrive 8 at a time (16-byte loads), the next 8
    // loaded while the current 8 are decoded: a load per symbol, waited on
    // at once, was a memory latency per symbol
    const uint32_t glast = (uint32_t)(sym_stride - 8);  // last 8-group of the row (the stride is a multiple of 64)
    uint32_t gcur = a & ~7u;
    uint4 qc = make_uint4(0, 0, 0, 0), qn = make_uint4(0, 0, 0, 0);
    if (a < b) {
        qc = *reinterpret_cast<const uint4*>(so + gcur);
        qn = *reinterpret_cast<const uint4*>(so + min(gcur + 8, glast));
    }
    for (uint32_t p = a; p < b; ++p) {
        if (p >= gcur + 8) {
            gcur += 8;
            qc = qn;
            qn = *reinterpret_cast<const uint4*>(so + min(gcur + 8, glast));
        }
        const uint32_t wq = (p >> 1) & 3u;
        const uint32_t dw = wq == 0 ? qc.x : wq == 1 ? qc.y : wq == 2 ? qc.z : qc.w;
        const uint32_t s = (p & 1u) ? dw >> 16 : dw & 0xffffu;
        if (s <= 1) {  // RUNA / RUNB digit
            if (!inrun) {
                inrun = true;
                runpos = p;
                run = 0;
                inc = 1;
            } else {
                tv[p] = 0;
            }
            run += inc << s;
            inc <<= 1;
            if (run > smax) run = smax + 1;  // saturate (the total check reports it)
            continue;
        }
        if (inrun) flush_run();
        if (s >= eob) {  // end of block (always the last symbol)
            tv[p] = 0;
            continue;
        }
        const uint32_t r = s - 1;
        uint32_t v, rr;
        if (r < D) {
            v = (rec_word(L, r >> 2, ch) >> (8 * (r & 3))) & 255u;
            rr = r;
        } else {
            uint32_t kk = r - D;
            v = 255u;
            for (int w = 0; w < 8; ++w) {
                const uint32_t u = L.used[w][ch];
                const uint32_t z = 32u - (uint32_t)__popc(u);
                if (kk < z) {
                    v = (uint32_t)w * 32u + select_zero(u, kk);
                    break;
                }
                kk -= z;
            }
            L.used[v >> 5][ch] |= 1u << (v & 31);
            rr = D;
            D++;
        }
        // entries [0, rr) move up one place, v goes to the front: words in
        // groups of 8 (eight independent LDS reads in flight, then the shifts)
        uint32_t carry = v;
        const uint32_t wl = rr >> 2;
        const uint32_t mlast = (rr & 3) == 3 ? 0xffffffffu : ((1u << (8 * ((rr & 3) + 1))) - 1u);
#if BZ2MI_MTF_QUAD
#if BZ2MI_MTF_BFI
        // quads in groups of kQG: reads in flight (unpredicated: a group
        // never passes quad 15), then the shifts; every quad is blended with
        // its mask (all bytes below quad ql, the partial mask at ql) and only
        // the write is predicated
        constexpr uint32_t kQG = BZ2MI_MTF_QGROUP;
        static_assert(16 % kQG == 0, "groups inside the 16 quads");
        const uint32_t ql = rr >> 4, cj = wl & 3u;
        const uint32_t m0 = cj > 0 ? 0xffffffffu : mlast;
        const uint32_t m1 = cj > 1 ? 0xffffffffu : cj == 1 ? mlast : 0u;
        const uint32_t m2 = cj > 2 ? 0xffffffffu : cj == 2 ? mlast : 0u;
        const uint32_t m3 = cj == 3 ? mlast : 0u;
        for (uint32_t g0 = 0; g0 <= ql; g0 += kQG) {
            uint4 o[kQG];
#pragma unroll
            for (uint32_t i = 0; i < kQG; ++i) o[i] = L.rec4[g0 + i][ch];
#pragma unroll
            for (uint32_t i = 0; i < kQG; ++i) {
                const uint32_t q = g0 + i;
                uint4 sh;
                sh.x = (o[i].x << 8) | carry;
                sh.y = __builtin_amdgcn_alignbit(o[i].y, o[i].x, 24);
                sh.z = __builtin_amdgcn_alignbit(o[i].z, o[i].y, 24);
                sh.w = __builtin_amdgcn_alignbit(o[i].w, o[i].z, 24);
                carry = o[i].w >> 24;
                const bool full = q < ql;
                const uint32_t k0 = full ? 0xffffffffu : m0, k1 = full ? 0xffffffffu : m1;
                const uint32_t k2 = full ? 0xffffffffu : m2, k3 = full ? 0xffffffffu : m3;
                const uint4 nv = make_uint4((sh.x & k0) | (o[i].x & ~k0), (sh.y & k1) | (o[i].y & ~k1),
                                            (sh.z & k2) | (o[i].z & ~k2), (sh.w & k3) | (o[i].w & ~k3));
                if (q <= ql) L.rec4[q][ch] = nv;
            }
        }
#else
        // quads in groups of kQG: reads in flight, then the shifts
        constexpr uint32_t kQG = BZ2MI_MTF_QGROUP;
        const uint32_t ql = rr >> 4, cj = wl & 3u;
        for (uint32_t g0 = 0; g0 <= ql; g0 += kQG) {
            uint4 o[kQG];
#pragma unroll
            for (uint32_t i = 0; i < kQG; ++i) o[i] = g0 + i <= ql ? L.rec4[g0 + i][ch] : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (uint32_t i = 0; i < kQG; ++i) {
                const uint32_t q = g0 + i;
                if (q > ql) break;
                uint4 sh;
                sh.x = (o[i].x << 8) | carry;
                sh.y = __builtin_amdgcn_alignbit(o[i].y, o[i].x, 24);
                sh.z = __builtin_amdgcn_alignbit(o[i].z, o[i].y, 24);
                sh.w = __builtin_amdgcn_alignbit(o[i].w, o[i].z, 24);
                carry = o[i].w >> 24;
                if (q < ql) {
                    L.rec4[q][ch] = sh;
                } else {
                    const uint32_t m0 = cj > 0 ? 0xffffffffu : mlast;
                    const uint32_t m1 = cj > 1 ? 0xffffffffu : cj == 1 ? mlast : 0u;
                    const uint32_t m2 = cj > 2 ? 0xffffffffu : cj == 2 ? mlast : 0u;
                    const uint32_t m3 = cj == 3 ? mlast : 0u;
                    L.rec4[q][ch] = make_uint4((sh.x & m0) | (o[i].x & ~m0), (sh.y & m1) | (o[i].y & ~m1),
                                                 (sh.z & m2) | (o[i].z & ~m2), (sh.w & m3) | (o[i].w & ~m3));
                }
            }
        }
#endif
#else
        for (uint32_t g0 = 0; g0 <= wl; g0 += 8) {
            uint32_t o[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = g0 + i <= wl ? L.rec[g0 + i][ch] : 0u;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t w = g0 + i;
                if (w > wl) break;
                const uint32_t sh = (o[i] << 8) | carry;
                carry = o[i] >> 24;
                L.rec[w][ch] = w < wl ? sh : ((sh & mlast) | (o[i] & ~mlast));
            }
        }
#endif
        tv[p] = v | (1u << 8);
        cnt += 1;
    }
    if (inrun) flush_run();
    // the chunk's list permutation: recency entries, then untaken indices ascending
    {
        uint32_t pos = D;
        for (int w = 0; w < 8 && pos < 256; ++w) {
            uint32_t z = ~L.used[w][ch];
            while (z && pos < 256) {
                const uint32_t bit = (uint32_t)__builtin_ctz(z);
                z &= z - 1;
                const uint32_t e = (uint32_t)w * 32u + bit;
                uint32_t& wd = rec_word(L, pos >> 2, ch);
                const uint32_t sh = 8 * (pos & 3);
                wd = (wd & ~(0xffu << sh)) | (e << sh);
                pos++;
            }
        }
    }
    // ---- passes B + C, chunk by chunk with the whole wave: list_c (entries =
    // output bytes; list_0 = the symbol map), then the chunk's bytes -- lanes
    // take consecutive symbols, offsets by a wave scan of their byte counts --
    // then list_{c+1}[i] = list_c[perm_c[i]]
    L.cnt[ch] = cnt;
    __syncthreads();
    if (ch >= 64) return;  // (passes B + C: wave 0)
    uint32_t total;
    {
        // lane l: chunks l*kMW .. l*kMW+kMW-1 -> their output offsets
        uint32_t cs[kMW], sum = 0;
#pragma unroll
        for (uint32_t i = 0; i < kMW; ++i) {
            cs[i] = L.cnt[lane * kMW + i];
            sum += cs[i];
        }
        const uint32_t incl = wave_incl_sum(sum);
        total = uniform((uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
        uint32_t acc = incl - sum;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t i = 0; i < kMW; ++i) {
            L.cnt[lane * kMW + i] = acc;
            acc += cs[i];
        }
        __builtin_amdgcn_wave_barrier();
    }
    uint32_t status = total > smax ? (uint32_t)kDecSize : 0u;
    const uint8_t* smp = symmaps + (size_t)k * 256;
#pragma unroll
    for (int j = 0; j < 4; ++j) L.lists[0][lane * 4 + j] = smp[lane * 4 + j];
    __builtin_amdgcn_wave_barrier();
    for (uint32_t c = 0; c < kMC && !status; ++c) {
        const uint8_t* lc = L.lists[c & 1];
        const uint32_t ca = uniform(L.ca[c]);
        const uint32_t cb = c == kMC - 1 ? ns : uniform(L.ca[c + 1]);
        uint32_t o = uniform(L.cnt[c]);
#if BZ2MI_MTF_PREFETCH > 1
        // the chunk's scratch words kPF 64-symbol steps at a time, the next
        // kPF loaded while these are written out: one load in flight per
        // step was a memory latency per 64 symbols (the wave walks the
        // block's symbols serially here)
        constexpr uint32_t kPF = BZ2MI_MTF_PREFETCH;
        uint32_t xb[kPF];
#pragma unroll
        for (uint32_t i = 0; i < kPF; ++i) {
            const uint32_t pn = ca + 64u * i + (uint32_t)lane;
            xb[i] = pn < cb ? tv[pn] : 0u;
        }
        for (uint32_t p0 = ca; p0 < cb; p0 += 64u * kPF) {
            uint32_t xc[kPF];
#pragma unroll
            for (uint32_t i = 0; i < kPF; ++i) {
                xc[i] = xb[i];
                const uint32_t pn = p0 + 64u * (kPF + i) + (uint32_t)lane;
                xb[i] = pn < cb ? tv[pn] : 0u;
            }
#pragma unroll
            for (uint32_t i = 0; i < kPF; ++i) {
                if (p0 + 64u * i >= cb) break;
                const uint32_t x = xc[i];
                const uint32_t n1 = x >> 8;
                const uint32_t inc1 = wave_incl_sum(n1);
                uint32_t q = o + inc1 - n1;
                if (n1) {
                    const uint8_t byte = lc[x & 255u];
                    for (uint32_t r2 = 0; r2 < n1; ++r2) out[q + r2] = byte;
                }
                o += (uint32_t)__builtin_amdgcn_readlane((int)inc1, 63);
            }
        }
#else
        uint32_t xn = ca + (uint32_t)lane < cb ? tv[ca + lane] : 0u;  // one 64-symbol step ahead
        for (uint32_t p0 = ca; p0 < cb; p0 += 64) {
            const uint32_t x = xn;
            const uint32_t pn = p0 + 64 + (uint32_t)lane;
            xn = pn < cb ? tv[pn] : 0u;
            const uint32_t n1 = x >> 8;
            const uint32_t inc1 = wave_incl_sum(n1);
            uint32_t q = o + inc1 - n1;
            if (n1) {
                const uint8_t byte = lc[x & 255u];
                for (uint32_t r2 = 0; r2 < n1; ++r2) out[q + r2] = byte;
            }
            o += (uint32_t)__builtin_amdgcn_readlane((int)inc1, 63);
        }
#endif
        if (c < kMC - 1) {
            uint32_t nv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t pi = (rec_word(L, lane, c) >> (8 * j)) & 255u;  // entry 4*lane + j of chunk c
                nv[j] = lc[pi];
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = 0; j < 4; ++j) L.lists[(c + 1) & 1][lane * 4 + j] = (uint8_t)nv[j];
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (status == 0 && orig >= total) status = kDecOrigPtr;
    if (lane == 0) {
        info->len = status == kDecSize ? 0u : total;
        if (status) info->status = status;
    }
}

// ---- K3: inverse BWT, one workgroup (256 threads) per block.  merged[r] =
// (i << 8) | byte for the stable counting sort of the BWT bytes (BlockDecompressor
// ::initialiseInverseBWT :233-262); the LF cycle from origPtr is the RLE1
// block.  2048 walkers (8 per thread) start at evenly spaced rows (walker 0 at
// origPtr), walk to the next start row (pass A: segment lengths and
// successors), thread 0 chains the segments from walker 0, and the walkers
// walk again writing their segment's bytes (pass B).
constexpr int kIT = kDecIbwtThreads;  // threads per inverse-BWT workgroup
constexpr int kIW = kIT / 64;
constexpr int kWPT = 8;               // walkers per thread
constexpr int kWalkers = kIT * kWPT;  // per block
constexpr uint16_t kEnd = 0xffff;
static_assert(kWalkers <= 0xffff, "walker ids fit 16 bits");
// BZ2MI_IBWT_ONEWALK (default): one walk of the LF cycle instead of two --
// every walker keeps its segment's bytes (8 in registers, stored 8 at a
// time to its kWCap-byte area of the workgroup's scratch) while it measures
// the segment, and once the segments are chained the bytes are copied to
// their offsets; only the bytes of a segment beyond kWCap (mean length n /
// 8192 ~ 11: about 1 segment in 10^5 at S = 90,000) are walked a second time.
// The walks are random 4-byte loads from the merged vector (a 64-byte line
// each): one walk halves them.
#ifndef BZ2MI_IBWT_ONEWALK
#define BZ2MI_IBWT_ONEWALK 1
#endif
constexpr uint32_t kWCap = BZ2MI_IBWT_WCAP;
static_assert((size_t)kWalkers * kWCap == kDecIbwtScratch, "walker scratch layout");

struct IbwtLds {
    uint32_t base[kIW][256];   // per-wave byte counts -> merged-vector bases
    uint32_t seglen[kWalkers];
    uint32_t sfx[kWalkers];    // suffix sums of segment lengths along the chain
    uint16_t nxt[kWalkers];    // successor segment (pointer jumping), kEnd past the last
#if BZ2MI_IBWT_ONEWALK
    uint32_t resume[kWalkers]; // row of byte kWCap of a segment longer than kWCap
#endif
    uint32_t tmp[kIW];
    uint32_t period;
};

__device__ __forceinline__ void ibwt_one(IbwtLds& L, uint32_t bi, const uint8_t* __restrict__ bwt, size_t stride,
                                         const DecBlockInfo* __restrict__ infos, const uint32_t* __restrict__ blocks,
                                         uint32_t* __restrict__ merged, size_t mstride, uint32_t* __restrict__ marks,
                                         size_t kstride, uint8_t* __restrict__ rle1, size_t rstride,
                                         uint32_t* __restrict__ bad_out, uint8_t* __restrict__ ws) {
    const uint32_t k = blocks[bi];  // decoded-candidate index
    const int t = threadIdx.x, w = wave_id(), lane = lane_id();
    const uint32_t n = infos[k].len;
    const uint32_t orig = infos[k].orig;
    const uint8_t* B = bwt + (size_t)bi * stride;
    uint32_t* M = merged + (size_t)bi * mstride;
    uint32_t* mark = marks + (size_t)bi * kstride;  // walker id of each start row
    uint8_t* out = rle1 + (size_t)bi * rstride;
    uint32_t* bad = bad_out + bi;
    // per-wave counts of each byte over the wave's 16th of the block
    const uint32_t q0 = (uint32_t)((uint64_t)n * w / kIW), q1 = (uint32_t)((uint64_t)n * (w + 1) / kIW);
    for (int j = 0; j < 4; ++j) L.base[w][lane * 4 + j] = 0;
    __syncthreads();
    for (uint32_t p0 = q0; p0 < q1; p0 += 64) {
        const uint32_t p = p0 + lane;
        const bool v = p < q1;
        const uint32_t c = v ? B[p] : 0u;
        const uint64_t peers = wave_match8(c, v);
        if (v && (peers & __lanemask_lt()) == 0) atomicAdd(&L.base[w][c], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    {
        // thread t < 256: byte t -> C[t] + counts of the earlier waves' parts
        uint32_t h = 0;
        if (t < 256)
            for (int q = 0; q < kIW; ++q) h += L.base[q][t];
        uint32_t total;
        const uint32_t cb = wg_excl_sum<kIT>(h, L.tmp, &total);
        __syncthreads();
        if (t < 256) {
            uint32_t acc = cb;
            for (int q = 0; q < kIW; ++q) {
                const uint32_t c = L.base[q][t];
                L.base[q][t] = acc;
                acc += c;
            }
        }
    }
    __syncthreads();
    for (uint32_t p0 = q0; p0 < q1; p0 += 64) {
        const uint32_t p = p0 + lane;
        const bool v = p < q1;
        const uint32_t c = v ? B[p] : 0u;
        const uint64_t peers = wave_match8(c, v);
        const uint64_t below = peers & __lanemask_lt();
        const uint32_t r = v ? L.base[w][c] + (uint32_t)__popcll(below) : 0u;
        __builtin_amdgcn_wave_barrier();
        if (v && below == 0) L.base[w][c] += (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        if (v) M[r] = (p << 8) | c;
    }
    // walker starts: walker 0 at origPtr, walker j at j*n/K (skipped when it
    // collides with an earlier start).  A start row gets bit 31 in merged[]
    // (i < 2^24, so the bit is free) and its walker id in mark[].
    __threadfence_block();
    __syncthreads();
    auto start_of = [&](int j) -> uint32_t { return j == 0 ? orig : (uint32_t)((uint64_t)n * j / kWalkers); };
    auto is_start = [&](int j) -> bool {
        const uint32_t s0 = start_of(j);
        return n > 0 && (j == 0 || (s0 != orig && s0 != start_of(j - 1)));
    };
    for (int j = t; j < kWalkers; j += kIT) {
        L.seglen[j] = 0;
        L.nxt[j] = kEnd;
        if (is_start(j)) {
            const uint32_t s0 = start_of(j);
            mark[s0] = (uint32_t)j;
            M[s0] |= 0x80000000u;
        }
    }
    __threadfence_block();
    __syncthreads();
    // pass A (kWPT walkers per thread): one load per walker and step -- the
    // entry of the row just reached tells whether it starts a segment; the
    // loads of all the thread's walkers are issued together
    uint32_t x[kWPT], len[kWPT], m[kWPT];
    bool act[kWPT];
#if BZ2MI_IBWT_ONEWALK
    uint32_t bw[kWPT][2];  // the segment's pending bytes (8), stored 8 at a time
#pragma unroll
    for (int q = 0; q < kWPT; ++q) {
        const int j = t + kIT * q;
        act[q] = is_start(j);
        x[q] = start_of(j);
        len[q] = 0;
        m[q] = act[q] ? M[x[q]] : 0u;
        bw[q][0] = bw[q][1] = 0;
    }
    {
        bool any1 = true;
        while (any1) {
            uint32_t nx[kWPT], mv[kWPT];
#pragma unroll
            for (int q = 0; q < kWPT; ++q) {
                nx[q] = (m[q] & 0x7fffffffu) >> 8;
                if (act[q] && (nx[q] >= n || len[q] >= n)) {  // inconsistent data (never for valid blocks)
                    act[q] = false;
                    if (bad) *bad = 1u;
                }
                if (act[q] && len[q] < kWCap) {
                    // byte len of the segment: the row's own byte
                    const uint32_t kb = len[q], by = m[q] & 255u, sh = 8u * (kb & 3u);
                    const bool hi = (kb & 4u) != 0;
                    bw[q][0] |= hi ? 0u : by << sh;
                    bw[q][1] |= hi ? by << sh : 0u;
                    if ((kb & 7u) == 7u) {
                        *reinterpret_cast<uint2*>(ws + (size_t)(t + kIT * q) * kWCap + (kb & ~7u)) =
                            make_uint2(bw[q][0], bw[q][1]);
                        bw[q][0] = bw[q][1] = 0;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < kWPT; ++q) mv[q] = act[q] ? M[nx[q]] : 0u;
            any1 = false;
#pragma unroll
            for (int q = 0; q < kWPT; ++q) {
                if (!act[q]) continue;
                const int j = t + kIT * q;
                len[q]++;
                x[q] = nx[q];
                m[q] = mv[q];
                if (len[q] == kWCap) L.resume[j] = x[q];
                if (m[q] >> 31) {
                    act[q] = false;
                    L.seglen[j] = len[q];
                    if (len[q] < kWCap && (len[q] & 7u))  // the last partial 8
                        *reinterpret_cast<uint2*>(ws + (size_t)j * kWCap + (len[q] & ~7u)) =
                            make_uint2(bw[q][0], bw[q][1]);
                    const uint32_t sj = mark[x[q]];
                    L.nxt[j] = sj == 0 ? kEnd : (uint16_t)sj;
                } else {
                    any1 = true;
                }
            }
        }
    }
    if (false)
#endif
    {
#pragma unroll
    for (int q = 0; q < kWPT; ++q) {
        const int j = t + kIT * q;
        act[q] = is_start(j);
        x[q] = start_of(j);
        len[q] = 0;
        m[q] = act[q] ? M[x[q]] : 0u;
    }
    bool any = true;
    while (any) {
        uint32_t nx[kWPT], mv[kWPT];
#pragma unroll
        for (int q = 0; q < kWPT; ++q) {
            nx[q] = (m[q] & 0x7fffffffu) >> 8;
            if (act[q] && (nx[q] >= n || len[q] >= n)) {  // inconsistent data (never for valid blocks)
                act[q] = false;
                if (bad) *bad = 1u;
            }
        }
#pragma unroll
        for (int q = 0; q < kWPT; ++q) mv[q] = act[q] ? M[nx[q]] : 0u;
        any = false;
#pragma unroll
        for (int q = 0; q < kWPT; ++q) {
            if (!act[q]) continue;
            len[q]++;
            x[q] = nx[q];
            m[q] = mv[q];
            if (m[q] >> 31) {
                act[q] = false;
                L.seglen[t + kIT * q] = len[q];
                const uint32_t sj = mark[x[q]];
                // the segment that returns to walker 0 ends the chain
                L.nxt[t + kIT * q] = sj == 0 ? kEnd : (uint16_t)sj;
            } else {
                any = true;
            }
        }
    }
    }
    __syncthreads();
    // chain the segments of origPtr's cycle by pointer jumping: sfx[j] = the
    // lengths from segment j to the chain's last; a segment's offset is
    // period - sfx[j].  Segments on other cycles never reach kEnd: a periodic
    // block (T = u^k, the SURVEY H2 case) has k cycles of n/k rows and its
    // output is the first cycle's bytes repeated, as the reference's n-step
    // walk produces.
#pragma unroll
    for (int q = 0; q < kWPT; ++q) L.sfx[t + kIT * q] = L.seglen[t + kIT * q];
    __syncthreads();
    for (int round = 0; (1 << round) < kWalkers; ++round) {
        uint32_t sv[kWPT];
        uint16_t nv[kWPT];
#pragma unroll
        for (int q = 0; q < kWPT; ++q) {
            const int j = t + kIT * q;
            const uint16_t nj = L.nxt[j];
            sv[q] = L.sfx[j] + (nj != kEnd ? L.sfx[nj] : 0u);
            nv[q] = nj != kEnd ? L.nxt[nj] : kEnd;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kWPT; ++q) {
            L.sfx[t + kIT * q] = sv[q];
            L.nxt[t + kIT * q] = nv[q];
        }
        __syncthreads();
    }
    if (t == 0) {
        const uint32_t o = n > 0 && L.nxt[0] == kEnd ? L.sfx[0] : 0u;
        L.period = o;
        if ((o == 0 || o > n || n % o != 0) && bad) *bad = 1u;
    }
    __syncthreads();
    const uint32_t per = L.period;
    // pass B: write the bytes of each segment
    uint32_t o[kWPT];
#if BZ2MI_IBWT_ONEWALK
    // the kept bytes to their offsets; segments longer than kWCap walk on
    // from their resume row for the rest
#pragma unroll
    for (int q = 0; q < kWPT; ++q) {
        const int j = t + kIT * q;
        const uint32_t sl = L.seglen[j], sf = L.sfx[j];
        const bool placed = is_start(j) && L.nxt[j] == kEnd && sf <= per && sl > 0;
        o[q] = placed ? per - sf : 0u;
        const uint32_t keep = placed ? min(sl, kWCap) : 0u;
        const uint8_t* src = ws + (size_t)j * kWCap;
        for (uint32_t c0 = 0; c0 < keep; c0 += 16) {
            const uint4 v = *reinterpret_cast<const uint4*>(src + c0);
            const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int b = 0; b < 16; ++b)
                if (c0 + (uint32_t)b < keep) out[o[q] + c0 + (uint32_t)b] = (uint8_t)(vv[b >> 2] >> (8 * (b & 3)));
        }
        len[q] = placed && sl > kWCap ? sl - kWCap : 0u;
        x[q] = len[q] ? L.resume[j] : 0u;
        o[q] += kWCap;
    }
    if (false)
#endif
    {
#pragma unroll
    for (int q = 0; q < kWPT; ++q) {
        const int j = t + kIT * q;
        act[q] = is_start(j);
        x[q] = start_of(j);
        const uint32_t sl = L.seglen[j], sf = L.sfx[j];
        const bool placed = act[q] && L.nxt[j] == kEnd && sf <= per && sl > 0;
        len[q] = placed ? sl : 0u;
        o[q] = placed ? per - sf : 0u;
    }
    }
    bool any = true;
    while (any) {
        uint32_t mv[kWPT];
#pragma unroll
        for (int q = 0; q < kWPT; ++q) mv[q] = len[q] ? M[x[q]] : 0u;
        any = false;
#pragma unroll
        for (int q = 0; q < kWPT; ++q) {
            if (!len[q]) continue;
            const uint32_t mm = mv[q] & 0x7fffffffu;
            out[o[q]++] = (uint8_t)mm;
            x[q] = mm >> 8;
            if (x[q] >= n) len[q] = 1;
            if (--len[q]) any = true;
        }
    }
    if (per && per < n && n % per == 0) {
        __threadfence_block();
        __syncthreads();
        for (uint32_t i = per + t; i < n; i += kIT) out[i] = out[i % per];
    }
}

// A persistent grid of one 1024-thread workgroup per CU (BZ2MI_IBWT_XCD
// per XCD, blocks taken in turn): 8192 walkers per block, 2M loads in flight
// chip-wide.  The walks are dependent random 4-byte loads, latency-bound:
// fewer workgroups (to keep the merged vectors in the XCDs' L2) measured
// slower, 8/16/24/32 per XCD: 101/64/55/58 ms per GiB random (the round-1
// kernel with 2048 walkers per block and 512 blocks in flight: 62).
__global__ __launch_bounds__(kIT) void dec_ibwt_kernel(const uint8_t* __restrict__ bwt, size_t stride,
                                                       const DecBlockInfo* __restrict__ infos,
                                                       const uint32_t* __restrict__ blocks, uint32_t nblocks,
                                                       uint32_t* __restrict__ merged, size_t mstride,
                                                       uint32_t* __restrict__ marks, size_t kstride,
                                                       uint8_t* __restrict__ rle1, size_t rstride,
                                                       uint32_t* __restrict__ bad_out, uint8_t* __restrict__ wscr) {
    __shared__ IbwtLds L;
    // (wscr: kWalkers * kWCap bytes per workgroup of the grid)
    uint8_t* ws = wscr + (size_t)blockIdx.x * ((size_t)kWalkers * kWCap);
    for (uint32_t bi = blockIdx.x; bi < nblocks; bi += gridDim.x) {
        ibwt_one(L, bi, bwt, stride, infos, blocks, merged, mstride, marks, kstride, rle1, rstride, bad_out, ws);
        __syncthreads();
    }
}

// ---- K4: RLE1 expansion (BlockDecompressor::read :55-88).  States before a
// byte: 0 = after a count byte or at the block start (any byte: emit 1, ->1),
// 1..3 = that many equal bytes so far (byte == previous: ->+1, at 3 -> 4 =
// "next byte is a count"; else emit 1, ->1), 4 = this byte is a count k: emit
// the run byte k+1 more... the reference emits k+1 copies of the run byte,
// the fourth included.  pass 0 counts (per chunk and entry state), pass 1
// writes; chunk c of a block covers [c*n/256, (c+1)*n/256).
#ifndef BZ2MI_RLE1_VEC16
#define BZ2MI_RLE1_VEC16 1
#endif
namespace {
struct Rle1Step {
    uint32_t st;
    uint32_t emit;
};
__device__ __forceinline__ uint32_t rle1_next(uint32_t st, uint32_t b, uint32_t prev, uint32_t* emit) {
    if (st == 4) {
        *emit = b + 1;
        return 0;
    }
    if (st == 0 || b != prev) {
        *emit = 1;
        return 1;
    }
    if (st == 3) {
        *emit = 0;
        return 4;
    }
    *emit = 1;
    return st + 1;
}
}  // namespace

__global__ __launch_bounds__(256) void dec_rle1_kernel(const uint8_t* __restrict__ rle1, size_t rstride,
                                                       const DecBlockInfo* __restrict__ infos,
                                                       const uint32_t* __restrict__ blocks, uint32_t nblocks,
                                                       uint32_t* __restrict__ chunk_state, uint64_t* __restrict__ out_len,
                                                       const uint64_t* __restrict__ out_off, uint8_t* __restrict__ out,
                                                       uint64_t cap, uint32_t* __restrict__ crc_out,
                                                       const uint32_t* __restrict__ crc_table, int pass) {
    __shared__ uint32_t ctab[256];
    __shared__ uint32_t clen[256][5];
    __shared__ uint32_t cexit[256][5];
    __shared__ uint32_t centry[256];
    __shared__ uint64_t coff[257];
    __shared__ uint32_t cpart[256];
    const uint32_t bi = blockIdx.x;
    if (bi >= nblocks) return;
    const int t = threadIdx.x;
    const uint32_t k = blocks[bi];
    const uint32_t n = infos[k].len;
    const uint8_t* X = rle1 + (size_t)bi * rstride;
    // chunk bounds on 16-byte boundaries: every thread reads its chunk with
    // 16-byte loads (the block buffer is 256-byte aligned and padded)
    auto cbound = [&](uint32_t c) -> uint32_t {
        return c == 0 ? 0u : (c >= 256 ? n : min(n, (uint32_t)((uint64_t)n * c / 256) & ~15u));
    };
    const uint32_t c0 = cbound(t), c1 = cbound(t + 1);
    auto for_each_byte = [&](auto&& fn) {
        for (uint32_t p = c0; p < c1; p += 16) {
            const uint4 v = *reinterpret_cast<const uint4*>(X + p);
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
            const uint32_t m = min(16u, c1 - p);
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if ((uint32_t)j < m) fn((wv[j >> 2] >> (8 * (j & 3))) & 255u);
        }
    };
    const uint32_t prev0 = c0 ? X[c0 - 1] : 0xffffffffu;
    if (pass == 0) {
        // all five entry states in lockstep until they agree, then one
        uint32_t st[5] = {0, 1, 2, 3, 4}, ln[5] = {0, 0, 0, 0, 0};
        uint32_t prev = prev0, s0 = 0, tail = 0;
        bool same = false;
        for_each_byte([&](uint32_t b) {
            if (!same) {
#pragma unroll
                for (int q = 0; q < 5; ++q) {
                    uint32_t e;
                    st[q] = rle1_next(st[q], b, prev, &e);
                    ln[q] += e;
                }
                same = st[0] == st[1] && st[0] == st[2] && st[0] == st[3] && st[0] == st[4];
                s0 = st[0];
            } else {
                uint32_t e;
                s0 = rle1_next(s0, b, prev, &e);
                tail += e;
            }
            prev = b;
        });
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            clen[t][q] = ln[q] + tail;
            cexit[t][q] = c0 == c1 ? (uint32_t)q : (same ? s0 : st[q]);
        }
        __syncthreads();
        if (t == 0) {
            uint32_t sx = 0;
            uint64_t o = 0;
            for (int c = 0; c < 256; ++c) {
                centry[c] = sx;
                coff[c] = o;
                o += clen[c][sx];
                sx = cexit[c][sx];
            }
            coff[256] = o;
        }
        __syncthreads();
        // entry state and output offset of the chunk (offsets < 2^29: a block
        // expands at most 259/5 times)
        chunk_state[(size_t)bi * 256 + t] = centry[t] | (uint32_t)(coff[t] << 3);
        if (t == 0) out_len[bi] = coff[256];
        return;
    }
    // pass 1: write and CRC
    ctab[t] = crc_table[t];
    const uint32_t cs = chunk_state[(size_t)bi * 256 + t];
    __syncthreads();
    const uint64_t total = out_len[bi];
    const uint64_t base = out_off[bi];
    const uint64_t off = cs >> 3;
    uint64_t o = base + off;
    uint32_t st = cs & 7u, prev = prev0;
    uint32_t r = 0;  // CRC register from 0
#if BZ2MI_RLE1_VEC16
    // the output collects in the 16-byte aligned block that holds o and
    // leaves in one 16-byte store when the block is the chunk's own; the
    // chunk's first and last blocks (shared with the neighbours) byte-wise.
    // (A byte store per output byte was an L2 write request per byte.)
    const uint64_t ostart = o;
    const uint64_t ao = (uint64_t)(reinterpret_cast<uintptr_t>(out) & 15u);  // (blocks by address)
    uint32_t b0w = 0, b1w = 0, b2w = 0, b3w = 0;
    // bytes [lo, hi) of the block at index blk (out + blk 16-byte aligned;
    // blk may lie before the output's start: then lo > 0 skips to ostart)
    auto flush = [&](int64_t blk, uint32_t hi) {
        const uint32_t lo = blk >= (int64_t)ostart ? 0u : (uint32_t)((int64_t)ostart - blk);
        if (lo == 0 && hi == 16 && (uint64_t)blk + 16 <= cap) {
            *reinterpret_cast<uint4*>(out + blk) = make_uint4(b0w, b1w, b2w, b3w);
        } else {
            const uint32_t wv[4] = {b0w, b1w, b2w, b3w};
#pragma unroll
            for (uint32_t j = 0; j < 16; ++j)
                if (j >= lo && j < hi && (uint64_t)(blk + j) < cap) out[blk + j] = (uint8_t)(wv[j >> 2] >> (8 * (j & 3)));
        }
        b0w = b1w = b2w = b3w = 0;
    };
    for_each_byte([&](uint32_t b) {
        uint32_t e;
        const uint32_t was = st;
        st = rle1_next(st, b, prev, &e);
        const uint32_t ob = was == 4 ? prev : b;  // a count byte repeats the run byte before it
        for (uint32_t q = 0; q < e; ++q) {
            const uint32_t pos = (uint32_t)((o + ao) & 15u), v = ob << (8 * (pos & 3u)), ws = pos >> 2;
            b0w |= ws == 0 ? v : 0u;
            b1w |= ws == 1 ? v : 0u;
            b2w |= ws == 2 ? v : 0u;
            b3w |= ws == 3 ? v : 0u;
            o++;
            if (pos == 15u) flush((int64_t)o - 16, 16u);
            r = (r << 8) ^ ctab[(r >> 24) ^ ob];
        }
        prev = b;
    });
    if ((o + ao) & 15u) flush((int64_t)o - (int64_t)((o + ao) & 15u), (uint32_t)((o + ao) & 15u));
#else
    for_each_byte([&](uint32_t b) {
        uint32_t e;
        const uint32_t was = st;
        st = rle1_next(st, b, prev, &e);
        const uint32_t ob = was == 4 ? prev : b;  // a count byte repeats the run byte before it
        for (uint32_t q = 0; q < e; ++q) {
            if (o < cap) out[o] = (uint8_t)ob;
            o++;
            r = (r << 8) ^ ctab[(r >> 24) ^ ob];
        }
        prev = b;
    });
#endif
    // block CRC: chunk registers shifted by the bytes after them
    const uint64_t after = total - (o - base);
    cpart[t] = crc_shift(r, after);
    __syncthreads();
    if (t < 64) {
        uint32_t v = cpart[t] ^ cpart[t + 64] ^ cpart[t + 128] ^ cpart[t + 192];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v ^= (uint32_t)__shfl_xor((int)v, d);
        if (t == 0) crc_out[bi] = ~(v ^ crc_shift(0xffffffffu, total));
    }
}

int dec_set_xpow8(const uint32_t* tab64) {
    return hipMemcpyToSymbol(HIP_SYMBOL(c_xpow8), tab64, 64 * sizeof(uint32_t)) == hipSuccess ? 0 : -1;
}

}  // namespace bz2mi
