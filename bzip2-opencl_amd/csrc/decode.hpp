// Device bzip2 decoder (decode.hip): shared types and kernel entry points.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bz2mi {

// a 48-bit magic found in the stream: bit position, 0 = block header /
// 1 = end of stream, and the 32 bits that follow it (the stored CRC)
struct DecCand {
    uint64_t bitpos;
    uint32_t type;
    uint32_t next32;
};

// status codes of a decoded block (messages in dapi: the reference's texts)
enum : uint32_t {
    kDecOk = 0,
    kDecTables = 1,      // "block Huffman tables invalid"       BlockDecompressor.hpp:158-162
    kDecData = 2,        // "Error decoding  block"              HuffmanStageDecoder.hpp:55,70
    kDecSize = 3,        // "BZip2 block exceeds declared block size"  BlockDecompressor.hpp:211,226
    kDecOrigPtr = 4,     // "BZip2 start pointer invalid"         BlockDecompressor.hpp:237
    kDecRandomised = 5,  // "BZip2 randomised blocks not implemented"  BlockDecompressor.hpp:272
};

struct DecBlockInfo {
    uint64_t end_bit;  // first bit after the block (after its end-of-block symbol)
    uint32_t status;
    uint32_t orig;     // origPtr
    uint32_t len;      // BWT (= RLE1) bytes (dec_mtf_kernel)
    uint32_t crc;      // stored block CRC
    uint32_t nsym;     // Huffman symbols, end-of-block included
    uint32_t alpha;    // symbols in use (the end-of-block symbol is alpha + 1)
    uint64_t data_bit; // first bit of the Huffman data (after the tables)
    uint32_t nsel;     // selectors
    uint32_t pad;
};

// per-candidate decoding tables (dec_huff_kernel -> dec_sym_kernel): 9-bit
// lookup tables, limits and bases per code length, symbol permutations,
// selectors
constexpr size_t kTabLimit = 6 * 512 * 2;                 // after the lookup tables
constexpr size_t kTabBase = kTabLimit + 6 * 25 * 4;
constexpr size_t kTabPerm = kTabBase + 6 * 25 * 4;
constexpr size_t kTabSel = kTabPerm + 6 * 258 * 2 + 8;    // (8: alignment pad)
constexpr size_t kTabBytes = (kTabSel + 18002 + 255) & ~(size_t)255;

__global__ void dec_scan_kernel(const uint8_t* in, uint64_t n, DecCand* cand, uint32_t* ncand, uint32_t cap);
__global__ void dec_huff_kernel(const uint8_t* in, uint64_t n, const DecCand* cand, const uint32_t* ids,
                                uint32_t nids, uint32_t max_sel, uint8_t* tabs, uint8_t* symmap_out,
                                DecBlockInfo* infos);
#ifndef BZ2MI_SYM_BLOCKS
#define BZ2MI_SYM_BLOCKS 2
#endif
constexpr int kDecSymBlocks = BZ2MI_SYM_BLOCKS;  // blocks per wave of dec_sym_kernel
constexpr int kDecIbwtThreads = 1024;             // threads per dec_ibwt_kernel workgroup
// waves per dec_mtf_kernel workgroup (pass A's chunks = 64 x waves): a 900 KB
// batch has ~1,200 blocks, one wave each leaves most SIMDs one latency-bound wave
#ifndef BZ2MI_DMTF_WAVES
#define BZ2MI_DMTF_WAVES 1
#endif
constexpr uint32_t kDecMtfThreads = 64 * BZ2MI_DMTF_WAVES;
// bytes an inverse-BWT walker keeps of its segment (beyond: walked again)
#ifndef BZ2MI_IBWT_WCAP
#define BZ2MI_IBWT_WCAP 128
#endif
constexpr size_t kDecIbwtScratch = (size_t)kDecIbwtThreads * 8 * BZ2MI_IBWT_WCAP;  // walker bytes per dec_ibwt_kernel workgroup
// symbol row j <- candidate sel[j]
__global__ void dec_sym_kernel(const uint8_t* in, uint64_t n, const uint8_t* tabs, const uint32_t* sel, uint32_t nids,
                               uint32_t smax, uint16_t* syms, size_t sym_stride, DecBlockInfo* infos);
__global__ void dec_symw_kernel(const uint8_t* in, uint64_t n, const uint8_t* tabs, const uint32_t* sel, uint32_t nids,
                                uint32_t smax, uint16_t* syms, size_t sym_stride, DecBlockInfo* infos);
// the windowed symbol decoder (one block per wave) instead of dec_sym_kernel
#ifndef BZ2MI_SYM_WINDOW
#define BZ2MI_SYM_WINDOW 1
#endif
// the windowed decoder's chain hops two codes per lane read
#ifndef BZ2MI_SYM_PAIRS
#define BZ2MI_SYM_PAIRS 1
#endif
// ... or finds the window's whole chain by pointer jumping over the lanes
#ifndef BZ2MI_SYM_JUMP
#define BZ2MI_SYM_JUMP 1
#endif
// chain block i: candidate blocks[i], symbol row sym_row[i]; BWT row i
__global__ void dec_mtf_kernel(const uint16_t* syms, size_t sym_stride, const uint8_t* symmaps,
                               const uint32_t* blocks, const uint32_t* sym_row, uint32_t nblocks, uint32_t smax,
                               uint32_t* scratch, size_t sstride, uint8_t* bwt, size_t stride, DecBlockInfo* infos);
__global__ void dec_ibwt_kernel(const uint8_t* bwt, size_t stride, const DecBlockInfo* infos,
                                const uint32_t* blocks, uint32_t nblocks, uint32_t* merged, size_t mstride,
                                uint32_t* marks, size_t kstride, uint8_t* rle1, size_t rstride, uint32_t* bad,
                                uint8_t* wscr);
__global__ void dec_rle1_kernel(const uint8_t* rle1, size_t rstride, const DecBlockInfo* infos,
                                const uint32_t* blocks, uint32_t nblocks, uint32_t* chunk_state, uint64_t* out_len,
                                const uint64_t* out_off, uint8_t* out, uint64_t cap, uint32_t* crc_out,
                                const uint32_t* crc_table, int pass);
int dec_set_xpow8(const uint32_t* tab64);

}  // namespace bz2mi
