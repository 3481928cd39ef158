/* TEST INFRASTRUCTURE ONLY (oracle/).
 *
 * cpu_ref: a plain-C restatement of the reference compressor's hot path
 * (Stan1slav337/Bzip2-OpenCL), stage by stage, used as the parity checker for
 * the HIP path and as the CPU baseline.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product library never
 * links it and never falls back to it.
 *
 * Parity is pinned against O_ref (oracle/_ref/liboref.so: the reference's own
 * kernel.cpp / BlockCompressor.hpp / BitOutputStream.hpp compiled from
 * /root/reference) and against the committed fixtures in tests/golden/.
 */
#ifndef CPU_REF_H
#define CPU_REF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- stage a1/a2: RLE1 + block split + CRC (BlockCompressor.hpp:69-154,
 *      CRC32.hpp:75-86).  Splits `in` into blocks of at most S RLE1 bytes.
 *      For block b: starts[b] = first input byte, lens[b] = RLE1 length,
 *      crcs[b] = block CRC; the RLE1 bytes go to blocks + b*stride.
 *      Returns the number of blocks (or -needed when max_blocks is too small). */
long long cpuref_split(const uint8_t* in, size_t n, int S, uint8_t* blocks, size_t stride,
                       uint64_t* starts, uint32_t* lens, uint32_t* crcs, size_t max_blocks);

/* CRC-32 (MSB-first, poly 0x04c11db7) of `n` bytes starting from `crc`
 * (initial value 0xffffffff; the block CRC is the complement). */
uint32_t cpuref_crc_update(uint32_t crc, const uint8_t* p, size_t n);

/* ---- stage a6: cyclic BWT of one RLE1 block, origPtr returned.  For a
 *      periodic block rotation 0 takes the smallest rank among the rotations
 *      equal to it (SURVEY H2/H8 decision). */
int cpuref_bwt(const uint8_t* T, int n, uint8_t* bwt);

/* ---- stage a8: MTF + RLE2 (kernel.cpp:2561-2649).  `present` = 256 flags of
 *      the RLE1 block.  Writes mtfLength symbols, returns mtfLength; *alpha =
 *      alphabet size; hist (258 bins) receives this block's histogram
 *      (overwritten, not accumulated). */
int cpuref_mtf(const uint8_t* bwt, int n, const uint8_t* present, uint16_t* mtf,
               uint32_t* hist, int* alpha);

/* ---- stages a7 + a9-a11: one block's payload bits, MSB-first, packed.
 *      origPtr(24) + symbol map + Huffman tables + data.  `seed` = the
 *      accumulated 258-bin frequency array the reference reads (H4).  Returns
 *      the number of bits written, or -1 if cap_bits is too small.
 *      If non-NULL, selectors (ceil(len/50)) and lengths ([6][258]) are
 *      exported for intermediate checks. */
long long cpuref_block_payload(int origPtr, const uint8_t* present, const uint16_t* mtf,
                               int mtfLength, int alpha, const uint32_t* seed, uint8_t* out,
                               uint64_t cap_bits, uint8_t* selectors, uint8_t* lengths);

/* H3 model of the reference run on an MI355X (OpenCL): tableFrequencies not
 * cleared between the four optimisation passes of a block (default off = O_ref,
 * zero-initialised per pass).  Process-wide; set before compressing. */
void cpuref_set_h3_accumulate(int on);

/* ---- whole stream (OutputStream.hpp semantics): level 1..9, parallel count
 *      p >= 1, block unit (10000 = reference, 100000 = 900 KB mode).
 *      threads > 1 compresses blocks on a pthread pool.  Returns the output
 *      size, -1 on bad arguments, -2 if cap is too small. */
long long cpuref_compress(const uint8_t* in, size_t n, int level, int p, int unit, uint8_t* out,
                          size_t cap, int threads);

/* ---- stream units: the protocol of include/bz2mi.h's
 *      bz2mi_unit_* restated on the host (same arguments, same results), so
 *      the distributed driver (bz2mi/shard.py) can be checked on CPU ranks.
 *      open = begin + chain (and RLE1/BWT/MTF): buf holds n_own bytes plus an
 *      n_halo tail halo (ends: it reaches the stream end); entry / exit as in
 *      bz2mi_unit_chain.  Returns NULL on bad arguments or a halo too short. */
typedef struct cpuref_unit cpuref_unit;
cpuref_unit* cpuref_unit_open(const uint8_t* buf, size_t n_own, size_t n_halo, int ends, int level, int p,
                              int unit, uint64_t entry, uint64_t first_block, uint64_t* exit_entry,
                              uint64_t* nblocks, int threads);
void cpuref_unit_sums(const cpuref_unit* u, uint32_t* sums);
int cpuref_unit_encode(cpuref_unit* u, const uint32_t* carried, uint64_t* bits, uint32_t* crc, int threads);
/* flags: 1 = stream header first, 2 = end-of-stream trailer last; returns the
 * byte count (the first byte's top bit_offset&7 bits are zero), -2 if cap is
 * too small */
long long cpuref_unit_assemble(const cpuref_unit* u, uint64_t bit_offset, uint32_t crc_before, int flags,
                               uint8_t* out, size_t cap);
void cpuref_unit_free(cpuref_unit* u);

/* Upper bound of the compressed size for cpuref_compress / the product. */
size_t cpuref_bound(size_t n, int level, int unit);

#ifdef __cplusplus
}
#endif
#endif
