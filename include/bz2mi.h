/*
 * bz2mi -- MI355X-native bzip2 block compression, C ABI.
 *
 * This is the drop-in boundary that replaces the reference's OpenCL device
 * layer (Stan1slav337/Bzip2-OpenCL include/opencl.hpp Device / Memory<T> /
 * Kernel, include/kernel.hpp, and the device program kernel.cpp:27-3162).
 * Plain pointers and sizes only; no exceptions cross it.  Every call returns
 * BZ2MI_OK (0) or a negative status; bz2mi_last_error() describes the last
 * failure of the calling thread.  A context is thread-compatible, not
 * thread-safe: one context per OutputStream, as in the reference.
 *
 * Output is bit-identical to the reference's CPU-serial semantics (O_ref,
 * SURVEY.md section 8c), including the per-slot Huffman seed carry-over that
 * makes the stream depend on the parallel block count `p`.
 */
#ifndef BZ2MI_H
#define BZ2MI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BZ2MI_OK 0
#define BZ2MI_EINVAL -1    /* bad argument (reference: std::invalid_argument) */
#define BZ2MI_EDEVICE -2   /* HIP runtime failure (reference: print_error + exit(1)) */
#define BZ2MI_ESPACE -3    /* output buffer too small */
#define BZ2MI_ESTATE -4    /* call out of order (e.g. write after finish) */
#define BZ2MI_EFORMAT -5   /* corrupt or unsupported .bz2 data (reference: std::runtime_error
                              from InputStream / BlockDecompressor; the message is the reference's) */

typedef struct bz2mi_ctx bz2mi_ctx;

/* Last error message of the calling thread ("" if none). */
const char* bz2mi_last_error(void);

/* Library / device information. */
int bz2mi_device_count(void);
const char* bz2mi_version(void);
/* ABI revision of this header's entry points: a host checks it at load time.
 *   3: bz2mi_unit_assemble / _host gained the trailing hip_stream argument;
 *      bz2mi_decompress* decode the first stream only (the reference)
 *   4: bz2mi_dlast_trailing, bz2mi_abi_version */
#define BZ2MI_ABI_VERSION 5
int bz2mi_abi_version(void);

/*
 * Create a compression context on HIP device `device`.
 *   level           1..9; block size S = unit * level        (OutputStream.hpp:65-77,
 *                   reference unit = BLOCKSIZE_DEFAULT = 10000, Config.hpp:30)
 *   parallel_blocks the reference's `p` (>= 1): block b uses Huffman seed slot
 *                   b mod p (OutputStream.hpp:79-81, 93)
 *   unit            10000 (reference parity) or 100000 (bzip2-standard 900 KB)
 * Replaces: OutputStream ctor's Device/Memory/Kernel setup (OutputStream.hpp:83-123,
 *           opencl.hpp:163-215 Device, :217-459 Memory, :461-539 Kernel).
 * Returns NULL on failure (see bz2mi_last_error).
 */
bz2mi_ctx* bz2mi_create(int level, int parallel_blocks, int unit, int device);
void bz2mi_destroy(bz2mi_ctx* ctx);

/* Upper bound of the compressed size of n input bytes. */
size_t bz2mi_compress_bound(size_t n, int level, int unit);

/*
 * Compress one batch of RLE1 blocks and append the resulting stream bits.
 * This is OutputStream::closeBlocks (OutputStream.hpp:190-240) around
 * kernel_close (kernel.cpp:3124-3159): block headers (0x314159265359, CRC,
 * randomised bit), the device compressor (BWT, MTF/RLE2, Huffman, packing),
 * and the bit-level stitching with the carried leftover bits.
 *   blocks  host memory; block j at blocks + j*stride, lens[j] bytes (1..S)
 *   crcs    block CRCs (BlockCompressor::getCRC, CRC32.hpp:70-73)
 * The first call also emits the stream header 'BZh'+level (OutputStream.hpp:126-128).
 * Complete bytes go to out (*out_len set); < 8 pending bits stay in ctx.
 */
int bz2mi_compress_rle1(bz2mi_ctx* ctx, const uint8_t* blocks, size_t stride, const uint32_t* lens,
                        const uint32_t* crcs, uint32_t nblocks, uint8_t* out, size_t cap,
                        size_t* out_len);

/*
 * Finish the stream: end-of-stream marker, stream CRC, zero padding
 * (OutputStream::close, OutputStream.hpp:163-176).  Writes the remaining
 * bytes to out.  Further compress calls return BZ2MI_ESTATE.
 */
int bz2mi_finish(bz2mi_ctx* ctx, uint8_t* out, size_t cap, size_t* out_len);

/*
 * Block-level entry, the direct analogue of one kernel_close launch
 * (kernel.cpp:3124-3159) over `nblocks` RLE1 blocks whose stream-global
 * indices are first_block_index .. +nblocks-1: writes each block's payload
 * (origPtr .. last data bit, kernel.cpp:3116-3121) packed MSB-first to
 * out + j*out_stride and its bit count to out_bits[j].  Advances the seed
 * carry-over state like a batch of the stream.
 */
int bz2mi_compress_blocks(bz2mi_ctx* ctx, const uint8_t* blocks, size_t stride, const uint32_t* lens,
                          uint32_t nblocks, uint8_t* out, size_t out_stride, uint64_t* out_bits);

/*
 * Whole-stream compression of host bytes (RLE1 front end + device path +
 * framing): the same bytes the reference's app.cpp writes for this input at
 * this level and p.  out must hold bz2mi_compress_bound() bytes.
 */
int bz2mi_compress(bz2mi_ctx* ctx, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                   size_t* out_len);

/*
 * Device-resident whole-stream compression: d_in / d_out are device pointers
 * (HBM), `hip_stream` a hipStream_t (NULL = the context's stream).  The RLE1
 * front end, block split and CRCs run on the device too.  *out_len receives
 * the stream size.  Used by bench.py with inputs resident in HBM.
 */
int bz2mi_compress_device(bz2mi_ctx* ctx, const void* d_in, size_t n, void* d_out, size_t cap,
                          size_t* out_len, void* hip_stream);

/* Timing of the last device batch, per stage, in milliseconds (HIP events
 * on the context stream): front, bwt, mtf, seed, huffman, assemble. */
int bz2mi_last_timings(bz2mi_ctx* ctx, float* ms6);

/* Volumes of the last bz2mi_compress_device call (collected once this has
 * been called): [0] input bytes, [1] blocks, [2] RLE1 bytes, [3] MTF/RLE2
 * symbols, [4] payload bits, [5] output bytes, [6] blocks in the last batch. */
int bz2mi_last_stats(bz2mi_ctx* ctx, uint64_t* out8);

/* Number of blocks compressed so far in this stream. */
uint64_t bz2mi_blocks_done(const bz2mi_ctx* ctx);

/* ---- one logical stream compressed in units ------
 * The reference compresses one stream on one device: OutputStream feeds the
 * blocks in order (OutputStream.hpp:131-142, 179-188), the per-slot frequency
 * array persists across batches (OutputStream.hpp:93, kernel.cpp:3155) and the
 * block bits are stitched and the stream CRC chained in block order
 * (OutputStream.hpp:190-240, :202).  Here the stream is cut into units --
 * contiguous byte ranges, each compressed by a context on any device or process
 * -- and the output is the same stream, bit for bit.  Per unit, in order:
 *
 *   begin     the unit's bytes [0, n_own) plus a tail halo [n_own, n_own+n_halo)
 *             (the bytes that follow it in the stream, bz2mi_unit_halo() of
 *             them, or up to the stream end: BZ2MI_UNIT_ENDS_STREAM) are in HBM;
 *             the data-parallel front end starts (asynchronous).
 *   chain     the unit's blocks (the RLE1 block split, OutputStream.hpp:179-188):
 *             `entry` = where its first block starts, from the previous unit's
 *             exit (the first unit: 0); returns the next unit's entry and the
 *             block count.  Block indices continue from `first_block` (the sum
 *             of the earlier units' counts).  Synchronous; then RLE1, CRC, BWT,
 *             MTF/RLE2 run asynchronously.
 *   sums      the unit's per-slot symbol histogram sums (p x 258 uint32, slot =
 *             stream block index mod p): its share of the persistent frequency
 *             array.
 *   encode    `carried` = the uint32 sum of the sums of every earlier unit:
 *             Huffman tables and block payloads; returns the unit's bits (81
 *             header bits + payload per block) and its CRC share
 *             XOR_b rotl(crc_b, m-1-b) over its m blocks.
 *   assemble  the unit's bytes for a stream bit offset: the first byte's top
 *             (bit_offset & 7) bits are zero (OR it into the previous unit's
 *             last byte); BZ2MI_UNIT_FIRST prepends "BZh<level>" (bit_offset
 *             0), BZ2MI_UNIT_LAST appends the end-of-stream marker with the
 *             stream CRC rotl(crc_before, m) ^ share and pads to a byte.
 * A unit whose entry lies at or past n_own has no blocks: chain returns
 * nblocks = 0 and exit = entry - n_own, and it takes no further part.
 * bz2mi_shard (bzip2-opencl_amd/bz2mi/shard.py) drives this protocol across
 * ranks with torch.distributed; a context runs its units' BWTs one at a time.
 */
typedef struct bz2mi_unit bz2mi_unit;
#define BZ2MI_UNIT_ENDS_STREAM 1 /* begin: the halo reaches the end of the stream */
#define BZ2MI_UNIT_FIRST 1       /* assemble: stream header first */
#define BZ2MI_UNIT_LAST 2        /* assemble: end-of-stream trailer last */
/* assemble in place: d_out is the whole stream's buffer and the unit's bits go
 * to stream bit bit_offset of it; the bits before it in its first 32-bit word
 * (the previous unit's, assembled before this call's work runs: same context,
 * or ordered through hip_stream) are kept.  *out_bytes = the stream's bytes up
 * to the unit's end.  No copy of the unit's bytes afterwards. */
#define BZ2MI_UNIT_IN_PLACE 4
#define BZ2MI_ENTRY_MIDRUN (1ull << 63) /* entry/exit flag: x[p] == x[p-1] in the stream */

/* tail halo bytes a unit needs (the longest raw span of one block) */
size_t bz2mi_unit_halo(int level, int unit);
bz2mi_unit* bz2mi_unit_create(bz2mi_ctx* ctx);
void bz2mi_unit_destroy(bz2mi_unit* u);
/* d_buf: device bytes (n_own + n_halo), read until the unit is assembled;
 * hip_stream: the stream that wrote them (NULL: the null stream) */
int bz2mi_unit_begin(bz2mi_unit* u, const void* d_buf, size_t n_own, size_t n_halo, int flags, void* hip_stream);
int bz2mi_unit_chain(bz2mi_unit* u, uint64_t entry, uint64_t first_block, uint64_t* exit_entry, uint64_t* nblocks);
/* Speculation (optional, between begin and chain; synchronous): chain the unit
 * from its own first byte while the real entry is still on its way.  A block's
 * end depends only on the bytes from its start on (RLE1 restarts at every
 * block start, OutputStream.hpp:179-188), so bz2mi_unit_chain then chains from
 * the entry only until one of its blocks starts where a speculative block
 * starts and takes the remaining blocks from the speculation (all of them when
 * entry == 0).  The result is the same as without it.  *nblocks (may be NULL) =
 * the speculative chain's blocks (0: it runs past the tail halo, not used). */
int bz2mi_unit_speculate(bz2mi_unit* u, uint64_t* nblocks);
/* after chain: [0] speculative blocks, [1] blocks taken from the speculation,
 * [2] blocks chained from the entry, [3] 1 if speculated */
int bz2mi_unit_chain_info(bz2mi_unit* u, uint64_t* out4);
int bz2mi_unit_sums(bz2mi_unit* u, uint32_t* sums);
int bz2mi_unit_encode(bz2mi_unit* u, const uint32_t* carried, uint64_t* bits, uint32_t* crc);
/* d_out: device memory, 4-byte aligned, >= (bits + 7 + 32 + 80) / 8 + 4 bytes;
 * hip_stream: the stream whose queued work may still use d_out (NULL: the null
 * stream) -- assembly writes d_out only after it; returns when the bytes are in d_out */
int bz2mi_unit_assemble(bz2mi_unit* u, uint64_t bit_offset, uint32_t crc_before, int flags, void* d_out, size_t cap,
                        size_t* out_bytes, void* hip_stream);
/* Host-memory forms for C++ hosts without a device allocator (the mirror
 * OutputStream): begin_host copies the bytes into a unit-owned device buffer
 * (asynchronous when `host` is pinned; it must stay unchanged until
 * bz2mi_unit_chain returns); assemble_host copies the unit's bytes back. */
void* bz2mi_host_alloc(size_t bytes); /* pinned host memory, NULL on failure */
void bz2mi_host_free(void* p);
int bz2mi_unit_begin_host(bz2mi_unit* u, const void* host, size_t n_own, size_t n_halo, int flags);
int bz2mi_unit_assemble_host(bz2mi_unit* u, uint64_t bit_offset, uint32_t crc_before, int flags, void* host_out,
                             size_t cap, size_t* out_bytes, void* hip_stream);
/* milliseconds of the unit's stages (HIP events): front scan, chain (host wall),
 * RLE1 + CRC + BWT, MTF, Huffman, assembly */
int bz2mi_unit_timings(bz2mi_unit* u, float* ms6);
/* volumes of the unit once encoded: [0] RLE1 bytes, [1] MTF/RLE2 symbols,
 * [2] payload bits, [3] blocks */
int bz2mi_unit_stats(bz2mi_unit* u, uint64_t* out4);

/* ---- decompression on the device ----------
 * Replaces the reference's InputStream (InputStream.hpp:36-159),
 * BlockDecompressor (BlockDecompressor.hpp:37-282) and HuffmanStageDecoder
 * (HuffmanStageDecoder.hpp:30-136): the blocks of the stream are decoded
 * together, as many at once as a memory budget allows (max(64 x the input,
 * 1 GiB) of per-block device buffers, BZ2MI_DEC_BUDGET overrides: a
 * legitimate stream is one window, an input of crafted magic matches is
 * decoded a bounded number of candidates at a time).  Errors are BZ2MI_EFORMAT with the reference's message ("Invalid BZip2
 * header", "BZip2 block CRC error", "BZip2 stream CRC error", "BZip2 stream
 * format error", "block Huffman tables invalid", "Error decoding  block",
 * "BZip2 block exceeds declared block size", "BZip2 start pointer invalid",
 * "BZip2 randomised blocks not implemented"), reported for the first failing
 * block in stream order as the reference's byte-at-a-time decoder would.
 *   unit   block-size unit of the digit in "BZh<digit>": 10000 = the
 *          reference's limit (Config.hpp:30), 100000 = stock bzip2 files.
 * By default only the first stream is decoded and the bytes after its end
 * marker are ignored (the reference's InputStream, InputStream.hpp:136-143);
 * with BZ2MI_DEC_CONCATENATED (bz2mi_dset_flags) concatenated streams are
 * decoded one after another (bzip2's behaviour), and bytes after the last
 * stream that do not start a new "BZh" header are ignored.
 */
typedef struct bz2mi_dctx bz2mi_dctx;
#define BZ2MI_DEC_CONCATENATED 1
bz2mi_dctx* bz2mi_dcreate(int unit, int device);
void bz2mi_ddestroy(bz2mi_dctx* d);
int bz2mi_dset_flags(bz2mi_dctx* d, int flags);

/* host buffers; on BZ2MI_ESPACE *out_len receives the size needed */
int bz2mi_decompress(bz2mi_dctx* d, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);

/* device buffers (HBM); hip_stream: hipStream_t or NULL (the context's) */
int bz2mi_decompress_device(bz2mi_dctx* d, const void* d_in, size_t n, void* d_out, size_t cap, size_t* out_len,
                            void* hip_stream);

/* Streaming decode with bounded memory (the reference's block-at-a-time
 * InputStream, InputStream.hpp:51-72,125-158).  in[0, n) is a window of the
 * compressed input and decoding resumes at window bit `start_bit`; every block
 * that lies whole inside the window is decoded, at most `cap` output bytes and
 * a bounded number of blocks per call (device memory of the decoded
 * candidates <= BZ2MI_DSTREAM_BUDGET bytes, default 1 GiB).  *end_bit: the
 * window bit where the next call resumes (the caller keeps the bytes from
 * *end_bit / 8 on and appends more input); *done = 1 once the stream (or, with
 * BZ2MI_DEC_CONCATENATED, the streams) ended.  *out_len = 0 with *done = 0:
 * the window holds no whole block yet -- hand over a longer one (final = 0)
 * or, with final = 1 (no more input), the call reports "Insufficient data".
 * An error is returned by the call after the one that returned the bytes of
 * the blocks before the failing one, as the reference throws when it reaches
 * that block.  BZ2MI_ESPACE: *out_len = the bytes the next block needs.
 * bz2mi_dstream_reset starts a new input. */
int bz2mi_dstream_reset(bz2mi_dctx* d);
int bz2mi_dstream(bz2mi_dctx* d, const uint8_t* in, size_t n, unsigned start_bit, int final, uint8_t* out,
                  size_t cap, uint64_t* end_bit, size_t* out_len, int* done);

/* bytes of the last bz2mi_decompress* input after the end of the last
 * stream it decoded (ignored, as by the reference's InputStream, which reads
 * the first stream; with BZ2MI_DEC_CONCATENATED: bytes that start no stream) */
int bz2mi_dlast_trailing(bz2mi_dctx* d, uint64_t* bytes);

/* milliseconds of the last call: [0] candidate scan, [1] Huffman symbols,
 * [2] MTF + RLE2 (and the stream walk), [3] inverse BWT, [4] RLE1 + CRC, [5] whole call */
int bz2mi_dlast_timings(bz2mi_dctx* d, float* ms6);

#ifdef __cplusplus
}
#endif
#endif
