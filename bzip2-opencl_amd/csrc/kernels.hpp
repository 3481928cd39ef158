// Kernel entry points of libbz2mi (declarations shared by the .hip files and
// the host launcher in api.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bz2mi {

// Scratch bytes one BWT workgroup slot needs for blocks of S bytes.
inline size_t bwt_slot_bytes(int S) { return (size_t)48 * (size_t)S + 4096; }
// ... and one bwt_level_kernel workgroup slot (two segment lists; the spill
// area is the block's per-rotation spill, d_lspill)
inline size_t bwt_level_slot_bytes(int S) { return 16 * ((size_t)S / 512 + 8) + 256; }

// BWT (bwt.hip): per-block counting sort by the first byte; levels of
// partitions by the next byte for the large buckets of all blocks at once
// (one launch per level); one wave per small bucket across all blocks; prefix
// doubling for the blocks with tie groups left.
struct BwtSeg {
    uint32_t start, len;
};
struct BwtItem {
    uint32_t block, start, len, depth;
};
constexpr int kBwtLevels = 4;  // global partition levels (the last one finishes its segments' subtrees)
__global__ void bwt_bucket_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, int nblocks,
                                  uint32_t* sa_all, uint8_t* bwt_out, uint32_t* orig_out, uint64_t* squeue,
                                  uint32_t* scount, size_t scap, BwtItem* lq, uint32_t* lcount, size_t lcap,
                                  uint32_t* present_out, uint64_t* bq, uint32_t* bq_count, size_t bq_cap);
// buckets of 512 < c <= 4096 rotations listed by bwt_bucket_kernel in bq (per
// block, bq_cap entries, count bq_count[b]): bigbucket_grid(blocks) of
// kBigBucketThreads
#ifndef BZ2MI_BIG_NT
#define BZ2MI_BIG_NT 512
#endif
#ifndef BZ2MI_BIG_XCD
#define BZ2MI_BIG_XCD 1
#endif
constexpr int kBigBucketThreads = BZ2MI_BIG_NT;
// workgroups per 900 KB block of a tie round (A/B: -DBZ2MI_TIE_SLICES=n)
#ifndef BZ2MI_TIE_SLICES
#define BZ2MI_TIE_SLICES 8
#endif
constexpr int kTieSlices = BZ2MI_TIE_SLICES;
inline dim3 bigbucket_grid(int nblocks) {
#if BZ2MI_BIG_XCD
    return dim3(8u * 256u * (((unsigned)nblocks + 7u) / 8u));
#else
    return dim3(256, nblocks);
#endif
}
__global__ void bwt_bigbucket_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, uint32_t* sa_all,
                                     uint8_t* bwt_out, uint32_t* orig_out, const uint64_t* bq,
                                     const uint32_t* bq_count, size_t bq_cap, uint64_t* tl, uint32_t* tcount,
                                     size_t tcap, BwtItem* lq, uint32_t* lcount, size_t lcap, int nblocks);
// Blocks of <= kBwtLdsText bytes: the first-byte sort and the sort of the
// small buckets in one launch, the block's text held in LDS (1024 threads, one
// workgroup per CU).  Large buckets still go to the level queue.
constexpr int kBwtLdsText = 90112;
// mode 0: every block, except that text-like ones (most rotations in large
// first-byte buckets) only get their symbol map and redo[b] = 1 (redo zeroed
// before): they go to bwt_text_kernel; mode 1: the blocks bwt_text_kernel
// handed back (redo[b] = 2)
__global__ void bwt_block_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, int nblocks,
                                 uint32_t* sa_all, uint8_t* bwt_out, uint32_t* orig_out, BwtItem* lq,
                                 uint32_t* lcount, size_t lcap, uint32_t* present_out, uint64_t* tl,
                                 uint32_t* tcount, size_t tcap, uint32_t* redo, int mode, uint64_t* squeue,
                                 uint32_t* scount, size_t scap);
// text-like blocks (redo[b] == 1): induced sorting with the text in LDS, deep
// ties ordered by prefix doubling; SA and BWT bytes complete, or redo[b] = 2.
// Scratch: `spill_all` (stride words per block), `grp_all` (the pair list),
// `key_all` / `glist_all` (tcap uint64 per block: the doubling keys and group
// lists; the tie queues of bwt_block_kernel, unused by text blocks).
__global__ void bwt_text_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, int nblocks,
                                uint32_t* sa_all, uint8_t* bwt_out, uint32_t* orig_out, uint32_t* redo,
                                uint32_t* spill_all, BwtSeg* grp_all, uint64_t* key_all, uint64_t* glist_all,
                                size_t tcap, uint32_t wq_cap);
__global__ void redo_all_kernel(uint32_t* redo, int nblocks);
__global__ void bwt_level_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, uint32_t* sa_all,
                                 uint8_t* bwt_out, uint32_t* orig_out, uint8_t* scratch, uint32_t* spill_all,
                                 size_t scratch_per_slot, int S, const BwtItem* lin, const uint32_t* lin_count, BwtItem* lout,
                                 uint32_t* lout_count, size_t lcap, uint64_t* squeue, uint32_t* scount, size_t scap,
                                 BwtSeg* grp_all, uint32_t* ngroups, uint32_t* p2list, uint32_t* p2count, int last,
                                 uint32_t smask);
__global__ void bwt_wlevel_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, uint32_t* sa_all,
                                  uint8_t* bwt_out, uint32_t* orig_out, uint32_t* spill_all, const BwtItem* lin,
                                  const uint32_t* lin_count, BwtItem* lout, uint32_t* lout_count, size_t lcap,
                                  uint64_t* squeue, uint32_t* scount, size_t scap, BwtSeg* grp_all, uint32_t* ngroups,
                                  uint32_t* p2list, uint32_t* p2count, uint32_t smask);
// with bwt_block_kernel: the levels' small batches in per-block lists (squeue
// + b * scap, count scount[b]), one workgroup per block, text in LDS
__global__ void bwt_block_small_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, int nblocks,
                                       uint32_t* sa_all, uint8_t* bwt_out, uint32_t* orig_out, const uint64_t* squeue,
                                       const uint32_t* scount, size_t scap, uint64_t* tl, uint32_t* tcount,
                                       size_t tcap);
__global__ void bwt_small_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, uint32_t* sa_all,
                                 uint8_t* bwt_out, uint32_t* orig_out, const uint64_t* squeue,
                                 const uint32_t* scount, size_t scap, uint64_t* tl, uint32_t* tcount, size_t tcap);
constexpr int kBwtTieRounds = 6;  // rounds of 8 more bytes for tie groups before prefix doubling
#ifndef BZ2MI_AB_TIE_ROUNDS_GRID
#define BZ2MI_AB_TIE_ROUNDS_GRID 3
#endif
constexpr int kBwtTieRoundsGrid = BZ2MI_AB_TIE_ROUNDS_GRID;  // ... before the grid-wide doubling
__global__ void bwt_tie_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, uint32_t* sa_all,
                               uint8_t* bwt_out, uint32_t* orig_out, const uint64_t* tin, const uint32_t* tin_count,
                               uint64_t* tout, uint32_t* tout_count, size_t tcap, BwtSeg* grp_all,
                               uint32_t* ngroups, uint32_t* p2list, uint32_t* p2count, int last, int nblocks, int xcd_map);
constexpr int kBwtShards = 64;  // queue shards (bwt.hip kShards)
__global__ void bwt_double_kernel(const uint8_t* blocks, size_t stride, const uint32_t* lens, int nblocks,
                                  uint32_t* sa_all, uint8_t* bwt_out, uint32_t* orig_out, uint8_t* scratch,
                                  size_t scratch_per_slot, int S, BwtSeg* grp_all, const uint32_t* ngroups,
                                  const uint32_t* p2list, const uint32_t* p2count, uint32_t* pull);
// Blocks beyond kBwtLdsText: prefix doubling over the whole grid, one launch
// per step and round (dbl_* kernels, bwt.hip), every group of every block of
// the batch in one flat list.  Per enlisted block (slot k = its p2list index)
// a scratch slot of dbl_slot_bytes(S); lists of dbl_list_cap(S) entries per slot.
struct DblGrid {
    const uint8_t* blocks;
    size_t stride;
    const uint32_t* lens;
    uint32_t* sa_all;
    uint8_t* bwt_out;
    uint32_t* orig_out;
    const BwtSeg* grp_all;
    const uint32_t* ngroups;
    const uint32_t* p2list;
    const uint32_t* p2count;
    uint8_t* scratch;
    size_t per_slot;
    int S;
    uint64_t* list[2];   // groups of <= 512 rotations (sq_pack entries, block field = slot)
    uint64_t* large[2];  // larger groups: slot << 40 | start << 20 | len
    uint32_t* ctr;       // kDblCtr counters per round (zeroed before the first launch)
};
constexpr int kDblCtr = 8;
constexpr int kDblMaxRounds = 20;  // 9 << 19 > 2^20 >= S
inline size_t dbl_slot_bytes(int S) {
    const size_t s = (size_t)S;
    return (36 * s + 4 * (s / 1024 + 8) + 255) & ~(size_t)255;
}
inline size_t dbl_list_cap(int S) { return (size_t)S / 2 + 2; }
inline size_t dbl_large_cap(int S) { return (size_t)S / 513 + 2; }
// rounds of the doubling for blocks of <= S bytes (h = 9 << r while h < S)
inline int dbl_rounds(int S) {
    int r = 0;
    while (r < kDblMaxRounds && (9ll << r) < (long long)S) ++r;
    return r;
}
__global__ void dbl_init_rank_kernel(DblGrid G);
__global__ void dbl_init_groups_kernel(DblGrid G);
__global__ void dbl_pairset_kernel(DblGrid G, int r);
__global__ void dbl_runend_kernel(DblGrid G, int r);
__global__ void dbl_decide_kernel(DblGrid G, int r);
__global__ void dbl_snap_kernel(DblGrid G, int r);
__global__ void dbl_sort_kernel(DblGrid G, int r);
__global__ void dbl_large_kernel(DblGrid G, int r);
__global__ void dbl_emit_kernel(DblGrid G);

// small-queue capacity (entries) per block and level-queue capacity per block
// (a shard holds the entries of every 64th block)
__host__ __device__ inline size_t bwt_squeue_per_block(int S) { return (size_t)S / 2 + 2; }
__host__ __device__ inline size_t bwt_lqueue_per_block(int S) { return (size_t)S / 512 + 2; }
// per-block group list capacity (BwtSeg entries) for a block stride
__host__ __device__ inline size_t bwt_group_stride(size_t stride) { return stride / 2 + 2; }

// MTF + RLE2, one workgroup of 1..8 waves per block (segments when the batch
// has few blocks; `scratch`: scratch_stride u16 per block, the segments'
// output before concatenation); `present` (8 words per block) comes from the BWT
void launch_mtf(int nb, const uint8_t* bwt, size_t stride, const uint32_t* lens, const uint32_t* present,
                uint16_t* mtf_out, size_t mtf_stride, uint32_t* mtf_len, uint32_t* alpha_out, uint32_t* hist_out,
                uint16_t* scratch, size_t scratch_stride, hipStream_t s);

constexpr int kSeedWaves = 16;  // waves per seed_kernel workgroup (pieces of a slot's chain)
__global__ void seed_kernel(const uint32_t* hist, uint32_t* seed, uint32_t* state, int nblocks, int p,
                            uint64_t first_block);

// phase stamps (make PHASES=1)
int huffman_phases(unsigned long long* out);
int bwt_phases(unsigned long long* out);
int mtf_phases(unsigned long long* out);
int fe_phases(unsigned long long* out);
int tbk_stats(unsigned long long* out);
int tbk_extra_stats(unsigned long long* out);
int blk_phase_stats(unsigned long long* out);
int tbk_resolve_stats(unsigned long long* out);
int dbl_stats(unsigned long long* out);
int tbk_trace(void* host_mapped);
int run_selftest(uint32_t* host_bad, int n);  // cross-lane primitive checks
int huffman_threads();  // workgroup size of huffman_kernel
__global__ void huffman_kernel(const uint16_t* mtf, size_t mtf_stride, const uint32_t* mtf_len,
                               const uint32_t* alpha_in, const uint32_t* seed, const uint32_t* present,
                               const uint32_t* orig, int nblocks, uint32_t* payload, size_t payload_words,
                               uint64_t* payload_bits);

__global__ void offsets_kernel(const uint64_t* bits, int nblocks, uint64_t prefix_bits, uint64_t* offs);

// Stream assembly state kept on the device (pipelined compress_device).
struct StreamDev {
    uint64_t word_base;   // output words already final
    uint64_t final_bits;  // stream length, set by the final batch
    uint32_t carry;       // MSB-aligned bits of the partial word at word_base
    uint32_t carry_bits;  // (the stream header "BZh<level>" is 32 carried bits)
    uint32_t crc;         // combined stream CRC so far
    uint32_t pad;
};
__global__ void offsets_dev_kernel(const uint64_t* bits, const uint32_t* crcs, int nblocks, StreamDev* st,
                                   uint64_t* offs);
__global__ void assemble_dev_kernel(const uint32_t* payload, size_t payload_words, const uint64_t* offs,
                                    const uint32_t* crc, int nblocks, int final_, const StreamDev* st,
                                    uint32_t* out, uint64_t cap_words);
__global__ void volume_kernel(const uint32_t* lens, const uint32_t* mtflen, const uint64_t* pbits, int nblocks,
                              unsigned long long* acc);
__global__ void advance_kernel(const uint64_t* offs, int nblocks, int final_, StreamDev* st, const uint32_t* out,
                               uint64_t cap_words);

__global__ void assemble_kernel(const uint32_t* payload, size_t payload_words, const uint64_t* offs,
                                const uint32_t* crc, int nblocks, uint64_t prefix, int prefix_bits, int final_,
                                uint32_t stream_crc, uint32_t* out);

// Device RLE1 front end (frontend.hip); chunks are 4096 bytes.
constexpr int kFeChunk = 4096;
// summ[c] = (first | last byte << 8, lead, trail, len); cfree[c] = the chunk's
// context-free cost (fe_costscan_kernel adds the incoming run's part)
__global__ void fe_summary_kernel(const uint8_t* x, uint64_t n, uint64_t nc, uint4* summ, uint32_t* cfree);
constexpr int kFeScanThreads = 1024;  // threads per scan workgroup
constexpr int kFeScanTile = kFeScanThreads * 8;  // chunks per scan workgroup
__global__ void fe_runscan_kernel(const uint4* summ, uint64_t nc, uint64_t* rsb, uint64_t* agg, int pass);
__global__ void fe_costscan_kernel(const uint32_t* cfree, const uint4* summ, const uint64_t* rsb, uint64_t nc,
                                   uint64_t* fc, uint64_t* agg, int pass);
// also laneinfo[c*64 + l] = the cost prefix of lane l's 64 bytes in chunk c |
// their run's piece phase before them << 16 (the chain's in-chunk lookups)
__global__ void fe_dmap_kernel(const uint8_t* x, const uint4* summ, const uint64_t* rsb, uint64_t n, uint64_t nc,
                               const uint64_t* fc, uint8_t* dmap, uint32_t* laneinfo);
constexpr int kFeChainThreads = 1024;  // one workgroup
// chain of one unit of the stream (own bytes [0, n_own), tail halo up to n),
// first block at `entry` (bit 63: mid-run); out[0] blocks, out[1] status
__global__ void fe_chain_kernel(const uint8_t* x, const uint32_t* laneinfo, const uint64_t* fc, const uint4* summ,
                                const uint8_t* dmap, uint64_t n, uint64_t nc, int S, uint64_t n_own, uint64_t entry,
                                int ends, uint64_t* bnd, uint64_t max_bnd, uint64_t* out, const uint64_t* spec,
                                uint64_t spec_nb);
// starts[0..nb] from the chain; nb_io[2] = exit token of the next unit
__global__ void fe_resolve_kernel(const uint8_t* x, const uint32_t* laneinfo, const uint64_t* fc, const uint4* summ,
                                  uint64_t n, uint64_t nc, uint64_t n_own, uint64_t entry, const uint64_t* bnd,
                                  uint64_t* nb_io, uint64_t* starts);
// RLE1 emission + block CRCs (crc_tabs: rle1.hpp crc_device_tables); blocks
// of >= 2 kFeSegLen raw bytes are cut into segments of ~kFeSegLen emitted by
// workgroups of their own (fe_segplan_kernel, two fe_rle1_kernel passes,
// fe_crccomb_kernel)
constexpr uint64_t kFeSegLen = 128 << 10;
struct FeSeg;
__global__ void fe_segplan_kernel(const uint8_t* x, uint64_t n, const uint64_t* starts, uint64_t first,
                                  uint64_t count, const uint64_t* rsb, const uint4* summ, FeSeg* segs,
                                  uint32_t* segfirst, uint64_t seg_cap, uint32_t* nseg);
__global__ void fe_rle1_kernel(const uint8_t* x, uint64_t n, const FeSeg* segs, const uint32_t* segfirst,
                               const uint32_t* nseg, uint32_t* segcnt, uint32_t* segcrc, int mode, uint8_t* blocks,
                               size_t stride, uint32_t* lens, uint32_t* crcs, const uint32_t* crc_tabs);
__global__ void fe_crccomb_kernel(const FeSeg* segs, const uint32_t* segfirst, uint64_t count, const uint32_t* segcrc,
                                  uint32_t* crcs, const uint32_t* crc_tabs);
// device bytes of one segment-table entry (FeSeg)
constexpr size_t kFeSegBytes = 24;

}  // namespace bz2mi
