// C-ABI launcher of libbz2mi (include/bz2mi.h): device memory, the per-batch
// kernel sequence and the stream state that OutputStream keeps in the
// reference (OutputStream.hpp:35-61).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bz2mi.h"
#include "common.hpp"
#include "host.hpp"
#include "kernels.hpp"
#include "rle1.hpp"

namespace {
thread_local std::string g_err;
}  // namespace

// shared with the decoder's host code (dapi.hip) and the shard launcher (shard.hip)
int bz2mi_set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

using namespace bz2mi::host;

namespace {

// BZ2MI_SYNC_DEBUG=1: synchronise and report after every launch (debug aid).
bool sync_debug() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("BZ2MI_SYNC_DEBUG");
        v = (e && *e && *e != '0') ? 1 : 0;
    }
    return v == 1;
}

#define STAGE_DONE(name)                                                              \
    do {                                                                              \
        if (sync_debug()) {                                                           \
            hipError_t e2_ = hipStreamSynchronize(s);                                 \
            fprintf(stderr, "[bz2mi] %s done: %s\n", name, hipGetErrorString(e2_));   \
        }                                                                             \
    } while (0)

}  // namespace

namespace bz2mi {
namespace host {

void free_batch(Batch& t) {
    for (void* p : t.ptrs())
        if (p) (void)hipFree(p);
    for (hipEvent_t e : {t.evA, t.evM, t.evFree})
        if (e) (void)hipEventDestroy(e);
    t = Batch{};
}

int ensure_batch(bz2mi_ctx* c, Batch& t, int nblocks) {
    if (nblocks <= t.cap) return BZ2MI_OK;
    const int cap = std::max(nblocks, 16);
    const size_t B = (size_t)cap;
    int r;
    if ((r = dalloc(&t.d_blocks, B * c->stride))) return r;
    if ((r = dalloc(&t.d_lens, B))) return r;
    if ((r = dalloc(&t.d_crc, B))) return r;
    if ((r = dalloc(&t.d_bwt, B * c->stride))) return r;
    if ((r = dalloc(&t.d_orig, B))) return r;
    if ((r = dalloc(&t.d_sa, B * c->stride))) return r;
    if ((r = dalloc(&t.d_bcnt, 1024))) return r;
    if ((r = dalloc(&t.d_ngroups, B))) return r;
    if ((r = dalloc(&t.d_p2list, B))) return r;
    if ((r = dalloc(&t.d_redo, B))) return r;
    if ((r = dalloc(&t.d_groups, B * bz2mi::bwt_group_stride(c->stride)))) return r;
    if ((r = dalloc(&t.d_mtf, B * c->mtf_stride))) return r;
    if ((r = dalloc(&t.d_mtflen, B))) return r;
    if ((r = dalloc(&t.d_alpha, B))) return r;
    if ((r = dalloc(&t.d_hist, B * bz2mi::kMaxAlpha))) return r;
    if ((r = dalloc(&t.d_present, B * 8))) return r;
    if ((r = dalloc(&t.d_seed, B * bz2mi::kMaxAlpha))) return r;
    if ((r = dalloc(&t.d_payload, B * c->payload_words))) return r;
    if ((r = dalloc(&t.d_pbits, B))) return r;
    if ((r = dalloc(&t.d_offs, B + 1))) return r;
    if (!t.evA) {
        HIPCHECK(hipEventCreateWithFlags(&t.evA, hipEventDisableTiming));
        HIPCHECK(hipEventCreateWithFlags(&t.evM, hipEventDisableTiming));
        HIPCHECK(hipEventCreateWithFlags(&t.evFree, hipEventDisableTiming));
    }
    t.cap = cap;
    return BZ2MI_OK;
}

// ---- the stages of one batch, each on its stream
// RLE1 emission + block CRCs of blocks [first, first+cnt) of the front end
int stage_front(bz2mi_ctx* c, Batch& t, const FrontBufs& f, const uint8_t* d_x, size_t n, uint64_t first,
                uint64_t cnt, hipStream_t s) {
    using namespace bz2mi;
    // the batch's segments, their emission counts (cut blocks only), the
    // emission, then the CRCs of the cut blocks; grid: every block plus one
    // workgroup per kFeSegLen bytes of the input (a bound on the extra segments)
    auto* seg = reinterpret_cast<const FeSeg*>(f.d_seg);
    hipLaunchKernelGGL(fe_segplan_kernel, dim3(1), dim3(1024), 0, s, d_x, (uint64_t)n, f.d_starts, first, cnt, f.d_rsb,
                       f.d_summ,                       reinterpret_cast<FeSeg*>(f.d_seg), f.d_segfirst, (uint64_t)f.seg_cap, f.d_nseg);
    // (the emission strides over the segments: one workgroup per block plus
    // at most 4 per CU for the extra segments of cut blocks)
    const unsigned grid = (unsigned)std::min<uint64_t>(
        f.seg_cap, cnt + std::min<uint64_t>(n / kFeSegLen + 1, 4 * (uint64_t)c->cus));
    // mode 0 (counts of cut blocks' inner segments): strided over the table
    const unsigned grid0 = std::min<unsigned>(grid, (unsigned)(4 * c->cus));
    for (int mode = 0; mode < 2; ++mode)
        hipLaunchKernelGGL(fe_rle1_kernel, dim3(mode ? grid : grid0), dim3(256), 0, s, d_x, (uint64_t)n, seg,
                           f.d_segfirst, f.d_nseg, f.d_segcnt, f.d_segcrc, mode, t.d_blocks, c->stride, t.d_lens,
                           t.d_crc, c->d_crctab);
    hipLaunchKernelGGL(fe_crccomb_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, seg, f.d_segfirst, cnt,
                       f.d_segcrc, t.d_crc, c->d_crctab);
    HIPCHECK(hipGetLastError());
    STAGE_DONE("front-rle1");
    return BZ2MI_OK;
}

// Blocks whose text fits in LDS take the block kernels; the rest take the
// grid path (big buckets, grid-wide doubling).  One predicate for the path and
// for the scratch it needs (A/B builds with -DBZ2MI_AB_NO_LDSTEXT send every
// block size to the grid path).
bool lds_text_path(int S) {
#ifdef BZ2MI_AB_NO_LDSTEXT
    (void)S;
    return false;
#else
    return S <= bz2mi::kBwtLdsText;
#endif
}

// The BWT's queues and (grid path) doubling scratch for batches of up to nb
// blocks; shared by the batches, so BWTs run one at a time (stream sA).
void free_bwt_scratch(bz2mi_ctx* c) {
    for (void* p : {(void*)c->d_sq, (void*)c->d_lq[0], (void*)c->d_lq[1], (void*)c->d_tq[0], (void*)c->d_tq[1],
                    (void*)c->d_tc, (void*)c->d_lspill, (void*)c->d_scb, (void*)c->d_dscratch, (void*)c->d_dlist[0],
                    (void*)c->d_dlist[1], (void*)c->d_dlarge[0], (void*)c->d_dlarge[1], (void*)c->d_dctr})
        if (p) (void)hipFree(p);
    c->d_dscratch = nullptr;
    c->d_dlist[0] = c->d_dlist[1] = c->d_dlarge[0] = c->d_dlarge[1] = nullptr;
    c->d_dctr = nullptr;
    c->d_sq = nullptr;
    c->d_lq[0] = c->d_lq[1] = nullptr;
    c->d_tq[0] = c->d_tq[1] = nullptr;
    c->d_tc = nullptr;
    c->d_lspill = nullptr;
    c->d_scb = nullptr;
    c->bwtq_blocks = 0;
}

int ensure_bwt_scratch(bz2mi_ctx* c, int nb) {
    using namespace bz2mi;
    if (nb <= c->bwtq_blocks) return BZ2MI_OK;
    free_bwt_scratch(c);
    const size_t B = (size_t)std::max(nb, 16);
    const size_t Bs = (B + kBwtShards - 1) / kBwtShards;  // blocks per shard
    int r;
    if ((r = dalloc(&c->d_sq, kBwtShards * Bs * bwt_squeue_per_block(c->S)))) return r;
    if ((r = dalloc(&c->d_lq[0], kBwtShards * Bs * bwt_lqueue_per_block(c->S)))) return r;
    if ((r = dalloc(&c->d_lq[1], kBwtShards * Bs * bwt_lqueue_per_block(c->S)))) return r;
    if ((r = dalloc(&c->d_tq[0], B * bwt_squeue_per_block(c->S)))) return r;
    if ((r = dalloc(&c->d_tq[1], B * bwt_squeue_per_block(c->S)))) return r;
    if ((r = dalloc(&c->d_tc, 2 * B))) return r;
    if ((r = dalloc(&c->d_lspill, B * c->stride))) return r;
    if ((r = dalloc(&c->d_scb, B))) return r;
    if (!lds_text_path(c->S)) {
        if ((r = dalloc(&c->d_dscratch, B * dbl_slot_bytes(c->S)))) return r;
        for (int k = 0; k < 2; ++k) {
            if ((r = dalloc(&c->d_dlist[k], B * dbl_list_cap(c->S)))) return r;
            if ((r = dalloc(&c->d_dlarge[k], B * dbl_large_cap(c->S)))) return r;
        }
        if ((r = dalloc(&c->d_dctr, (size_t)kDblCtr * (kDblMaxRounds + 2)))) return r;
    }
    c->bwtq_blocks = (int)B;
    return BZ2MI_OK;
}

// Device bytes per block of one batch set (ensure_batch) and of the BWT
// scratch (ensure_bwt_scratch): what a batch of B blocks costs, for sizing
// batches against the free HBM.
size_t batch_block_bytes(const bz2mi_ctx* c) {
    const size_t st = c->stride;
    return 2 * st + 4 * st + 8 * bz2mi::bwt_group_stride(st) + 2 * c->mtf_stride + 4 * c->payload_words +
           8 * (size_t)bz2mi::kMaxAlpha + 32 + 64;
}
size_t bwt_block_bytes(const bz2mi_ctx* c) {
    using namespace bz2mi;
    size_t b = 3 * 8 * bwt_squeue_per_block(c->S) + 2 * sizeof(BwtItem) * bwt_lqueue_per_block(c->S) + 4 * c->stride +
               16;
    if (!lds_text_path(c->S)) b += dbl_slot_bytes(c->S) + 16 * (dbl_list_cap(c->S) + dbl_large_cap(c->S));
    return b;
}

int stage_bwt(bz2mi_ctx* c, Batch& t, int nb, hipStream_t s) {
    using namespace bz2mi;
    if (nb > c->bwtq_blocks) {  // the queues are reallocated: earlier BWTs on s must be done
        HIPCHECK(hipStreamSynchronize(s));
        if (int r = ensure_bwt_scratch(c, nb)) return r;
    }
    const size_t Bs = ((size_t)c->bwtq_blocks + kBwtShards - 1) / kBwtShards;
    const size_t scap = Bs * bwt_squeue_per_block(c->S), lcap = Bs * bwt_lqueue_per_block(c->S);
    const size_t tcap = bwt_squeue_per_block(c->S);
    HIPCHECK(hipMemsetAsync(t.d_bcnt, 0, 1024 * sizeof(uint32_t), s));
    HIPCHECK(hipMemsetAsync(t.d_ngroups, 0, nb * sizeof(uint32_t), s));
    HIPCHECK(hipMemsetAsync(c->d_tc, 0, nb * sizeof(uint32_t), s));
    const int slots = std::min(nb, c->bwt_slots);
    uint32_t* scount = t.d_bcnt;             // kBwtShards counters
    uint32_t* lcount = t.d_bcnt + kBwtShards;  // level d: lcount + d * kBwtShards (queue d_lq[d & 1])
    uint32_t* tc[2] = {c->d_tc, c->d_tc + c->bwtq_blocks};
    uint32_t* p2count = t.d_bcnt + 768;
    uint32_t* pull = t.d_bcnt + 769;
    // A/B builds only (-DBZ2MI_AB_NO_LDSTEXT / _NO_TEXTBWT / _NO_WLEVEL): the
    // product has no run-time path switches
    // LDS-text path (blocks fit in LDS): the small batches of the levels go to
    // per-block lists (counts d_scb, capacity tcap each) instead of the shards
    const bool blk = lds_text_path(c->S);
    uint32_t* sq_count = blk ? c->d_scb : scount;
    const size_t sq_cap = blk ? tcap : scap;
    const uint32_t smask = blk ? 0xffffffffu : (uint32_t)(kBwtShards - 1);
    if (blk) {
        HIPCHECK(hipMemsetAsync(c->d_scb, 0, nb * sizeof(uint32_t), s));
        HIPCHECK(hipMemsetAsync(t.d_redo, 0, nb * sizeof(uint32_t), s));
        // mode 0 defers text-like blocks to the induced-sorting text kernel,
        // mode 1 takes the ones it hands back
#ifdef BZ2MI_AB_NO_TEXTBWT
        constexpr bool text_path = false;
#else
        constexpr bool text_path = true;
#endif
        for (int mode = 0; mode < 2; ++mode) {
            if (mode == 1 && text_path) {
                hipLaunchKernelGGL(bwt_text_kernel, dim3(nb), dim3(1024), 0, s, t.d_blocks, c->stride, t.d_lens, nb,
                                   t.d_sa, t.d_bwt, t.d_orig, t.d_redo, c->d_lspill, t.d_groups, c->d_tq[0],
                                   c->d_tq[1], tcap, c->wq_cap);
                HIPCHECK(hipGetLastError());
            }
            if (mode == 1 && !text_path) {  // every text-like block back to the general path
                hipLaunchKernelGGL(redo_all_kernel, dim3((nb + 255) / 256), dim3(256), 0, s, t.d_redo, nb);
            }
            hipLaunchKernelGGL(bwt_block_kernel, dim3(nb), dim3(1024), 0, s, t.d_blocks, c->stride, t.d_lens, nb,
                               t.d_sa, t.d_bwt, t.d_orig, c->d_lq[1], lcount + kBwtShards, lcap, t.d_present,
                               c->d_tq[0], tc[0], tcap, t.d_redo, mode, c->d_sq, c->d_scb, tcap);
        }
    } else {
        // mid-size first-byte buckets listed in the second tie list (free
        // until the tie rounds), sorted whole by bwt_bigbucket_kernel; its
        // counts start at zero (the bucket kernel also writes them, 0/1-byte
        // blocks included)
        HIPCHECK(hipMemsetAsync(tc[1], 0, nb * sizeof(uint32_t), s));
        hipLaunchKernelGGL(bwt_bucket_kernel, dim3(nb), dim3(256), 0, s, t.d_blocks, c->stride, t.d_lens, nb, t.d_sa,
                           t.d_bwt, t.d_orig, c->d_sq, scount, scap, c->d_lq[1], lcount + kBwtShards, lcap,
                           t.d_present, c->d_tq[1], tc[1], tcap);
        HIPCHECK(hipGetLastError());
        hipLaunchKernelGGL(bwt_bigbucket_kernel, bigbucket_grid(nb), dim3(kBigBucketThreads), 0, s, t.d_blocks, c->stride,
                           t.d_lens, t.d_sa, t.d_bwt, t.d_orig, c->d_tq[1], tc[1], tcap, c->d_tq[0], tc[0], tcap,
                           c->d_lq[0], lcount + 2 * kBwtShards, lcap, nb);
    }
    HIPCHECK(hipGetLastError());
    STAGE_DONE("bwt_bucket");
    if (blk && getenv("BZ2MI_BWT_STATS")) {  // debug: how the blocks went (0 general, 1 text, 2 handed back)
        std::vector<uint32_t> r(nb);
        HIPCHECK(hipMemcpyAsync(r.data(), t.d_redo, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        unsigned cnt[4] = {0, 0, 0, 0};
        for (uint32_t v : r) cnt[v < 4 ? v : 3]++;
        fprintf(stderr, "[bz2mi] bwt blocks: general %u, text %u, handed back %u\n", cnt[0], cnt[1], cnt[2] + cnt[3]);

    }
#ifdef BZ2MI_AB_NO_WLEVEL
    constexpr bool wlevel = false;
#else
    constexpr bool wlevel = true;
#endif
    for (int d = 1; d <= kBwtLevels; ++d) {
        if (wlevel && d < kBwtLevels) {
            hipLaunchKernelGGL(bwt_wlevel_kernel, dim3(c->wlevel_grid), dim3(256), 0, s, t.d_blocks, c->stride,
                               t.d_lens, t.d_sa, t.d_bwt, t.d_orig, c->d_lspill, c->d_lq[d & 1],
                               lcount + d * kBwtShards, c->d_lq[(d + 1) & 1], lcount + (d + 1) * kBwtShards, lcap,
                               c->d_sq, sq_count, sq_cap, t.d_groups, t.d_ngroups, t.d_p2list, p2count, smask);
            HIPCHECK(hipGetLastError());
            continue;
        }
        hipLaunchKernelGGL(bwt_level_kernel, dim3(c->level_slots), dim3(256), 0, s, t.d_blocks, c->stride, t.d_lens,
                           t.d_sa, t.d_bwt, t.d_orig, c->d_lscratch, c->d_lspill, bwt_level_slot_bytes(c->S), c->S, c->d_lq[d & 1],
                           lcount + d * kBwtShards, c->d_lq[(d + 1) & 1], lcount + (d + 1) * kBwtShards, lcap,
                           c->d_sq, sq_count, sq_cap, t.d_groups, t.d_ngroups, t.d_p2list, p2count,
                           d == kBwtLevels ? 1 : 0, smask);
        HIPCHECK(hipGetLastError());
    }
    STAGE_DONE("bwt_levels");
    if (blk)
        hipLaunchKernelGGL(bwt_block_small_kernel, dim3(nb), dim3(1024), 0, s, t.d_blocks, c->stride, t.d_lens, nb,
                           t.d_sa, t.d_bwt, t.d_orig, c->d_sq, c->d_scb, tcap, c->d_tq[0], tc[0], tcap);
    else
        hipLaunchKernelGGL(bwt_small_kernel, dim3(c->small_grid), dim3(256), 0, s, t.d_blocks, c->stride, t.d_lens,
                           t.d_sa, t.d_bwt, t.d_orig, c->d_sq, scount, scap, c->d_tq[0], tc[0], tcap);
    HIPCHECK(hipGetLastError());
    STAGE_DONE("bwt_small");
    // tie rounds of 8 bytes, then the doubling (fewer on the grid path, whose
    // doubling resolves long repeated passages directly)
    // (big blocks: 8 workgroups per block, each a slice of its list)
    const int tie_rounds = blk ? kBwtTieRounds : kBwtTieRoundsGrid;
    for (int r = 0; r < tie_rounds; ++r) {
        HIPCHECK(hipMemsetAsync(tc[(r + 1) & 1], 0, nb * sizeof(uint32_t), s));
        // (900 KB blocks: 8 slices per block, dealt to the XCDs by block)
        const dim3 tgrid = blk ? dim3(nb, 1) : dim3(8u * (unsigned)kTieSlices * (((unsigned)nb + 7u) / 8u));
        hipLaunchKernelGGL(bwt_tie_kernel, tgrid, dim3(256), 0, s, t.d_blocks, c->stride, t.d_lens, t.d_sa,
                           t.d_bwt, t.d_orig, c->d_tq[r & 1], tc[r & 1], c->d_tq[(r + 1) & 1], tc[(r + 1) & 1], tcap,
                           t.d_groups, t.d_ngroups, t.d_p2list, p2count, r + 1 == tie_rounds ? 1 : 0, nb, blk ? 0 : 1);
        HIPCHECK(hipGetLastError());
    }
    STAGE_DONE("bwt_ties");
    if (blk) {
        hipLaunchKernelGGL(bwt_double_kernel, dim3(slots), dim3(256), 0, s, t.d_blocks, c->stride, t.d_lens, nb,
                           t.d_sa, t.d_bwt, t.d_orig, c->d_scratch, bwt_slot_bytes(c->S), c->S, t.d_groups,
                           t.d_ngroups, t.d_p2list, p2count, pull);
        HIPCHECK(hipGetLastError());
        if (getenv("BZ2MI_BWT_STATS")) {  // debug: blocks that reached the doubling
            uint32_t np = 0;
            HIPCHECK(hipMemcpyAsync(&np, p2count, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            HIPCHECK(hipStreamSynchronize(s));
            fprintf(stderr, "[bz2mi] doubling: %u blocks\n", np);
        }
    } else {
        // grid-wide doubling: every launch returns at once when nothing is left;
        // when no block has groups left after the tie rounds (random-like
        // data) its ~100 launches are skipped (one count read back instead)
        {
            uint32_t np = 0;
            HIPCHECK(hipMemcpyAsync(&np, p2count, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            HIPCHECK(hipStreamSynchronize(s));
            if (np == 0) {
                STAGE_DONE("bwt");
                return BZ2MI_OK;
            }
        }
        DblGrid G{t.d_blocks, c->stride, t.d_lens, t.d_sa, t.d_bwt, t.d_orig, t.d_groups, t.d_ngroups, t.d_p2list,
                  p2count, c->d_dscratch, dbl_slot_bytes(c->S), c->S, {c->d_dlist[0], c->d_dlist[1]},
                  {c->d_dlarge[0], c->d_dlarge[1]}, c->d_dctr};
#ifndef BZ2MI_AB_DBL_GRID
#define BZ2MI_AB_DBL_GRID 4
#endif
        const dim3 grid((unsigned)c->cus * BZ2MI_AB_DBL_GRID), blk256(256);
        HIPCHECK(hipMemsetAsync(c->d_dctr, 0, sizeof(uint32_t) * kDblCtr * (kDblMaxRounds + 2), s));
        hipLaunchKernelGGL(dbl_init_rank_kernel, grid, blk256, 0, s, G);
        hipLaunchKernelGGL(dbl_init_groups_kernel, grid, blk256, 0, s, G);
        const int R = dbl_rounds(c->S);
        for (int r = 0; r < R; ++r) {
            hipLaunchKernelGGL(dbl_pairset_kernel, grid, blk256, 0, s, G, r);
            hipLaunchKernelGGL(dbl_runend_kernel, grid, blk256, 0, s, G, r);
            hipLaunchKernelGGL(dbl_decide_kernel, grid, blk256, 0, s, G, r);
            hipLaunchKernelGGL(dbl_snap_kernel, grid, blk256, 0, s, G, r);
            hipLaunchKernelGGL(dbl_sort_kernel, grid, blk256, 0, s, G, r);
            hipLaunchKernelGGL(dbl_large_kernel, grid, blk256, 0, s, G, r);
        }
        hipLaunchKernelGGL(dbl_emit_kernel, grid, blk256, 0, s, G);
        HIPCHECK(hipGetLastError());
        if (getenv("BZ2MI_DBL_STATS")) {  // debug: per-round group counts
            std::vector<uint32_t> h((size_t)kDblCtr * (kDblMaxRounds + 2));
            uint32_t np = 0;
            HIPCHECK(hipMemcpyAsync(h.data(), c->d_dctr, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            HIPCHECK(hipMemcpyAsync(&np, p2count, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            HIPCHECK(hipStreamSynchronize(s));
            fprintf(stderr, "[bz2mi] doubling: %u blocks\n", np);
            for (int r = 0; r < R; ++r) {
                const uint32_t* q = &h[(size_t)kDblCtr * r];
                if (q[0] + q[2] == 0) break;
                fprintf(stderr, "  round %d: groups %u large %u -> kept %u; pairs on %u decided %u undecided %u\n", r,
                        q[0], q[2], q[1], q[6], q[3], q[4]);
            }
        }
    }
    STAGE_DONE("bwt");
    return BZ2MI_OK;
}

int stage_mtf(bz2mi_ctx* c, Batch& t, int nb, hipStream_t s) {
    using namespace bz2mi;
    // segment scratch: the block's SA area (free after the BWT), stride uint32 = 2 * stride u16
    launch_mtf(nb, t.d_bwt, c->stride, t.d_lens, t.d_present, t.d_mtf, c->mtf_stride, t.d_mtflen, t.d_alpha, t.d_hist,
               reinterpret_cast<uint16_t*>(t.d_sa), 2 * c->stride, s);
    HIPCHECK(hipGetLastError());
    STAGE_DONE("mtf");
    return BZ2MI_OK;
}

int stage_seed(bz2mi_ctx* c, Batch& t, int nb, uint64_t first_block, uint32_t* state, hipStream_t s) {
    using namespace bz2mi;
    const int ng = c->p * ((kMaxAlpha + 63) / 64);
    hipLaunchKernelGGL(seed_kernel, dim3(ng), dim3(kSeedWaves * 64), 0, s, t.d_hist, t.d_seed, state, nb, c->p,
                       first_block);
    HIPCHECK(hipGetLastError());
    STAGE_DONE("seed");
    return BZ2MI_OK;
}

int stage_huffman(bz2mi_ctx* c, Batch& t, int nb, hipStream_t s) {
    using namespace bz2mi;
    const size_t sel_bytes = ((size_t)(c->S + 1 + 49) / 50 + 15) & ~(size_t)15;
    hipLaunchKernelGGL(huffman_kernel, dim3(nb), dim3(huffman_threads()), sel_bytes, s, t.d_mtf, c->mtf_stride, t.d_mtflen, t.d_alpha,
                       t.d_seed, t.d_present, t.d_orig, nb, t.d_payload, c->payload_words, t.d_pbits);
    HIPCHECK(hipGetLastError());
    STAGE_DONE("huffman");
    return BZ2MI_OK;
}

int ensure_front(FrontBufs& f, int S, size_t n) {
    if (n <= f.n_cap && f.d_dmap) return BZ2MI_OK;
    const size_t cap = std::max(n, (size_t)1 << 20);
    const size_t nc = (cap + bz2mi::kFeChunk - 1) / bz2mi::kFeChunk;
    const size_t maxb = (cap + cap / 4) / (size_t)(S - 5) + 8;
    int r;
    if ((r = dalloc(&f.d_dmap, cap + cap / 4 + 4096))) return r;
    if ((r = dalloc(&f.d_lane, nc * 64 + 64))) return r;
    if ((r = dalloc(&f.d_summ, nc + 1))) return r;
    if ((r = dalloc(&f.d_rsb, nc + 2))) return r;
    if ((r = dalloc(&f.d_agg, nc / kFeScanTile + 2))) return r;
    if ((r = dalloc(&f.d_ccost, nc + 1))) return r;
    if ((r = dalloc(&f.d_fc, nc + 2))) return r;
    if ((r = dalloc(&f.d_bnd, maxb + 2))) return r;
    if ((r = dalloc(&f.d_starts, maxb + 3))) return r;
    if ((r = dalloc(&f.d_nb, 4))) return r;
    if ((r = dalloc(&f.d_spec, maxb + 3))) return r;
    // segments: one per block, plus one per kFeSegLen raw bytes of a cut block
    const size_t segs = maxb + cap / bz2mi::kFeSegLen + 8;
    if ((r = dalloc(&f.d_seg, segs * bz2mi::kFeSegBytes))) return r;
    if ((r = dalloc(&f.d_segfirst, maxb + 8))) return r;
    if ((r = dalloc(&f.d_nseg, 4))) return r;
    HIPCHECK(hipMemset(f.d_nseg, 0, 4 * sizeof(uint32_t)));  // [1]: segment table overflow (sticky)
    if ((r = dalloc(&f.d_segcnt, segs))) return r;
    if ((r = dalloc(&f.d_segcrc, segs))) return r;
    f.seg_cap = segs;
    f.n_cap = cap;
    f.maxb = maxb;
    return BZ2MI_OK;
}

void free_front(FrontBufs& f) {
    for (void* p : f.ptrs())
        if (p) (void)hipFree(p);
    f = FrontBufs{};
}

int enqueue_front_scan(FrontBufs& f, const uint8_t* d_x, size_t n, hipStream_t s) {
    using namespace bz2mi;
    if (n == 0) return BZ2MI_OK;
    const uint64_t nc = (n + kFeChunk - 1) / kFeChunk;
    const dim3 g4((unsigned)((nc + 3) / 4));
    hipLaunchKernelGGL(fe_summary_kernel, g4, dim3(256), 0, s, d_x, (uint64_t)n, nc, f.d_summ, f.d_ccost);
    const dim3 gs((unsigned)((nc + kFeScanTile - 1) / kFeScanTile));
    for (int pass = 0; pass < 2; ++pass)
        hipLaunchKernelGGL(fe_runscan_kernel, gs, dim3(kFeScanThreads), 0, s, f.d_summ, nc, f.d_rsb, f.d_agg, pass);
    for (int pass = 0; pass < 2; ++pass)
        hipLaunchKernelGGL(fe_costscan_kernel, gs, dim3(kFeScanThreads), 0, s, f.d_ccost, f.d_summ, f.d_rsb, nc, f.d_fc,
                           f.d_agg, pass);
    hipLaunchKernelGGL(fe_dmap_kernel, g4, dim3(256), 0, s, d_x, f.d_summ, f.d_rsb, (uint64_t)n, nc, f.d_fc, f.d_dmap,
                       f.d_lane);
    HIPCHECK(hipGetLastError());
    STAGE_DONE("front-scan");
    return BZ2MI_OK;
}

__global__ void copy_u64_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int run_chain(bz2mi_ctx* c, FrontBufs& f, const uint8_t* d_x, size_t n, size_t n_own, uint64_t entry, bool ends,
              uint64_t* nb_out, uint64_t* exit_out, hipStream_t s, uint64_t spec_nb, uint64_t spec_exit,
              uint64_t* spliced) {
    using namespace bz2mi;
    const uint64_t nc = (n + kFeChunk - 1) / kFeChunk;
    if (spec_nb > f.maxb) return fail(BZ2MI_EINVAL, "run_chain: speculation longer than the block table");
    hipLaunchKernelGGL(fe_chain_kernel, dim3(1), dim3(kFeChainThreads), 0, s, d_x, f.d_lane, f.d_fc, f.d_summ, f.d_dmap,
                       (uint64_t)n, nc, c->S, (uint64_t)n_own, entry, ends ? 1 : 0, f.d_bnd, (uint64_t)f.maxb,
                       f.d_nb, f.d_spec, spec_nb);
    HIPCHECK(hipGetLastError());
    STAGE_DONE("front-chain");
    uint64_t hv[4] = {0, 0, 0, 0};
    HIPCHECK(hipMemcpyAsync(hv, f.d_nb, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    if (hv[1] == 1) return fail(BZ2MI_EINVAL, "stream unit: the last block runs past the tail halo");
    const uint64_t J = hv[3];  // merged into the speculative chain at its block J
    if (hv[1] != 0 || hv[0] > f.maxb || (J == 0 && hv[0] == 0) || (J != 0 && (J >= spec_nb || hv[0] == 0)))
        return fail(BZ2MI_EDEVICE, "front end produced an invalid block count");
    uint64_t nb = hv[0];
    hipLaunchKernelGGL(fe_resolve_kernel, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s, d_x, f.d_lane, f.d_fc,
                       f.d_summ, (uint64_t)n, nc, (uint64_t)n_own, entry, f.d_bnd, f.d_nb, f.d_starts);
    HIPCHECK(hipGetLastError());
    STAGE_DONE("front-resolve");
    if (spliced) *spliced = 0;
    if (J) {
        // starts[nb] == spec[J]: the speculative starts after it and its end
        const uint64_t tail = spec_nb - J;
        if (nb + tail > f.maxb) return fail(BZ2MI_EDEVICE, "front end produced an invalid block count");
        // (a kernel: a DMA copy here measured as waiting for the other streams' work)
        hipLaunchKernelGGL(copy_u64_kernel, dim3((unsigned)std::min<uint64_t>((tail + 255) / 256, 64)), dim3(256), 0, s,
                           f.d_spec + J + 1, f.d_starts + nb + 1, tail);
        HIPCHECK(hipGetLastError());
        nb += tail;
        if (spliced) *spliced = tail;
        if (exit_out) *exit_out = spec_exit;
        if (hipStreamSynchronize(s) != hipSuccess) return fail(BZ2MI_EDEVICE, "run_chain: splice failed");
    } else if (exit_out) {
        HIPCHECK(hipMemcpyAsync(exit_out, f.d_nb + 2, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
    }
    *nb_out = nb;
    return BZ2MI_OK;
}

}  // namespace host
}  // namespace bz2mi

namespace {

// host-driven paths: batch set 0 plus the assembly staging buffer
int ensure_capacity(bz2mi_ctx* c, int nblocks) {
    int r;
    if ((r = ensure_batch(c, c->sets[0], nblocks))) return r;
    const size_t words = (size_t)c->sets[0].cap * (c->payload_words + 4) + 64;
    if (words > c->out_words) {
        if ((r = dalloc(&c->d_out, words))) return r;
        c->out_words = words;
    }
    return BZ2MI_OK;
}

// Host-driven kernel sequence for `nb` RLE1 blocks already in set 0
// (d_blocks/d_lens/d_crc), all on the context stream.  Produces
// d_payload/d_pbits.
int run_blocks(bz2mi_ctx* c, int nb) {
    hipStream_t s = c->stream;
    Batch& t = c->sets[0];
    int r;
    (void)hipGetLastError();
    HIPCHECK(hipEventRecord(c->ev[0], s));
    if ((r = stage_bwt(c, t, nb, s))) return r;
    HIPCHECK(hipEventRecord(c->ev[1], s));
    if ((r = stage_mtf(c, t, nb, s))) return r;
    HIPCHECK(hipEventRecord(c->ev[2], s));
    if ((r = stage_seed(c, t, nb, c->blocks_done, c->d_state, s))) return r;
    HIPCHECK(hipEventRecord(c->ev[3], s));
    if ((r = stage_huffman(c, t, nb, s))) return r;
    HIPCHECK(hipEventRecord(c->ev[4], s));
    return BZ2MI_OK;
}

// Lay the stream bits of `nb` compressed blocks (plus prefix: the stream
// header on the first call, else the carried bits; plus the trailer when
// final_) into dst as a byte stream.  Returns the total bit count; the last
// partial byte stays in dst.
int assemble_to(bz2mi_ctx* c, int nb, bool final_, uint32_t* dst, size_t dst_bytes, uint64_t* total_bits_out) {
    using namespace bz2mi;
    hipStream_t s = c->stream;
    uint64_t prefix = c->carry;
    int prefix_bits = c->carry_bits;
    if (!c->header_done) {
        // 'B' 'Z' 'h' '0'+level (OutputStream.hpp:126-128); nothing is carried yet
        prefix = ((uint64_t)0x425a68u << 40) | ((uint64_t)('0' + c->level) << 32);
        prefix_bits = 32;
    }
    (void)hipGetLastError();
    hipLaunchKernelGGL(offsets_kernel, dim3(1), dim3(256), 0, s, c->sets[0].d_pbits, nb, (uint64_t)prefix_bits, c->sets[0].d_offs);
    HIPCHECK(hipGetLastError());
    uint64_t end_bits = 0;
    HIPCHECK(hipMemcpyAsync(&end_bits, c->sets[0].d_offs + nb, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    if (final_) end_bits += 80;
    const uint64_t words = (end_bits + 31) / 32;
    if (words * 4 > dst_bytes) return fail(BZ2MI_ESPACE, "output buffer too small");
    hipLaunchKernelGGL(assemble_kernel, dim3(nb + 2), dim3(256), 0, s, c->sets[0].d_payload, c->payload_words, c->sets[0].d_offs,
                       c->sets[0].d_crc, nb, prefix, prefix_bits, final_ ? 1 : 0, c->stream_crc, dst);
    HIPCHECK(hipGetLastError());
    STAGE_DONE("assemble");
    HIPCHECK(hipEventRecord(c->ev[5], s));
    *total_bits_out = final_ ? (end_bits + 7) & ~7ull : end_bits;  // final: zero padding
    c->header_done = true;
    return BZ2MI_OK;
}

void record_timings(bz2mi_ctx* c, int nb) {
    if (nb > 0) {
        float ms;
        for (int i = 0; i < 5; ++i)
            if (hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]) == hipSuccess) c->last_ms[i + 1] = ms;
    }
    (void)hipGetLastError();  // timing queries must not leave a sticky error behind
}

// Assemble into the context's staging buffer and copy complete bytes to host.
int assemble(bz2mi_ctx* c, int nb, bool final_, uint8_t* out, size_t cap, size_t* out_len) {
    uint64_t total_bits = 0;
    int r = assemble_to(c, nb, final_, c->d_out, c->out_words * 4, &total_bits);
    if (r) return r;
    const size_t nbytes = (size_t)(total_bits >> 3);
    const int rem = (int)(total_bits & 7);
    if (nbytes > cap) return fail(BZ2MI_ESPACE, "output buffer too small");
    c->h_stage.resize(nbytes + 8);
    HIPCHECK(hipMemcpyAsync(c->h_stage.data(), c->d_out, nbytes + (rem ? 1 : 0), hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    std::memcpy(out, c->h_stage.data(), nbytes);
    *out_len = nbytes;
    c->carry = rem ? ((uint64_t)c->h_stage[nbytes] << 56) & (~0ull << (64 - rem)) : 0;
    c->carry_bits = rem;
    record_timings(c, nb);
    return BZ2MI_OK;
}

void reset_stream(bz2mi_ctx* c) {
    c->blocks_done = 0;
    c->stream_crc = 0;
    c->carry = 0;
    c->carry_bits = 0;
    c->header_done = false;
    c->finished = false;
    (void)hipMemsetAsync(c->d_state, 0, sizeof(uint32_t) * c->p * bz2mi::kMaxAlpha, c->stream);
}

// Per-batch stage timing: events 2*i / 2*i+1 bracket stage i of a batch
// (0 RLE1+CRC, 1 BWT, 2 MTF, 3 seed, 4 Huffman, 5 assembly).
hipEvent_t* batch_events(bz2mi_ctx* c, uint64_t k) {
    const size_t need = (size_t)(k + 1) * 12;
    while (c->tev.size() < need) {
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        c->tev.push_back(e);
    }
    return c->tev.data() + k * 12;
}

// Whole stream from device bytes.  Front end (RLE1 split) for the whole input
// on the context stream, then the blocks in batches through a three-stream
// pipeline: stream A runs RLE1 emission, block CRCs and the BWT of batch k
// while stream M runs the MTF of batch k-1 and stream B the seeds, Huffman
// coding and assembly of batch k-2 (the seed carry-over and the stream
// offsets chain through stream B in batch order).  The stream state (bit
// offset, carried partial word, stream CRC) stays on the device, so the host
// waits once, for the final length.
int compress_device_impl(bz2mi_ctx* c, const uint8_t* d_x, size_t n, uint8_t* d_out, size_t cap, size_t* out_len) {
    using namespace bz2mi;
    hipStream_t s = c->stream;
    int r;
    reset_stream(c);
    if ((r = ensure_front(c->fe, c->S, n))) return r;
    uint64_t nb = 0;
    (void)hipGetLastError();
    HIPCHECK(hipEventRecord(c->ev[6], s));
    if (n > 0) {
        if ((r = enqueue_front_scan(c->fe, d_x, n, s))) return r;
        if ((r = run_chain(c, c->fe, d_x, n, n, 0, true, &nb, nullptr, s))) return r;
    }
    HIPCHECK(hipEventRecord(c->ev[7], s));
    // batches: the batch buffers and the BWT scratch are sized before the
    // pipeline starts; when an allocation fails (another context or process
    // holds much of HBM) every batch buffer is freed and the batch halved
    uint64_t bsz = (uint64_t)c->batch_blocks;
    bool recovered = false;
    {
        // at most ~80 % of what is free now, counting the buffers this context
        // already holds (they are reused or freed below)
        size_t fr = 0, tot = 0;
        if (nb && hipMemGetInfo(&fr, &tot) == hipSuccess) {
            size_t held = (size_t)c->bwtq_blocks * bwt_block_bytes(c);
            for (const Batch& t : c->sets) held += (size_t)t.cap * batch_block_bytes(c);
            const size_t avail = (fr + held) / 10 * 8;
            const uint64_t want = std::min(bsz, nb);
            const size_t per1 = batch_block_bytes(c) + bwt_block_bytes(c);  // one batch: one set
            const size_t per3 = kSets * batch_block_bytes(c) + bwt_block_bytes(c);
            if (want * (want < nb ? per3 : per1) > avail) {
                const uint64_t fit = std::max<uint64_t>(1, avail / per3);
                const uint64_t k = (nb + fit - 1) / fit;  // batches
                bsz = std::max<uint64_t>(1, (nb + k - 1) / k);
            }
        }
    }
    for (;;) {
        const uint64_t want = std::max<uint64_t>(std::min(bsz, nb), 1);
        const int sets_try = (int)std::min<uint64_t>(nb ? (nb + bsz - 1) / bsz : 1, kSets);
        r = BZ2MI_OK;
        for (int k = 0; k < sets_try && !r; ++k) r = ensure_batch(c, c->sets[k], (int)want);
        if (!r && (int)want > c->bwtq_blocks) {
            HIPCHECK(hipStreamSynchronize(c->sA));
            r = ensure_bwt_scratch(c, (int)want);
        }
        if (!r) break;
        if (want <= 1) return r;
        for (hipStream_t st : {c->sA, c->sM, c->sB}) HIPCHECK(hipStreamSynchronize(st));
        for (Batch& t : c->sets) free_batch(t);
        free_bwt_scratch(c);
        (void)hipGetLastError();
        // (halved for this call only: a later call sizes its batch again
        // from the HBM then free)
        bsz = (want + 1) / 2;
        recovered = true;
    }
    if (recovered) clear_error();
    const uint64_t nbat = nb ? (nb + bsz - 1) / bsz : 1;
    // output: word-aligned destination, else an aligned staging buffer
    uint32_t* out32 = (uint32_t*)d_out;
    const bool staged = ((uintptr_t)d_out & 3) != 0;
    if (staged) {
        if (cap + 8 > c->ostage_cap) {
            if ((r = dalloc(&c->d_ostage, cap + 8))) return r;
            c->ostage_cap = cap + 8;
        }
        out32 = (uint32_t*)c->d_ostage;
    }
    const uint64_t cap_words = cap / 4;
    // device stream state: the header "BZh<level>" (OutputStream.hpp:126-128) is carried in
    c->h_sd = StreamDev{};
    c->h_sd.carry = (0x425a68u << 8) | (uint32_t)('0' + c->level);
    c->h_sd.carry_bits = 32;
    HIPCHECK(hipMemcpyAsync(c->d_sd, &c->h_sd, sizeof(StreamDev), hipMemcpyHostToDevice, s));
    HIPCHECK(hipMemsetAsync(c->d_vol, 0, 4 * sizeof(unsigned long long), s));
    HIPCHECK(hipEventRecord(c->ev[0], s));
    HIPCHECK(hipStreamWaitEvent(c->sA, c->ev[0], 0));
    HIPCHECK(hipStreamWaitEvent(c->sM, c->ev[0], 0));
    HIPCHECK(hipStreamWaitEvent(c->sB, c->ev[0], 0));
    for (uint64_t k = 0; k < nbat; ++k) {
        Batch& t = c->sets[k % kSets];
        const uint64_t first = k * bsz;
        const uint64_t cnt = nb ? std::min(bsz, nb - first) : 0;
        const bool last = k + 1 == nbat;
        hipEvent_t* te = batch_events(c, k);
        if (cnt) {
            if (k >= (uint64_t)kSets) HIPCHECK(hipStreamWaitEvent(c->sA, t.evFree, 0));
            HIPCHECK(hipEventRecord(te[0], c->sA));
            if ((r = stage_front(c, t, c->fe, d_x, n, first, cnt, c->sA))) return r;
            HIPCHECK(hipEventRecord(te[1], c->sA));
            HIPCHECK(hipEventRecord(te[2], c->sA));
            if ((r = stage_bwt(c, t, (int)cnt, c->sA))) return r;
            HIPCHECK(hipEventRecord(te[3], c->sA));
            HIPCHECK(hipEventRecord(t.evA, c->sA));
            HIPCHECK(hipStreamWaitEvent(c->sM, t.evA, 0));
            HIPCHECK(hipEventRecord(te[4], c->sM));
            if ((r = stage_mtf(c, t, (int)cnt, c->sM))) return r;
            HIPCHECK(hipEventRecord(te[5], c->sM));
            HIPCHECK(hipEventRecord(t.evM, c->sM));
            HIPCHECK(hipStreamWaitEvent(c->sB, t.evM, 0));
            HIPCHECK(hipEventRecord(te[6], c->sB));
            if ((r = stage_seed(c, t, (int)cnt, first, c->d_state, c->sB))) return r;
            HIPCHECK(hipEventRecord(te[7], c->sB));
            HIPCHECK(hipEventRecord(te[8], c->sB));
            if ((r = stage_huffman(c, t, (int)cnt, c->sB))) return r;
            HIPCHECK(hipEventRecord(te[9], c->sB));
            hipLaunchKernelGGL(volume_kernel, dim3(16), dim3(256), 0, c->sB, t.d_lens, t.d_mtflen, t.d_pbits, (int)cnt,
                               c->d_vol);
        }
        HIPCHECK(hipEventRecord(te[10], c->sB));
        hipLaunchKernelGGL(offsets_dev_kernel, dim3(1), dim3(256), 0, c->sB, t.d_pbits, t.d_crc, (int)cnt, c->d_sd,
                           t.d_offs);
        hipLaunchKernelGGL(assemble_dev_kernel, dim3((unsigned)cnt + 2), dim3(256), 0, c->sB, t.d_payload,
                           c->payload_words, t.d_offs, t.d_crc, (int)cnt, last ? 1 : 0, c->d_sd, out32, cap_words);
        hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64), 0, c->sB, t.d_offs, (int)cnt, last ? 1 : 0, c->d_sd,
                           out32, cap_words);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipEventRecord(te[11], c->sB));
        HIPCHECK(hipEventRecord(t.evFree, c->sB));
    }
    HIPCHECK(hipMemcpyAsync(&c->h_sd, c->d_sd, sizeof(StreamDev), hipMemcpyDeviceToHost, c->sB));
    HIPCHECK(hipStreamSynchronize(c->sB));
    {
        uint32_t segov = 0;
        HIPCHECK(hipMemcpy(&segov, c->fe.d_nseg + 1, sizeof(segov), hipMemcpyDeviceToHost));
        if (segov) return fail(BZ2MI_EDEVICE, "front end: RLE1 segment table overflow");
    }
    const uint64_t bytes = (c->h_sd.final_bits + 7) / 8;
    if (bytes > cap_words * 4) return fail(BZ2MI_ESPACE, "output buffer too small");
    if (staged) HIPCHECK(hipMemcpy(d_out, c->d_ostage, bytes, hipMemcpyDeviceToDevice));
    // stage times summed over the batches (stages of different batches overlap)
    float fe_ms = 0;
    if (hipEventElapsedTime(&fe_ms, c->ev[6], c->ev[7]) != hipSuccess) fe_ms = 0;
    float sum[6] = {fe_ms, 0, 0, 0, 0, 0};
    for (uint64_t k = 0; k < nbat; ++k) {
        hipEvent_t* te = batch_events(c, k);
        float ms;
        if (nb) {
            if (hipEventElapsedTime(&ms, te[0], te[1]) == hipSuccess) sum[0] += ms;
            if (hipEventElapsedTime(&ms, te[2], te[3]) == hipSuccess) sum[1] += ms;
            if (hipEventElapsedTime(&ms, te[4], te[5]) == hipSuccess) sum[2] += ms;
            if (hipEventElapsedTime(&ms, te[6], te[7]) == hipSuccess) sum[3] += ms;
            if (hipEventElapsedTime(&ms, te[8], te[9]) == hipSuccess) sum[4] += ms;
        }
        if (hipEventElapsedTime(&ms, te[10], te[11]) == hipSuccess) sum[5] += ms;
    }
    (void)hipGetLastError();
    for (int i = 0; i < 6; ++i) c->last_ms[i] = sum[i];
    c->stats[0] = n;
    c->stats[1] = nb;
    c->stats[5] = bytes;
    {
        unsigned long long vol[4] = {0, 0, 0, 0};
        HIPCHECK(hipMemcpy(vol, c->d_vol, sizeof(vol), hipMemcpyDeviceToHost));
        c->stats[2] = vol[0];
        c->stats[3] = vol[1];
        c->stats[4] = vol[2];
        c->stats[6] = nb;
    }
    c->blocks_done = nb;
    c->finished = true;
    *out_len = bytes;
    return BZ2MI_OK;
}

}  // namespace

extern "C" {

const char* bz2mi_last_error(void) { return g_err.c_str(); }

const char* bz2mi_version(void) { return "bz2mi 0.4 (gfx950)"; }
int bz2mi_abi_version(void) { return BZ2MI_ABI_VERSION; }

int bz2mi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

size_t bz2mi_compress_bound(size_t n, int level, int unit) {
    const size_t S = (size_t)unit * (size_t)level;
    const size_t blocks = (n + n / 4) / (S - 5) + 2;
    const size_t per = (S + 1) * 20 / 8 + (S / 50 + 2) + 6 * 258 * 5 + 1024;
    return 64 + blocks * per;
}

bz2mi_ctx* bz2mi_create(int level, int parallel_blocks, int unit, int device) {
    if (level < 1 || level > 9) {
        fail(BZ2MI_EINVAL, "Invalid block size");
        return nullptr;
    }
    if (parallel_blocks < 1) {
        fail(BZ2MI_EINVAL, "Invalid parallel block count");
        return nullptr;
    }
    if (unit < 100 || (size_t)unit * level > (1u << 20) - 16) {
        fail(BZ2MI_EINVAL, "Invalid block unit");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
        fail(BZ2MI_EDEVICE, "no HIP device available for bz2mi");
        return nullptr;
    }
    auto* c = new bz2mi_ctx();
    c->level = level;
    c->p = parallel_blocks;
    c->unit = unit;
    c->S = unit * level;
    c->device = device;
    c->stride = ((size_t)c->S + 16 + 63) & ~(size_t)63;
    c->mtf_stride = ((size_t)c->S + 10 + 31) & ~(size_t)31;  // (+8: room for 16-byte reads past a group)
    {
        const size_t S = (size_t)c->S;
        const size_t bits = 24 + 272 + 18 + (S / 50 + 1) * 6 + 6 * (5 + 258 * 39) + (S + 1) * 20;
        c->payload_words = (bits + 31) / 32 + 4;
    }
    // stream B (seeds, Huffman, assembly) at the highest priority: when the
    // stages of several batches / stream units are in flight, the kernels that
    // finish a unit are dispatched ahead of the MTF / BWT kernels of later ones
    // (at equal priority the hardware queues served those first and the
    // units' Huffman kernels formed a tail).  Stream A (RLE1 emission, BWT:
    // the long pole) too: the next unit's RLE1 + BWT are dispatched ahead of
    // the previous unit's MTF (N = 1 unit line 40.4 -> 41.3 GB/s).
    int prio_lo = 0, prio_hi = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
    // A/B knob BZ2MI_STREAM_PRIO: five digits for stream, A, M, B, F
    // (0 default, 1 highest, 2 lowest)
    int pr[5] = {0, 1, 0, 1, 0};
    if (const char* e = getenv("BZ2MI_STREAM_PRIO"))
        for (int i = 0; i < 5 && e[i]; ++i) pr[i] = e[i] - '0';
    auto mk = [&](hipStream_t* st, int k) {
        if (pr[k] == 0) return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
        return hipStreamCreateWithPriority(st, hipStreamNonBlocking, pr[k] == 1 ? prio_hi : prio_lo);
    };
    if (hipSetDevice(device) != hipSuccess || mk(&c->stream, 0) != hipSuccess || mk(&c->sA, 1) != hipSuccess ||
        mk(&c->sM, 2) != hipSuccess || mk(&c->sB, 3) != hipSuccess || mk(&c->sF, 4) != hipSuccess) {
        fail(BZ2MI_EDEVICE, "hipStreamCreate failed");
        bz2mi_destroy(c);
        return nullptr;
    }
    c->own_stream = true;
    hipDeviceProp_t prop;
    int cus = 256;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) cus = prop.multiProcessorCount;
    c->cus = cus;
    c->bwt_slots = cus * 4;
    {
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(bz2mi::bwt_small_kernel),
                                                         256, 0) != hipSuccess || occ < 1)
            occ = 2;
        c->small_grid = std::max(8, cus * occ / 8 * 8);  // multiple of 8 (XCD split)
        occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(bz2mi::bwt_level_kernel),
                                                         256, 0) != hipSuccess || occ < 1)
            occ = 4;
        c->level_slots = std::max(8, cus * occ / 8 * 8);
        occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(bz2mi::bwt_wlevel_kernel),
                                                         256, 0) != hipSuccess || occ < 1)
            occ = 4;
        c->wlevel_grid = std::max(8, cus * occ / 8 * 8);
    }
    if ((bz2mi::host::lds_text_path(c->S) && dalloc(&c->d_scratch, c->bwt_slots * bz2mi::bwt_slot_bytes(c->S))) ||
        dalloc(&c->d_lscratch, c->level_slots * bz2mi::bwt_level_slot_bytes(c->S)) ||
        dalloc(&c->d_state, (size_t)c->p * bz2mi::kMaxAlpha) || dalloc(&c->d_sd, 1) || dalloc(&c->d_vol, 4)) {
        bz2mi_destroy(c);
        return nullptr;
    }
    (void)hipMemset(c->d_state, 0, sizeof(uint32_t) * c->p * bz2mi::kMaxAlpha);
    std::vector<uint32_t> crctabs(bz2mi::kCrcTabWords);
    bz2mi::crc_device_tables(crctabs.data());
    if (dalloc(&c->d_crctab, crctabs.size()) ||
        hipMemcpy(c->d_crctab, crctabs.data(), crctabs.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
        bz2mi_destroy(c);
        return nullptr;
    }
    // Batches of about 1.5 GB of block input (BZ2MI_BATCH_BLOCKS overrides),
    // run through the three-stream pipeline when the input is larger.
    // Measured on MI355X, 1 GiB random: one batch 24.6 GB/s, batches of 3000
    // blocks 25.1, 2400 25.3, 2000 24.5, 1000 21.8 (before the staged BWT
    // scatter); after it one batch and batches of 3072 both give 26.0 -- one
    // batch keeps the per-stage event times per launch (the roofline figures).
    c->batch_blocks = std::min(16384, std::max(64, (int)((1536u << 20) / (unsigned)c->S)));
    // the grid doubling's scratch: at most ~52 GB per batch, so a 1 GiB input
    // is one batch at S = 900,000 (1,193 blocks; measured one batch 35.1 GB/s
    // vs two of 666 blocks 33.6), allocated as the batches grow
    // -- and at most half of the HBM free when the context is made (a second
    // context or process on the GPU); compress_device_impl halves the batch
    // further if an allocation still fails
    if (!bz2mi::host::lds_text_path(c->S)) {
        const size_t per = bz2mi::dbl_slot_bytes(c->S) + 16 * (bz2mi::dbl_list_cap(c->S) + bz2mi::dbl_large_cap(c->S));
        size_t budget = (size_t)52e9, fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > 0) budget = std::min(budget, fr / 2);
        c->batch_blocks = std::min(c->batch_blocks, std::max(16, (int)(budget / per)));
    }
    if (const char* e = getenv("BZ2MI_BATCH_BLOCKS")) c->batch_blocks = std::max(1, atoi(e));
    // test hook: the text kernel's work queue limited to this many ring slots,
    // so that a push overruns and the block is handed back to the general path
    if (const char* e = getenv("BZ2MI_DEBUG_WQ_RING")) c->wq_cap = (uint32_t)std::max(1, atoi(e));
    for (auto& e : c->ev) (void)hipEventCreate(&e);
    if (hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess) {
        fail(BZ2MI_EDEVICE, "hipEventCreate failed");
        bz2mi_destroy(c);
        return nullptr;
    }
    return c;
}

void bz2mi_destroy(bz2mi_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (hipStream_t st : {c->stream, c->sA, c->sM, c->sB, c->sF})
        if (st) (void)hipStreamSynchronize(st);
    std::vector<void*> ptrs = {c->d_dscratch, c->d_dlist[0], c->d_dlist[1], c->d_dlarge[0], c->d_dlarge[1], c->d_dctr,
                               c->d_out, c->d_scratch, c->d_sq, c->d_lq[0], c->d_lq[1], c->d_tq[0], c->d_tq[1],
                               c->d_tc, c->d_lscratch, c->d_lspill, c->d_scb, c->d_state, c->d_crctab, c->d_sd, c->d_vol, c->d_ostage, c->d_in,
                               c->d_hout};
    for (int k = 0; k < 2; ++k) {
        if (c->h_pin[k]) (void)hipHostFree(c->h_pin[k]);
        if (c->ev_pin[k]) (void)hipEventDestroy(c->ev_pin[k]);
    }
    for (Batch& t : c->sets) free_batch(t);
    free_front(c->fe);
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->tev)
        if (e) (void)hipEventDestroy(e);
    if (c->own_stream)
        for (hipStream_t st : {c->stream, c->sA, c->sM, c->sB, c->sF})
            if (st) (void)hipStreamDestroy(st);
    delete c;
}

uint64_t bz2mi_blocks_done(const bz2mi_ctx* c) { return c ? c->blocks_done : 0; }

int bz2mi_last_stats(bz2mi_ctx* c, uint64_t* out8) {
    if (!c || !out8) return fail(BZ2MI_EINVAL, "null argument");
    c->want_stats = true;  // later device calls also collect the per-stage volumes
    for (int i = 0; i < 8; ++i) out8[i] = c->stats[i];
    return BZ2MI_OK;
}

int bz2mi_last_timings(bz2mi_ctx* c, float* ms6) {
    if (!c || !ms6) return fail(BZ2MI_EINVAL, "null argument");
    for (int i = 0; i < 6; ++i) ms6[i] = c->last_ms[i];
    return BZ2MI_OK;
}

int bz2mi_compress_blocks(bz2mi_ctx* c, const uint8_t* blocks, size_t stride, const uint32_t* lens,
                          uint32_t nblocks, uint8_t* out, size_t out_stride, uint64_t* out_bits) {
    if (!c || (!blocks && nblocks) || !lens) return fail(BZ2MI_EINVAL, "null argument");
    if (c->finished) return fail(BZ2MI_ESTATE, "Write beyond end of stream");
    if (nblocks == 0) return BZ2MI_OK;
    for (uint32_t j = 0; j < nblocks; ++j)
        if (lens[j] < 1 || lens[j] > (uint32_t)c->S) return fail(BZ2MI_EINVAL, "block length out of range");
    HIPCHECK(hipSetDevice(c->device));
    int r;
    if ((r = ensure_capacity(c, (int)nblocks))) return r;
    HIPCHECK(hipMemcpy2DAsync(c->sets[0].d_blocks, c->stride, blocks, stride, std::min(stride, c->stride), nblocks,
                              hipMemcpyHostToDevice, c->stream));
    HIPCHECK(hipMemcpyAsync(c->sets[0].d_lens, lens, nblocks * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    if ((r = run_blocks(c, (int)nblocks))) return r;
    std::vector<uint64_t> bits(nblocks);
    HIPCHECK(hipMemcpyAsync(bits.data(), c->sets[0].d_pbits, nblocks * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    for (uint32_t j = 0; j < nblocks; ++j) {
        const size_t nbytes = (size_t)((bits[j] + 7) / 8);
        if (nbytes > out_stride) return fail(BZ2MI_ESPACE, "out_stride too small");
        HIPCHECK(hipMemcpy(out + (size_t)j * out_stride, c->sets[0].d_payload + (size_t)j * c->payload_words, nbytes,
                           hipMemcpyDeviceToHost));
        out_bits[j] = bits[j];
    }
    c->blocks_done += nblocks;
    return BZ2MI_OK;
}

int bz2mi_compress_rle1(bz2mi_ctx* c, const uint8_t* blocks, size_t stride, const uint32_t* lens,
                        const uint32_t* crcs, uint32_t nblocks, uint8_t* out, size_t cap, size_t* out_len) {
    if (!c || !out_len || (nblocks && (!blocks || !lens || !crcs))) return fail(BZ2MI_EINVAL, "null argument");
    if (c->finished) return fail(BZ2MI_ESTATE, "Write beyond end of stream");
    *out_len = 0;
    if (nblocks == 0) return BZ2MI_OK;
    for (uint32_t j = 0; j < nblocks; ++j)
        if (lens[j] < 1 || lens[j] > (uint32_t)c->S) return fail(BZ2MI_EINVAL, "block length out of range");
    HIPCHECK(hipSetDevice(c->device));
    int r;
    if ((r = ensure_capacity(c, (int)nblocks))) return r;
    HIPCHECK(hipMemcpy2DAsync(c->sets[0].d_blocks, c->stride, blocks, stride, std::min(stride, c->stride), nblocks,
                              hipMemcpyHostToDevice, c->stream));
    HIPCHECK(hipMemcpyAsync(c->sets[0].d_lens, lens, nblocks * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    HIPCHECK(hipMemcpyAsync(c->sets[0].d_crc, crcs, nblocks * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    if ((r = run_blocks(c, (int)nblocks))) return r;
    if ((r = assemble(c, (int)nblocks, false, out, cap, out_len))) return r;
    for (uint32_t j = 0; j < nblocks; ++j) c->stream_crc = ((c->stream_crc << 1) | (c->stream_crc >> 31)) ^ crcs[j];
    c->blocks_done += nblocks;
    return BZ2MI_OK;
}

int bz2mi_finish(bz2mi_ctx* c, uint8_t* out, size_t cap, size_t* out_len) {
    if (!c || !out_len) return fail(BZ2MI_EINVAL, "null argument");
    if (c->finished) {
        *out_len = 0;
        return BZ2MI_OK;
    }
    HIPCHECK(hipSetDevice(c->device));
    int r;
    if ((r = ensure_capacity(c, 1))) return r;
    if ((r = assemble(c, 0, true, out, cap, out_len))) return r;
    c->finished = true;
    return BZ2MI_OK;
}

// Host bytes in and out (the reference's Memory<T> write / read around
// kernel_close, OutputStream.hpp:83-116): the device buffers are the
// context's and persist across calls (grown when needed), and the copies run
// through two pinned staging buffers of kPinBytes -- the host memcpy of one
// piece overlaps the DMA of the other.
namespace {
constexpr size_t kPinBytes = (size_t)16 << 20;

void free_pinned(bz2mi_ctx* c) {
    for (int k = 0; k < 2; ++k) {
        if (c->h_pin[k]) (void)hipHostFree(c->h_pin[k]);
        if (c->ev_pin[k]) (void)hipEventDestroy(c->ev_pin[k]);
        c->h_pin[k] = nullptr;
        c->ev_pin[k] = nullptr;
    }
}

// all four (two buffers, two events) or none: a partial failure frees what
// was made, so the next call retries instead of using a null buffer/event
int ensure_pinned(bz2mi_ctx* c) {
    if (c->h_pin[0] && c->h_pin[1] && c->ev_pin[0] && c->ev_pin[1]) return BZ2MI_OK;
    free_pinned(c);
    for (int k = 0; k < 2; ++k) {
        if (hipHostMalloc((void**)&c->h_pin[k], kPinBytes, hipHostMallocDefault) != hipSuccess) {
            c->h_pin[k] = nullptr;
            free_pinned(c);
            return fail(BZ2MI_EDEVICE, "hipHostMalloc failed");
        }
        if (hipEventCreateWithFlags(&c->ev_pin[k], hipEventDisableTiming) != hipSuccess) {
            c->ev_pin[k] = nullptr;
            free_pinned(c);
            return fail(BZ2MI_EDEVICE, "hipEventCreate failed");
        }
    }
    return BZ2MI_OK;
}

int copy_in_pinned(bz2mi_ctx* c, uint8_t* d_dst, const uint8_t* in, size_t n) {
    for (size_t off = 0, k = 0; off < n; off += kPinBytes, ++k) {
        const size_t len = std::min(kPinBytes, n - off);
        HIPCHECK(hipEventSynchronize(c->ev_pin[k & 1]));  // the DMA that last read this buffer is done
        memcpy(c->h_pin[k & 1], in + off, len);
        HIPCHECK(hipMemcpyAsync(d_dst + off, c->h_pin[k & 1], len, hipMemcpyHostToDevice, c->stream));
        HIPCHECK(hipEventRecord(c->ev_pin[k & 1], c->stream));
    }
    return BZ2MI_OK;
}

int copy_out_pinned(bz2mi_ctx* c, uint8_t* out, const uint8_t* d_src, size_t n) {
    const size_t np = (n + kPinBytes - 1) / kPinBytes;
    for (size_t k = 0; k <= np; ++k) {
        if (k < np) {  // piece k to pinned buffer k & 1 (its previous piece was copied out below)
            const size_t off = k * kPinBytes, len = std::min(kPinBytes, n - off);
            HIPCHECK(hipMemcpyAsync(c->h_pin[k & 1], d_src + off, len, hipMemcpyDeviceToHost, c->stream));
            HIPCHECK(hipEventRecord(c->ev_pin[k & 1], c->stream));
        }
        if (k >= 1) {  // piece k - 1 to the caller while piece k is in flight
            const size_t q = k - 1, off = q * kPinBytes, len = std::min(kPinBytes, n - off);
            HIPCHECK(hipEventSynchronize(c->ev_pin[q & 1]));
            memcpy(out + off, c->h_pin[q & 1], len);
        }
    }
    return BZ2MI_OK;
}
}  // namespace

int bz2mi_compress(bz2mi_ctx* c, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    if (!c || !out_len || (n && !in)) return fail(BZ2MI_EINVAL, "null argument");
    HIPCHECK(hipSetDevice(c->device));
    int r;
    if (n + 64 > c->in_cap) {
        c->in_cap = 0;
        if ((r = dalloc(&c->d_in, n + 64))) return r;
        c->in_cap = n + 64;
    }
    const size_t dcap = bz2mi_compress_bound(n, c->level, c->unit);
    if (dcap > c->hout_cap) {
        c->hout_cap = 0;
        if ((r = dalloc(&c->d_hout, dcap))) return r;
        c->hout_cap = dcap;
    }
    if ((r = ensure_pinned(c))) return r;
    if ((r = copy_in_pinned(c, c->d_in, in, n))) return r;
    size_t got = 0;
    if ((r = compress_device_impl(c, c->d_in, n, c->d_hout, dcap, &got))) return r;
    if (got > cap) return fail(BZ2MI_ESPACE, "output buffer too small");
    if ((r = copy_out_pinned(c, out, c->d_hout, got))) return r;
    *out_len = got;
    return BZ2MI_OK;
}

int bz2mi_compress_device(bz2mi_ctx* c, const void* d_in, size_t n, void* d_out, size_t cap, size_t* out_len,
                          void* hip_stream) {
    if (!c || !out_len || (n && !d_in) || !d_out) return fail(BZ2MI_EINVAL, "null argument");
    HIPCHECK(hipSetDevice(c->device));
    // inputs written on the caller's stream (NULL: the null stream, where torch
    // writes by default) are complete before the context's streams read them
    HIPCHECK(hipEventRecord(c->ev_in, (hipStream_t)hip_stream));
    HIPCHECK(hipStreamWaitEvent(c->stream, c->ev_in, 0));
    int r = compress_device_impl(c, (const uint8_t*)d_in, n, (uint8_t*)d_out, cap, out_len);
    if (r) return r;
    return BZ2MI_OK;
}

// phase stamps of the representative workgroup of the last launch (builds
// with PHASES=1; returns 0 otherwise): kernel 0 = huffman, 1 = bwt, 2 = mtf,
// 3 = front end, 4 = text BWT sums
int bz2mi_debug_phases(int kernel, unsigned long long* out16) {
    if (!out16) return BZ2MI_EINVAL;
    switch (kernel) {
        case 0: return bz2mi::huffman_phases(out16);
        case 1: return bz2mi::bwt_phases(out16);
        case 2: return bz2mi::mtf_phases(out16);
        case 3: return bz2mi::fe_phases(out16);
        case 4: return bz2mi::tbk_stats(out16);
        case 5: return bz2mi::tbk_resolve_stats(out16);
        case 6: return bz2mi::dbl_stats(out16);
        case 7: return bz2mi::tbk_extra_stats(out16);
        case 8: return bz2mi::blk_phase_stats(out16);
        default: return BZ2MI_EINVAL;
    }
}

// TBK_TRACE builds: the text kernel's waves store their position to this
// host-mapped buffer (16 words per block); returns 0 in other builds
int bz2mi_debug_trace(void* host_mapped) { return bz2mi::tbk_trace(host_mapped); }

// device self-test of the cross-lane primitives: fills bad[0..9] with
// mismatch counts (all zero on a healthy build); returns the number of checks
int bz2mi_debug_selftest(uint32_t* bad, int n) {
    if (!bad || n < 10) return BZ2MI_EINVAL;
    return bz2mi::run_selftest(bad, n);
}

}  // extern "C"
