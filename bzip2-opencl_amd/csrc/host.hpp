// Host-side state of libbz2mi shared by the C-ABI launchers (api.hip: the
// whole-stream and OutputStream entry points; shard.hip: one logical stream
// compressed in units on several devices): the compression context, the
// device buffers of a batch of blocks, the front-end buffers and the stage
// launchers (each enqueues the kernels of one stage on a stream).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/bz2mi.h"
#include "kernels.hpp"

int bz2mi_set_error(int code, const std::string& msg);

namespace bz2mi {
namespace host {

inline int fail(int code, const std::string& msg) { return bz2mi_set_error(code, msg); }
// forget the message of a failure the caller recovered from (a batch halved
// after an allocation failure, a speculation that ran past its halo)
inline void clear_error() { (void)bz2mi_set_error(BZ2MI_OK, std::string()); }

#define HIPCHECK(expr)                                                                                  \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return ::bz2mi::host::fail(BZ2MI_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// BZ2MI_DEBUG_MAX_ALLOC=<bytes> (tests): any larger device allocation fails
// as if HBM were short, to exercise the callers' fallbacks
inline size_t debug_max_alloc() {
    static size_t v = [] {
        const char* e = getenv("BZ2MI_DEBUG_MAX_ALLOC");
        return (e && *e) ? (size_t)strtoull(e, nullptr, 10) : (size_t)0;
    }();
    return v;
}

template <class T>
int dalloc(T** p, size_t count) {
    if (*p) {
        (void)hipFree(*p);
        *p = nullptr;
    }
    if (count == 0) count = 1;
    if (debug_max_alloc() && count * sizeof(T) > debug_max_alloc())
        return fail(BZ2MI_EDEVICE, "hipMalloc: out of memory (BZ2MI_DEBUG_MAX_ALLOC)");
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        return fail(BZ2MI_EDEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    return BZ2MI_OK;
}

// Front-end arrays of one byte stream (frontend.hip K1-K7): the D map, chunk
// summaries and scans (d_ccost: the chunks' context-free costs), the block
// chain and its positions.  Per-byte costs are recomputed where needed.
struct FrontBufs {
    size_t n_cap = 0, maxb = 0;
    uint8_t* d_dmap = nullptr;
    uint32_t* d_lane = nullptr;  // per 64-byte lane: cost prefix | phase << 16
    uint4* d_summ = nullptr;
    uint64_t* d_rsb = nullptr;
    uint32_t* d_ccost = nullptr;
    uint64_t* d_fc = nullptr;
    uint64_t* d_bnd = nullptr;
    uint64_t* d_starts = nullptr;
    uint64_t* d_nb = nullptr;  // [0] blocks, [1] chain status, [2] exit token, [3] speculation merge index
    uint64_t* d_spec = nullptr;  // speculative block starts (bz2mi_unit_speculate)
    uint64_t* d_agg = nullptr;  // scan tile aggregates
    // RLE1 emission segments (frontend.hip FeSeg): table, per-block first
    // entry, total, per-segment emission counts and raw CRCs
    uint8_t* d_seg = nullptr;
    uint32_t* d_segfirst = nullptr;
    uint32_t* d_nseg = nullptr;
    uint32_t* d_segcnt = nullptr;
    uint32_t* d_segcrc = nullptr;
    size_t seg_cap = 0;
    std::vector<void*> ptrs() const {
        return {d_dmap, d_lane, d_summ, d_rsb, d_ccost, d_fc, d_bnd, d_starts, d_nb, d_spec, d_agg,
                d_seg, d_segfirst, d_nseg, d_segcnt, d_segcrc};
    }
};

}  // namespace host
}  // namespace bz2mi

// Device buffers of one batch of blocks (RLE1 input to Huffman payloads).
// The pipelined compress_device keeps kSets of them in flight.
namespace bz2mi {
namespace host {

struct Batch {
    int cap = 0;  // blocks
    uint8_t* d_blocks = nullptr;
    uint32_t* d_lens = nullptr;
    uint32_t* d_crc = nullptr;
    uint8_t* d_bwt = nullptr;
    uint32_t* d_orig = nullptr;
    // BWT (bwt.hip): per-block SA, group lists, counters
    uint32_t* d_sa = nullptr;
    uint32_t* d_bcnt = nullptr;  // [0, 64) small-queue shard counts, [64 + 64 d) level-d queue shard counts,
                                 // [768] blocks with groups, [769] doubling pull
                                 // counter, [8 + d] level-d queue entries
    uint32_t* d_ngroups = nullptr;
    uint32_t* d_p2list = nullptr;
    uint32_t* d_redo = nullptr;  // blocks the SA-free BWT pass hands back
    bz2mi::BwtSeg* d_groups = nullptr;
    // MTF / Huffman
    uint16_t* d_mtf = nullptr;
    uint32_t* d_mtflen = nullptr;
    uint32_t* d_alpha = nullptr;
    uint32_t* d_hist = nullptr;
    uint32_t* d_present = nullptr;
    uint32_t* d_seed = nullptr;
    uint32_t* d_payload = nullptr;
    uint64_t* d_pbits = nullptr;
    uint64_t* d_offs = nullptr;
    // pipeline hand-offs: stage A done, MTF done, buffers free again
    hipEvent_t evA = nullptr, evM = nullptr, evFree = nullptr;

    std::vector<void*> ptrs() const {
        return {d_blocks, d_lens, d_crc, d_bwt, d_orig, d_sa, d_bcnt, d_ngroups, d_p2list, d_redo, d_groups, d_mtf, d_mtflen, d_alpha, d_hist, d_present, d_seed, d_payload,
                d_pbits, d_offs};
    }
};

constexpr int kSets = 3;

}  // namespace host
}  // namespace bz2mi

struct bz2mi_ctx {
    int level = 9, p = 10, unit = 10000, S = 90000, device = 0;
    size_t stride = 0;           // device bytes per block slot
    size_t mtf_stride = 0;       // uint16 per block
    size_t payload_words = 0;    // uint32 per block
    hipStream_t stream = nullptr;  // front end and the host-driven entry points
    hipStream_t sA = nullptr, sM = nullptr, sB = nullptr;  // pipeline: RLE1+CRC+BWT / MTF / Huffman+assembly
    hipStream_t sF = nullptr;  // stream units: front-end scans (ahead of the chains on `stream`)
    bool own_stream = false;
    int cus = 256;
    int bwt_slots = 0;
    int batch_blocks = 0;  // blocks per pipelined batch (0: from the block size)
    uint32_t wq_cap = 0xffffffffu;  // text kernel work-queue slots (BZ2MI_DEBUG_WQ_RING: fewer, tests)
    bool want_stats = false;

    bz2mi::host::Batch sets[bz2mi::host::kSets];
    uint32_t* d_out = nullptr;   // staging for the host-driven assembly
    size_t out_words = 0;
    uint8_t* d_scratch = nullptr;  // BWT workgroup slots (one BWT runs at a time: stream sA)
    uint64_t* d_sq = nullptr;      // BWT small-segment queue (all blocks of a batch)
    bz2mi::BwtItem* d_lq[2] = {nullptr, nullptr};  // BWT level queues (ping-pong)
    uint64_t* d_tq[2] = {nullptr, nullptr};         // BWT per-block tie-group lists (ping-pong)
    uint32_t* d_tc = nullptr;                       // their per-block counts (2 x blocks)
    int small_grid = 0;                             // resident workgroups of bwt_small_kernel
    int level_slots = 0;                            // resident workgroups of bwt_level_kernel
    uint8_t* d_lscratch = nullptr;                  // their scratch slots
    int wlevel_grid = 0;                            // resident workgroups of bwt_wlevel_kernel
    uint32_t* d_lspill = nullptr;                   // wave-level stage spill (one word per rotation of a batch)
    uint32_t* d_scb = nullptr;                      // per-block small-batch counts (LDS-text path)
    // grid-wide prefix doubling (blocks beyond kBwtLdsText): slots, group lists, counters
    uint8_t* d_dscratch = nullptr;
    uint64_t* d_dlist[2] = {nullptr, nullptr};
    uint64_t* d_dlarge[2] = {nullptr, nullptr};
    uint32_t* d_dctr = nullptr;
    int bwtq_blocks = 0;           // capacity of the queues in blocks
    uint32_t* d_state = nullptr;   // p x 258 persistent seed sums (H4)
    uint32_t* d_crctab = nullptr;
    bz2mi::StreamDev* d_sd = nullptr;
    unsigned long long* d_vol = nullptr;  // [3] volumes of the last compress_device call
    bz2mi::StreamDev h_sd{};
    uint8_t* d_ostage = nullptr;   // aligned output staging for unaligned destinations
    size_t ostage_cap = 0;
    // front end of the whole-stream path (device RLE1)
    bz2mi::host::FrontBufs fe;
    uint8_t* d_in = nullptr;        // staging for host input
    size_t in_cap = 0;
    // bz2mi_compress (host bytes): the stream in HBM, kept across calls, and
    // two pinned staging buffers the copies are pipelined through
    uint8_t* d_hout = nullptr;
    size_t hout_cap = 0;
    uint8_t* h_pin[2] = {nullptr, nullptr};
    hipEvent_t ev_pin[2] = {nullptr, nullptr};
    hipEvent_t ev[8] = {};
    hipEvent_t ev_in = nullptr;  // caller stream -> context stream hand-off
    std::vector<hipEvent_t> tev;  // per-batch stage timing events (12 per batch)
    float last_ms[6] = {0, 0, 0, 0, 0, 0};
    uint64_t stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};

    // stream state of the host-driven path (OutputStream.hpp:39-44)
    uint64_t blocks_done = 0;
    uint32_t stream_crc = 0;
    uint64_t carry = 0;      // MSB-aligned pending bits
    int carry_bits = 0;
    bool header_done = false;
    bool finished = false;

    std::vector<uint8_t> h_stage;
};

namespace bz2mi {
namespace host {

int ensure_front(FrontBufs& f, int S, size_t n);
void free_front(FrontBufs& f);
// K1-K5 (summaries, run scan, costs, cost scan, D map) of n bytes at d_x
int enqueue_front_scan(FrontBufs& f, const uint8_t* d_x, size_t n, hipStream_t s);
// K6-K7: the chain of the unit [0, n_own) of d_x[0, n) from `entry`; *nb_out
// (host) = blocks, *exit_out = the next unit's entry.  Synchronous on s.
// With a speculation (spec: f.d_spec[0, spec_nb] = block starts and end of the
// chain from byte 0, spec_exit its exit token) the chain stops where it meets
// a speculative block start and the speculative tail is spliced on
// (*spliced = blocks taken from it).
int run_chain(bz2mi_ctx* c, FrontBufs& f, const uint8_t* d_x, size_t n, size_t n_own, uint64_t entry, bool ends,
              uint64_t* nb_out, uint64_t* exit_out, hipStream_t s, uint64_t spec_nb = 0, uint64_t spec_exit = 0,
              uint64_t* spliced = nullptr);
int ensure_batch(bz2mi_ctx* c, Batch& t, int nblocks);
void free_batch(Batch& t);
int stage_front(bz2mi_ctx* c, Batch& t, const FrontBufs& f, const uint8_t* d_x, size_t n, uint64_t first,
                uint64_t cnt, hipStream_t s);
bool lds_text_path(int S);
int ensure_bwt_scratch(bz2mi_ctx* c, int nb);
void free_bwt_scratch(bz2mi_ctx* c);
int stage_bwt(bz2mi_ctx* c, Batch& t, int nb, hipStream_t s);
int stage_mtf(bz2mi_ctx* c, Batch& t, int nb, hipStream_t s);
int stage_seed(bz2mi_ctx* c, Batch& t, int nb, uint64_t first_block, uint32_t* state, hipStream_t s);
int stage_huffman(bz2mi_ctx* c, Batch& t, int nb, hipStream_t s);

}  // namespace host
}  // namespace bz2mi
