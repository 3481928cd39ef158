// C-ABI of the device decoder (include/bz2mi.h, bz2mi_d*): buffers, the kernel
// sequence of decode.hip and the host-side walk of the stream structure
// (InputStream::initializeStream / initializeNextBlock, InputStream.hpp:96-158).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bz2mi.h"
#include "decode.hpp"
#include "rle1.hpp"

int bz2mi_set_error(int code, const std::string& msg);

namespace {

#define DCHECK(expr)                                                                                 \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            return bz2mi_set_error(BZ2MI_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

const char* dec_message(uint32_t status) {
    switch (status) {
        case bz2mi::kDecTables: return "block Huffman tables invalid";
        case bz2mi::kDecData: return "Error decoding  block";
        case bz2mi::kDecSize: return "BZip2 block exceeds declared block size";
        case bz2mi::kDecOrigPtr: return "BZip2 start pointer invalid";
        case bz2mi::kDecRandomised: return "BZip2 randomised blocks not implemented";
        default: return "BZip2 stream format error";
    }
}

// set by grow() when the device was out of memory: run_decode retries the
// window with smaller budgets
thread_local bool g_dec_oom = false;

template <class T>
int grow(T** p, size_t* cap, size_t count) {
    if (count <= *cap && *p) return BZ2MI_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t c = std::max<size_t>(count, 1);
    hipError_t e = hipMalloc((void**)p, c * sizeof(T));
    if (e != hipSuccess) {
        if (e == hipErrorOutOfMemory) {
            g_dec_oom = true;
            (void)hipGetLastError();  // not sticky: the retry may allocate less
        }
        return bz2mi_set_error(BZ2MI_EDEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    *cap = c;
    return BZ2MI_OK;
}

}  // namespace

// The stream structure walked so far (InputStream::initializeStream /
// initializeNextBlock, InputStream.hpp:96-158), carried from one window of
// the input to the next.
struct DecWalk {
    bool started = false;    // a stream header was read
    bool in_stream = false;  // inside a stream (its header read, its end marker not yet)
    bool finished = false;   // no more streams are decoded
    uint32_t S = 0;          // block size limit of the current stream
    uint32_t scrc = 0;       // stream CRC of the blocks so far
};

struct bz2mi_dctx {
    int unit = 10000, device = 0, cus = 256;
    uint64_t trailing = 0;  // input bytes after the last decoded stream (ignored)
    int flags = 0;  // BZ2MI_DEC_CONCATENATED: every stream of the input (bzip2), else the first (reference)
    hipStream_t stream = nullptr;
    uint32_t* d_crctab = nullptr;
    uint32_t* d_cnt = nullptr;
    bz2mi::DecCand* d_cand = nullptr;
    size_t cand_cap = 0;
    uint32_t* d_ids = nullptr;
    size_t ids_cap = 0;
    uint8_t* d_bwt = nullptr;
    size_t bwt_cap = 0;
    uint16_t* d_syms = nullptr;
    size_t syms_cap = 0;
    uint8_t* d_symmap = nullptr;
    size_t symmap_cap = 0;
    uint8_t* d_tabs = nullptr;
    size_t tabs_cap = 0;
    bz2mi::DecBlockInfo* d_info = nullptr;
    size_t info_cap = 0;
    uint32_t* d_blocks = nullptr;
    size_t blocks_cap = 0;
    uint32_t* d_merged = nullptr;
    size_t merged_cap = 0;
    uint32_t* d_marks = nullptr;
    size_t marks_cap = 0;
    uint8_t* d_iscr = nullptr;  // inverse-BWT walker bytes (kDecIbwtScratch per workgroup of its grid)
    size_t iscr_cap = 0;
    uint8_t* d_rle1 = nullptr;
    size_t rle1_cap = 0;
    uint32_t* d_cstate = nullptr;
    size_t cstate_cap = 0;
    uint64_t* d_olen = nullptr;
    size_t olen_cap = 0;
    uint64_t* d_ooff = nullptr;
    size_t ooff_cap = 0;
    uint32_t* d_crc = nullptr;
    size_t crc_cap = 0;
    uint32_t* d_bad = nullptr;
    size_t bad_cap = 0;
    uint8_t* d_in = nullptr;  // staging (host input / unaligned device input)
    size_t in_cap = 0;
    uint8_t* d_out = nullptr;  // staging for host output
    size_t out_cap = 0;
    hipEvent_t ev[6] = {};
    hipEvent_t ev_in = nullptr;  // null stream -> decoder stream hand-off
    float ms[6] = {0, 0, 0, 0, 0, 0};
    DecWalk walk;              // stream structure across windows
    int pending = BZ2MI_OK;    // streaming: an error found after the bytes returned
    std::string pending_msg;
};

namespace {

// inverse-BWT workgroups per XCD (A/B builds: -DBZ2MI_AB_IBWT_XCD=n)
#ifndef BZ2MI_AB_IBWT_XCD
#define BZ2MI_AB_IBWT_XCD 32  // measured 8/16/24/32: 101/64/55/58 ms per GiB random, 100/59/45/42 text
#endif
constexpr int ibwt_wg_per_xcd() { return BZ2MI_AB_IBWT_XCD; }

// an element of the stream in order: a header, a block, an end marker
struct DecEvent {
    enum : uint32_t { kStart, kBlock, kEnd } type;
    uint32_t k;     // kBlock: decoded-candidate id
    uint32_t val;   // kStart: block size limit; kBlock / kEnd: stored CRC
    uint64_t pos;   // window bit where it starts
    uint64_t next;  // window bit after it
};

struct WinResult {
    uint64_t end_bit = 0;  // window bit where the next call starts
    size_t out_len = 0;    // bytes written (or needed, count mode)
    bool done = false;     // the streams have ended
    int err = BZ2MI_OK;    // an error after the bytes written (streaming: reported by the next call)
    std::string msg;
};

// the longest a block's bits can be at block size limit S: header, symbol
// map, selectors (unary, <= 6 bits), delta-coded tables (<= 5 + 42 bits per
// symbol), <= S + 2 symbols of <= 20 bits
uint64_t max_header_bits(uint32_t S) {
    return 32 + 48 + 1 + 24 + 16 + 256 + 3 + 15 + 7ull * (S / 50 + 2) + 6ull * (5 + 258ull * 42);
}
uint64_t max_block_bits(uint32_t S) { return max_header_bits(S) + 20ull * (S + 2); }

// Device bytes of a block candidate's tables (K2a) and of a candidate with
// valid tables (symbols, and the per-block stages' vectors when it is on the
// chain): a window's candidate counts are memory budgets over these.
size_t table_bytes() { return bz2mi::kTabBytes + 256 + sizeof(bz2mi::DecBlockInfo) + 8; }
size_t symbol_bytes(int unit) {
    const size_t smax = (size_t)9 * unit;
    const size_t stride = (smax + 255) & ~(size_t)255, sym_stride = (smax + 2 + 63) & ~(size_t)63;
    return 2 * sym_stride + stride                                 // symbols, BWT row
           + 4 * std::max(stride, sym_stride) + 4 * stride + stride  // merged, marks, RLE1 row
           + 256 * 4 + 64;                                         // chunk states, sizes
}

// One window of the input: the blocks of d_in[0, n) from window bit `start`,
// the tables of at most `kmax_c` block candidates and the symbols of at most
// `kmax_s` of them decoded, at most `cap` output bytes
// (cap == SIZE_MAX with d_out == nullptr: count mode, sizes only).  `final`:
// no input follows the window (a block cut by its end is an error, not a
// reason to stop).  Walk state in d->walk; errors in stream order.
int run_window(bz2mi_dctx* d, const uint8_t* d_in, size_t n, uint64_t start, bool final, size_t kmax_c,
               size_t kmax_s, uint8_t* d_out, size_t cap, WinResult* res, hipStream_t s) {
    using namespace bz2mi;
    int r;
    DecWalk& W = d->walk;
    *res = WinResult{};
    res->end_bit = start;
    if (W.finished) {
        res->done = true;
        return BZ2MI_OK;
    }
    const bool count_only = d_out == nullptr;
    DCHECK(hipEventRecord(d->ev[0], s));
    // ---- K1: candidates in the window (one per 16 input bytes at most: a
    // window with more magic matches -- crafted input -- is shortened until
    // its matches fit, and decides only what its shorter range can)
    const size_t cap_c = n / 16 + 65536;
    if ((r = grow(&d->d_cand, &d->cand_cap, cap_c))) return r;
    uint32_t ncand = 0;
    for (;;) {
        DCHECK(hipMemsetAsync(d->d_cnt, 0, 4 * sizeof(uint32_t), s));
        if (n) {
            const uint64_t words = (n + 7) / 8;
            hipLaunchKernelGGL(dec_scan_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, d_in,
                               (uint64_t)n, d->d_cand, d->d_cnt, (uint32_t)d->cand_cap);
            DCHECK(hipGetLastError());
        }
        DCHECK(hipMemcpyAsync(&ncand, d->d_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        DCHECK(hipStreamSynchronize(s));
        if (ncand <= d->cand_cap) break;
        const size_t shorter = (size_t)((double)n * d->cand_cap / ncand / 2) & ~(size_t)7;
        if (shorter * 8 <= start + 80) return bz2mi_set_error(BZ2MI_EFORMAT, "BZip2 stream format error");
        n = shorter;
        final = false;
    }
    const uint64_t nbits = (uint64_t)n * 8;
    DCHECK(hipEventRecord(d->ev[1], s));
    std::vector<DecCand> cand(ncand);
    if (ncand) DCHECK(hipMemcpy(cand.data(), d->d_cand, ncand * sizeof(DecCand), hipMemcpyDeviceToHost));
    cand.erase(std::remove_if(cand.begin(), cand.end(), [&](const DecCand& c) { return c.bitpos < start; }),
               cand.end());
    std::sort(cand.begin(), cand.end(), [](const DecCand& a, const DecCand& b) { return a.bitpos < b.bitpos; });
    ncand = (uint32_t)cand.size();
    if (ncand) DCHECK(hipMemcpy(d->d_cand, cand.data(), ncand * sizeof(DecCand), hipMemcpyHostToDevice));
    // ---- K2a: headers and tables of the first kmax_c block candidates; K2b:
    // the symbols of the first kmax_s of them whose tables are valid (memory
    // bounded whatever the number of magic matches)
    std::vector<uint32_t> ids;
    std::vector<int64_t> id_of(ncand, -1);
    for (uint32_t i = 0; i < ncand && ids.size() < kmax_c; ++i)
        if (cand[i].type == 0) {
            id_of[i] = (int64_t)ids.size();
            ids.push_back(i);
        }
    const uint32_t smax = (uint32_t)(9 * d->unit);
    const uint32_t max_sel = d->unit == 10000 ? (uint32_t)(smax / 50 + 1) : (uint32_t)(smax / 50 + 2);
    const size_t stride = ((size_t)smax + 255) & ~(size_t)255;
    const size_t sym_stride = ((size_t)smax + 2 + 63) & ~(size_t)63;
    const size_t nk = ids.size();
    if ((r = grow(&d->d_ids, &d->ids_cap, 2 * nk))) return r;
    if ((r = grow(&d->d_symmap, &d->symmap_cap, nk * 256))) return r;
    if ((r = grow(&d->d_tabs, &d->tabs_cap, nk * kTabBytes))) return r;
    if ((r = grow(&d->d_info, &d->info_cap, nk))) return r;
    std::vector<DecBlockInfo> info(nk);
    std::vector<uint32_t> row(nk, 0xffffffffu);  // candidate -> symbol row
    std::vector<uint32_t> sel;                    // symbol row -> candidate
    if (nk) {
        DCHECK(hipMemcpyAsync(d->d_ids, ids.data(), nk * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(dec_huff_kernel, dim3((unsigned)nk), dim3(64), (max_sel + 7) / 8 * 4, s, d_in, (uint64_t)n,
                           d->d_cand, d->d_ids, (uint32_t)nk, max_sel, d->d_tabs, d->d_symmap, d->d_info);
        DCHECK(hipGetLastError());
        DCHECK(hipMemcpyAsync(info.data(), d->d_info, nk * sizeof(DecBlockInfo), hipMemcpyDeviceToHost, s));
        DCHECK(hipStreamSynchronize(s));
        for (uint32_t k = 0; k < nk && sel.size() < kmax_s; ++k)
            if (info[k].status == 0) {
                row[k] = (uint32_t)sel.size();
                sel.push_back(k);
            }
        if (!sel.empty()) {
            if ((r = grow(&d->d_syms, &d->syms_cap, sel.size() * sym_stride))) return r;
            DCHECK(hipMemcpyAsync(d->d_ids + nk, sel.data(), sel.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
#if BZ2MI_SYM_WINDOW
            hipLaunchKernelGGL(dec_symw_kernel, dim3((unsigned)sel.size()), dim3(64), 0, s, d_in, (uint64_t)n,
                               d->d_tabs, d->d_ids + nk, (uint32_t)sel.size(), smax, d->d_syms, sym_stride, d->d_info);
#else
            hipLaunchKernelGGL(dec_sym_kernel, dim3((unsigned)((sel.size() + kDecSymBlocks - 1) / kDecSymBlocks)),
                               dim3(64), 0, s, d_in, (uint64_t)n, d->d_tabs, d->d_ids + nk, (uint32_t)sel.size(), smax,
                               d->d_syms, sym_stride, d->d_info);
#endif
            DCHECK(hipGetLastError());
            DCHECK(hipMemcpyAsync(info.data(), d->d_info, nk * sizeof(DecBlockInfo), hipMemcpyDeviceToHost, s));
        }
    }
    DCHECK(hipEventRecord(d->ev[2], s));
    DCHECK(hipStreamSynchronize(s));
    // ---- the stream structure (InputStream.hpp:96-158) over the candidates:
    // events in stream order, up to the first error or the end of what this
    // window can decide
    auto find = [&](uint64_t bit) -> int64_t {
        auto it = std::lower_bound(cand.begin(), cand.end(), bit,
                                   [](const DecCand& c, uint64_t b) { return c.bitpos < b; });
        return (it != cand.end() && it->bitpos == bit) ? (int64_t)(it - cand.begin()) : -1;
    };
    std::vector<uint8_t> hdr(4);
    auto header_at = [&](uint64_t byte, int* digit) -> int {
        if (hipMemcpy(hdr.data(), d_in + byte, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        if (hdr[0] != 'B' || hdr[1] != 'Z' || hdr[2] != 'h' || hdr[3] < '1' || hdr[3] > '9') return 0;
        *digit = hdr[3] - '0';
        return 1;
    };
    std::vector<DecEvent> ev;
    int err_status = -1;  // a structural / decode error at the end of the events
    std::string err_msg;
    bool walk_done = false;
    {
        bool started = W.started, in_stream = W.in_stream;
        uint32_t S = W.S;
        uint64_t pos = start;
        for (;;) {
            if (!in_stream) {
                // the reference's InputStream ends at the first end-of-stream
                // marker (InputStream.hpp:136-143); bzip2 goes on to the next stream
                if (started && !(d->flags & BZ2MI_DEC_CONCATENATED)) {
                    walk_done = true;
                    break;
                }
                const uint64_t byte = (pos + 7) / 8;
                int digit = 0;
                const int h = byte + 4 <= n ? header_at(byte, &digit) : 2;
                if (h < 0) return bz2mi_set_error(BZ2MI_EDEVICE, "hipMemcpy (stream header)");
                if (h == 2 && !final) break;  // the next header is not in the window yet
                if (h != 1) {
                    if (!started) {
                        err_status = 0;
                        err_msg = (h == 2 && n == 0 && start == 0) ? "Insufficient data" : "Invalid BZip2 header";
                    } else {
                        walk_done = true;  // bytes after the last stream that start no header: ignored
                    }
                    break;
                }
                S = (uint32_t)(digit * d->unit);
                ev.push_back(DecEvent{DecEvent::kStart, 0, S, pos, byte * 8 + 32});
                pos = byte * 8 + 32;
                started = in_stream = true;
            }
            const int64_t ci = find(pos);
            if (ci < 0) {
                if (!final && pos + 80 > nbits) break;  // the magic is not in the window yet
                err_status = 0;
                err_msg = pos + 48 > nbits ? "Insufficient data" : "BZip2 stream format error";
                break;
            }
            if (cand[ci].type == 1) {
                if (pos + 80 > nbits) {
                    if (!final) break;
                    err_status = 0;
                    err_msg = "Insufficient data";
                    break;
                }
                ev.push_back(DecEvent{DecEvent::kEnd, 0, cand[ci].next32, pos, pos + 80});
                pos += 80;
                in_stream = false;
                continue;
            }
            if (id_of[ci] < 0) break;  // beyond this window's candidates: the next call
            const uint32_t k = (uint32_t)id_of[ci];
            if (info[k].status == 0 && row[k] == 0xffffffffu) break;  // beyond the symbol rows: the next call
            // a failure that the window's end may have caused waits for more
            // input: a header / table failure within a header's length of the
            // end, a data failure within a block's length
            if (!final) {
                const uint64_t room = nbits - pos;
                const bool data_fail = info[k].status == kDecData || (!info[k].status && info[k].end_bit > nbits);
                if (data_fail && room < max_block_bits(S)) break;
                if (info[k].status && !data_fail && room < max_header_bits(S)) break;
            }
            if (info[k].status) {
                err_status = (int)info[k].status;
                err_msg = dec_message(info[k].status);
                break;
            }
            if (info[k].end_bit > nbits) {
                err_status = 0;
                err_msg = "Insufficient data";
                break;
            }
            ev.push_back(DecEvent{DecEvent::kBlock, k, info[k].crc, pos, info[k].end_bit});
            pos = info[k].end_bit;
        }
        res->end_bit = pos;  // (moved back below if events are cut)
    }
    std::vector<uint32_t> chain;  // decoded-candidate ids of the blocks, stream order
    std::vector<size_t> chain_ev;  // their event indices
    std::vector<uint32_t> chain_S;
    {
        uint32_t S = W.S;
        for (size_t i = 0; i < ev.size(); ++i) {
            if (ev[i].type == DecEvent::kStart) S = ev[i].val;
            if (ev[i].type == DecEvent::kBlock) {
                chain.push_back(ev[i].k);
                chain_ev.push_back(i);
                chain_S.push_back(S);
            }
        }
    }
    size_t keep_ev = ev.size();  // events applied by this call
    auto cut_at_block = [&](size_t i) {  // events from chain block i on are dropped
        keep_ev = chain_ev[i];
        chain.resize(i);
        chain_ev.resize(i);
        chain_S.resize(i);
    };
    // ---- K2b (MTF / RLE2) over the blocks of the chain; its errors (block
    // size, origPtr) end the chain at the first failing block
    if (!chain.empty()) {
        const size_t nc = chain.size();
        if ((r = grow(&d->d_blocks, &d->blocks_cap, 2 * nc))) return r;
        if ((r = grow(&d->d_bwt, &d->bwt_cap, nc * stride))) return r;
        // d_merged (the inverse BWT's vector, free until then) is the scratch
        if ((r = grow(&d->d_merged, &d->merged_cap, nc * sym_stride))) return r;
        std::vector<uint32_t> rows(nc);
        for (size_t i = 0; i < nc; ++i) rows[i] = row[chain[i]];
        DCHECK(hipMemcpyAsync(d->d_blocks, chain.data(), nc * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        DCHECK(hipMemcpyAsync(d->d_blocks + nc, rows.data(), nc * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(dec_mtf_kernel, dim3((unsigned)nc), dim3(kDecMtfThreads), 0, s, d->d_syms, sym_stride, d->d_symmap,
                           d->d_blocks, d->d_blocks + nc, (uint32_t)nc, smax, d->d_merged, sym_stride, d->d_bwt,
                           stride, d->d_info);
        DCHECK(hipGetLastError());
        DCHECK(hipMemcpyAsync(info.data(), d->d_info, nk * sizeof(DecBlockInfo), hipMemcpyDeviceToHost, s));
        DCHECK(hipStreamSynchronize(s));
        for (size_t i = 0; i < chain.size(); ++i) {
            const DecBlockInfo& bi = info[chain[i]];
            const uint32_t st = bi.status ? bi.status : (bi.len > chain_S[i] ? (uint32_t)kDecSize : 0u);
            if (st) {
                err_status = (int)st;
                err_msg = dec_message(st);
                cut_at_block(i);
                break;
            }
        }
    }
    DCHECK(hipEventRecord(d->ev[3], s));
    // ---- K3 / K4 over the blocks of the chain
    size_t nb = chain.size();
    std::vector<uint64_t> olen(nb), ooff(nb + 1, 0);
    std::vector<uint32_t> crc(nb), bad(nb, 0);
    bool cut_by_cap = false;
    if (nb) {
        if ((r = grow(&d->d_blocks, &d->blocks_cap, nb))) return r;
        if ((r = grow(&d->d_merged, &d->merged_cap, std::max(nb * stride, nb * sym_stride)))) return r;
        if ((r = grow(&d->d_marks, &d->marks_cap, nb * stride))) return r;
        const size_t ibwt_grid = std::min<size_t>(nb, (size_t)8 * ibwt_wg_per_xcd());
        if ((r = grow(&d->d_iscr, &d->iscr_cap, ibwt_grid * kDecIbwtScratch))) return r;
        if ((r = grow(&d->d_rle1, &d->rle1_cap, nb * stride))) return r;
        if ((r = grow(&d->d_cstate, &d->cstate_cap, nb * 256))) return r;
        if ((r = grow(&d->d_olen, &d->olen_cap, nb))) return r;
        if ((r = grow(&d->d_ooff, &d->ooff_cap, nb))) return r;
        if ((r = grow(&d->d_crc, &d->crc_cap, nb))) return r;
        if ((r = grow(&d->d_bad, &d->bad_cap, nb))) return r;
        DCHECK(hipMemsetAsync(d->d_bad, 0, nb * sizeof(uint32_t), s));
        DCHECK(hipMemcpyAsync(d->d_blocks, chain.data(), nb * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(dec_ibwt_kernel, dim3((unsigned)ibwt_grid), dim3(kDecIbwtThreads), 0, s, d->d_bwt, stride,
                           d->d_info, d->d_blocks, (uint32_t)nb, d->d_merged, stride, d->d_marks, stride, d->d_rle1,
                           stride, d->d_bad, d->d_iscr);
        DCHECK(hipGetLastError());
        DCHECK(hipEventRecord(d->ev[4], s));
        hipLaunchKernelGGL(dec_rle1_kernel, dim3((unsigned)nb), dim3(256), 0, s, d->d_rle1, stride, d->d_info,
                           d->d_blocks, (uint32_t)nb, d->d_cstate, d->d_olen, (const uint64_t*)nullptr,
                           (uint8_t*)nullptr, (uint64_t)0, d->d_crc, d->d_crctab, 0);
        DCHECK(hipGetLastError());
        DCHECK(hipMemcpyAsync(olen.data(), d->d_olen, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        DCHECK(hipStreamSynchronize(s));
        for (size_t i = 0; i < nb; ++i) ooff[i + 1] = ooff[i] + olen[i];
        if (!count_only && ooff[nb] > cap) {
            // the blocks that fit; the rest waits for the next call
            size_t fit = 0;
            while (fit < nb && ooff[fit + 1] <= cap) fit++;
            if (fit == 0) {
                res->out_len = olen[0];
                return bz2mi_set_error(BZ2MI_ESPACE, "output buffer too small");
            }
            cut_at_block(fit);
            nb = fit;
            cut_by_cap = true;
        }
        if (!count_only) {
            DCHECK(hipMemcpyAsync(d->d_ooff, ooff.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(dec_rle1_kernel, dim3((unsigned)nb), dim3(256), 0, s, d->d_rle1, stride, d->d_info,
                               d->d_blocks, (uint32_t)nb, d->d_cstate, d->d_olen, d->d_ooff, d_out, (uint64_t)cap,
                               d->d_crc, d->d_crctab, 1);
            DCHECK(hipGetLastError());
        }
        DCHECK(hipMemcpyAsync(crc.data(), d->d_crc, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        DCHECK(hipMemcpyAsync(bad.data(), d->d_bad, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    } else {
        DCHECK(hipEventRecord(d->ev[4], s));
    }
    DCHECK(hipEventRecord(d->ev[5], s));
    DCHECK(hipStreamSynchronize(s));
    if (cut_by_cap) {
        err_status = -1;  // an error after the cut is the next call's
        walk_done = false;
    }
    // ---- the events in stream order: block CRCs (BlockDecompressor::checkCRC
    // :101-109), stream CRCs (InputStream.hpp:136-143), then the first error
    // the walk stopped at; the bytes of the blocks before a failing one count
    size_t bi = 0;
    uint64_t at = start;
    for (size_t i = 0; i < keep_ev; ++i) {
        const DecEvent& e = ev[i];
        if (e.type == DecEvent::kStart) {
            W.started = W.in_stream = true;
            W.S = e.val;
            W.scrc = 0;
        } else if (e.type == DecEvent::kBlock) {
            // (an inconsistent BWT -- `bad` -- yields garbage bytes: the reference
            // would find the same CRC mismatch)
            // (count mode writes nothing and computes no CRCs: sizes only)
            if (!count_only && (bad[bi] || crc[bi] != e.val)) {
                res->end_bit = e.pos;
                res->out_len = ooff[bi];
                res->err = BZ2MI_EFORMAT;
                res->msg = "BZip2 block CRC error";
                return BZ2MI_OK;
            }
            W.scrc = ((W.scrc << 1) | (W.scrc >> 31)) ^ crc[bi];
            bi++;
        } else {
            if (!count_only && W.scrc != e.val) {
                res->end_bit = e.pos;
                res->out_len = ooff[bi];
                res->err = BZ2MI_EFORMAT;
                res->msg = "BZip2 stream CRC error";
                return BZ2MI_OK;
            }
            W.in_stream = false;
            W.scrc = 0;
        }
        at = e.next;
    }
    res->out_len = ooff[bi];
    if (keep_ev < ev.size()) res->end_bit = at;
    if (err_status >= 0) {
        res->err = BZ2MI_EFORMAT;
        res->msg = err_msg;
    }
    if (walk_done) {
        W.finished = true;
        res->done = true;
    }
    float t;
    for (int k = 0; k < 5; ++k) d->ms[k] += hipEventElapsedTime(&t, d->ev[k], d->ev[k + 1]) == hipSuccess ? t : 0.f;
    d->ms[5] += hipEventElapsedTime(&t, d->ev[0], d->ev[5]) == hipSuccess ? t : 0.f;
    return BZ2MI_OK;
}

// Candidates one window may decode: symbols for max(64 x input, 1 GiB) of
// memory (a legitimate stream is one window: a block's symbols and stage
// vectors are ~12 bytes per decoded byte), capped at half the device's free
// memory and kDecBudgetMax so the budget bounds memory whatever the input
// size (a larger stream is decoded in several windows; BZ2MI_DEC_BUDGET sets
// the budget), tables for as many candidates or 2 x the input, whichever is
// more (a crafted input of magic matches everywhere costs tables for that
// many, not per match).
constexpr size_t kDecBudgetMax = (size_t)32 << 30;
void window_kmax(const bz2mi_dctx* d, size_t n, size_t* kmax_c, size_t* kmax_s) {
    size_t budget = std::max<size_t>((size_t)64 * n, (size_t)1 << 30);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr) budget = std::min(budget, fr / 2);
    budget = std::min(budget, kDecBudgetMax);
    if (const char* e = getenv("BZ2MI_DEC_BUDGET")) budget = (size_t)strtoull(e, nullptr, 10);
    *kmax_s = std::max<size_t>(64, budget / symbol_bytes(d->unit));
    *kmax_c = std::max<size_t>(*kmax_s, std::min<size_t>(2 * n, budget) / table_bytes());
}

// the whole decode of n bytes at d_in (4-byte aligned) into d_out: windows
// from the walk's position on until the streams end
int run_decode(bz2mi_dctx* d, const uint8_t* d_in, size_t n, uint8_t* d_out, size_t cap, size_t* out_len,
               hipStream_t s) {
    *out_len = 0;
    d->walk = DecWalk{};
    d->trailing = 0;
    for (float& m : d->ms) m = 0.f;
    size_t kmax_c, kmax_s;
    window_kmax(d, n, &kmax_c, &kmax_s);
    uint64_t bit = 0;
    size_t total = 0;
    bool counting = false;  // the output did not fit: sizes only, for *out_len
    for (;;) {
        const size_t byte = (size_t)(bit / 8);
        // (windows start on 4-byte boundaries: the bit reader loads aligned words)
        const size_t wb = byte & ~(size_t)3;
        WinResult res;
        int r = run_window(d, d_in + wb, n - wb, bit - (uint64_t)wb * 8, true, kmax_c, kmax_s,
                           counting ? nullptr : d_out + total,
                           counting ? SIZE_MAX : cap - total, &res, s);
        if (r == BZ2MI_ESPACE && !counting) {
            counting = true;
            continue;  // (the walk state is unchanged by a call that fails this way)
        }
        if (r == BZ2MI_EDEVICE && g_dec_oom && kmax_s > 64) {
            // out of device memory while sizing this window's buffers (before
            // the walk moves): the same window again with half the budgets
            g_dec_oom = false;
            kmax_s = std::max<size_t>(64, kmax_s / 2);
            kmax_c = std::max<size_t>(kmax_s, kmax_c / 2);
            continue;
        }
        g_dec_oom = false;
        if (r != BZ2MI_OK) return r;
        total += res.out_len;
        if (res.err != BZ2MI_OK) return bz2mi_set_error(res.err, res.msg);
        const uint64_t next = (uint64_t)wb * 8 + res.end_bit;
        if (res.done) {
            d->trailing = n - std::min<uint64_t>(n, (next + 7) / 8);
            break;
        }
        if (next == bit && res.out_len == 0) return bz2mi_set_error(BZ2MI_EFORMAT, "BZip2 stream format error");
        bit = next;
    }
    if (counting) {
        *out_len = total;
        return bz2mi_set_error(BZ2MI_ESPACE, "output buffer too small");
    }
    *out_len = total;
    return BZ2MI_OK;
}

}  // namespace

extern "C" {

bz2mi_dctx* bz2mi_dcreate(int unit, int device) {
    if (unit != 10000 && unit != 100000) {
        bz2mi_set_error(BZ2MI_EINVAL, "Invalid block size unit");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        bz2mi_set_error(BZ2MI_EDEVICE, "no HIP device (bz2mi has no CPU fallback)");
        return nullptr;
    }
    if (device < 0 || device >= ndev || hipSetDevice(device) != hipSuccess) {
        bz2mi_set_error(BZ2MI_EINVAL, "invalid device");
        return nullptr;
    }
    bz2mi_dctx* d = new bz2mi_dctx();
    d->unit = unit;
    d->device = device;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess) d->cus = prop.multiProcessorCount;
    }
    bool ok = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc((void**)&d->d_crctab, 256 * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc((void**)&d->d_cnt, 4 * sizeof(uint32_t)) == hipSuccess &&
              hipMemcpy(d->d_crctab, bz2mi::kCrc.t.data(), 256 * sizeof(uint32_t), hipMemcpyHostToDevice) ==
                  hipSuccess;
    for (auto& e : d->ev) ok = ok && hipEventCreate(&e) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&d->ev_in, hipEventDisableTiming) == hipSuccess;
    // x^(8 * 2^k) mod P for the CRC combination
    uint32_t xp[64];
    {
        auto mulmod = [](uint32_t a, uint32_t b) {
            uint32_t r = 0;
            for (int i = 31; i >= 0; --i) {
                r = (r << 1) ^ ((r >> 31) ? 0x04c11db7u : 0u);
                if ((b >> i) & 1u) r ^= a;
            }
            return r;
        };
        xp[0] = 0x100u;  // x^8
        for (int k = 1; k < 64; ++k) xp[k] = mulmod(xp[k - 1], xp[k - 1]);
    }
    ok = ok && bz2mi::dec_set_xpow8(xp) == 0;
    if (!ok) {
        bz2mi_set_error(BZ2MI_EDEVICE, "bz2mi_dcreate: HIP allocation failed");
        bz2mi_ddestroy(d);
        return nullptr;
    }
    return d;
}

void bz2mi_ddestroy(bz2mi_dctx* d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    for (void* p : {(void*)d->d_crctab, (void*)d->d_cnt, (void*)d->d_cand, (void*)d->d_ids, (void*)d->d_bwt,
                    (void*)d->d_syms, (void*)d->d_symmap, (void*)d->d_tabs, (void*)d->d_info, (void*)d->d_blocks, (void*)d->d_merged,
                    (void*)d->d_marks, (void*)d->d_iscr, (void*)d->d_rle1, (void*)d->d_cstate, (void*)d->d_olen, (void*)d->d_ooff,
                    (void*)d->d_crc, (void*)d->d_in, (void*)d->d_out, (void*)d->d_bad})
        if (p) (void)hipFree(p);
    for (auto& e : d->ev)
        if (e) (void)hipEventDestroy(e);
    if (d->ev_in) (void)hipEventDestroy(d->ev_in);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

int bz2mi_decompress_device(bz2mi_dctx* d, const void* d_in, size_t n, void* d_out, size_t cap, size_t* out_len,
                            void* hip_stream) {
    if (!d || !out_len || (n && !d_in) || (cap && !d_out)) return bz2mi_set_error(BZ2MI_EINVAL, "null argument");
    DCHECK(hipSetDevice(d->device));
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : d->stream;
    if (!hip_stream) {  // input written on the null stream (torch's default) is complete first
        DCHECK(hipEventRecord(d->ev_in, nullptr));
        DCHECK(hipStreamWaitEvent(s, d->ev_in, 0));
    }
    const uint8_t* in = (const uint8_t*)d_in;
    if (((uintptr_t)in & 3u) != 0) {  // the bit reader loads aligned words
        int r;
        if ((r = grow(&d->d_in, &d->in_cap, n))) return r;
        DCHECK(hipMemcpyAsync(d->d_in, in, n, hipMemcpyDeviceToDevice, s));
        in = d->d_in;
    }
    return run_decode(d, in, n, (uint8_t*)d_out, cap, out_len, s);
}

int bz2mi_decompress(bz2mi_dctx* d, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    if (!d || !out_len || (n && !in) || (cap && !out)) return bz2mi_set_error(BZ2MI_EINVAL, "null argument");
    DCHECK(hipSetDevice(d->device));
    int r;
    if ((r = grow(&d->d_in, &d->in_cap, n))) return r;
    if ((r = grow(&d->d_out, &d->out_cap, cap))) return r;
    if (n) DCHECK(hipMemcpyAsync(d->d_in, in, n, hipMemcpyHostToDevice, d->stream));
    r = run_decode(d, d->d_in, n, d->d_out, cap, out_len, d->stream);
    if (r != BZ2MI_OK) return r;
    if (*out_len) DCHECK(hipMemcpy(out, d->d_out, *out_len, hipMemcpyDeviceToHost));
    return BZ2MI_OK;
}

int bz2mi_dstream_reset(bz2mi_dctx* d) {
    if (!d) return bz2mi_set_error(BZ2MI_EINVAL, "null argument");
    d->walk = DecWalk{};
    d->pending = BZ2MI_OK;
    d->pending_msg.clear();
    return BZ2MI_OK;
}

int bz2mi_dstream(bz2mi_dctx* d, const uint8_t* in, size_t n, unsigned start_bit, int final, uint8_t* out,
                  size_t cap, uint64_t* end_bit, size_t* out_len, int* done) {
    if (!d || !end_bit || !out_len || !done || (n && !in) || (cap && !out))
        return bz2mi_set_error(BZ2MI_EINVAL, "null argument");
    *out_len = 0;
    *done = 0;
    *end_bit = start_bit;
    if (d->pending != BZ2MI_OK) {  // found by the previous call, after the bytes it returned
        const int e = d->pending;
        d->pending = BZ2MI_OK;
        return bz2mi_set_error(e, d->pending_msg);
    }
    if ((uint64_t)start_bit > (uint64_t)n * 8) return bz2mi_set_error(BZ2MI_EINVAL, "start bit beyond the window");
    if (d->walk.finished) {
        *done = 1;
        return BZ2MI_OK;
    }
    DCHECK(hipSetDevice(d->device));
    int r;
    if ((r = grow(&d->d_in, &d->in_cap, n + 8))) return r;
    if ((r = grow(&d->d_out, &d->out_cap, cap))) return r;
    if (n) DCHECK(hipMemcpyAsync(d->d_in, in, n, hipMemcpyHostToDevice, d->stream));
    for (float& m : d->ms) m = 0.f;
    size_t budget = (size_t)1 << 30;  // device bytes of decoded blocks per call
    if (const char* e = getenv("BZ2MI_DSTREAM_BUDGET")) budget = (size_t)strtoull(e, nullptr, 10);
    const size_t kmax_s = std::max<size_t>(64, budget / symbol_bytes(d->unit));
    const size_t kmax_c = std::max<size_t>(kmax_s, 2 * n / table_bytes());
    WinResult res;
    r = run_window(d, d->d_in, n, start_bit, final != 0, kmax_c, kmax_s, d->d_out, cap, &res, d->stream);
    if (r == BZ2MI_ESPACE) *out_len = res.out_len;
    if (r != BZ2MI_OK) return r;
    if (res.out_len) DCHECK(hipMemcpy(out, d->d_out, res.out_len, hipMemcpyDeviceToHost));
    *end_bit = res.end_bit;
    *out_len = res.out_len;
    *done = res.done ? 1 : 0;
    if (res.err != BZ2MI_OK) {
        if (res.out_len == 0) return bz2mi_set_error(res.err, res.msg);
        d->pending = res.err;
        d->pending_msg = res.msg;
    }
    return BZ2MI_OK;
}

int bz2mi_dset_flags(bz2mi_dctx* d, int flags) {
    if (!d || (flags & ~BZ2MI_DEC_CONCATENATED)) return bz2mi_set_error(BZ2MI_EINVAL, "invalid decoder flags");
    d->flags = flags;
    return BZ2MI_OK;
}

int bz2mi_dlast_trailing(bz2mi_dctx* d, uint64_t* bytes) {
    if (!d || !bytes) return bz2mi_set_error(BZ2MI_EINVAL, "null argument");
    *bytes = d->trailing;
    return BZ2MI_OK;
}

int bz2mi_dlast_timings(bz2mi_dctx* d, float* ms6) {
    if (!d || !ms6) return bz2mi_set_error(BZ2MI_EINVAL, "null argument");
    for (int k = 0; k < 6; ++k) ms6[k] = d->ms[k];
    return BZ2MI_OK;
}

}  // extern "C"
