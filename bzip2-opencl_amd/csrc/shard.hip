// Stream units (include/bz2mi.h "one logical stream compressed in units",
// SURVEY.md section 8(e)): one logical .bz2 stream compressed in contiguous
// byte ranges on any number of devices / processes, bit-identical to the
// single-device stream.
//
// What ties the blocks of a stream together in the reference, and how a unit
// gets it:
//  * the block split is a chain (a block ends where S-6 RLE1 bytes have been
//    flushed, OutputStream.hpp:179-188, BlockCompressor.hpp:69-96): the chain
//    kernel runs from the entry the previous unit hands over and stops at the
//    first block that starts past the unit (fe_chain_kernel), its exit being
//    the next unit's entry.  RLE1 state restarts at every block start, so the
//    unit's front end treats its buffer (own bytes + tail halo) as a stream of
//    its own.
//  * the per-slot frequency array is never cleared (OutputStream.hpp:93,
//    kernel.cpp:2613/2641-2643/3155): a unit's seeds are its own
//    per-slot running sums plus the sums of every earlier unit (`carried`).
//  * the block bits are concatenated without alignment and the stream CRC is
//    chained (OutputStream.hpp:190-240, :202): a unit returns its bit count and
//    CRC share, and is laid out at the stream bit offset the caller computes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "../../include/bz2mi.h"
#include "common.hpp"
#include "host.hpp"
#include "kernels.hpp"

using namespace bz2mi::host;

struct bz2mi_unit {
    bz2mi_ctx* c = nullptr;
    FrontBufs fe;
    Batch t;
    const uint8_t* d_x = nullptr;
    size_t n_own = 0, n = 0;
    bool ends = false;
    uint64_t nb = 0, first_block = 0;
    uint32_t* d_state = nullptr;  // p x 258: this unit's slot sums, then the carried seeds
    bz2mi::StreamDev* d_sd = nullptr;
    unsigned long long* d_vol = nullptr;  // RLE1 bytes, MTF/RLE2 symbols, payload bits (volume_kernel)
    int stage = 0;                // 1 begun, 2 chained, 3 encoded
    uint64_t bits = 0;
    uint32_t crc = 0;
    float chain_ms = 0;
    // speculation (bz2mi_unit_speculate): the chain from byte 0, its block
    // count and exit token; chain outcome: blocks taken from it, blocks chained
    bool spec_tried = false;
    uint64_t spec_nb = 0, spec_exit = 0;
    uint64_t spliced = 0, chained = 0;
    hipEvent_t ev_in = nullptr;
    hipEvent_t ev[12] = {};  // stage brackets: front, rle1+bwt, mtf, (seed), huffman, assembly
    uint8_t* d_own = nullptr;  // host-fed units: device copy of the bytes
    size_t own_cap = 0;
    uint8_t* d_out = nullptr;  // host-fed units: assembled bytes
    size_t out_cap = 0;
    uint8_t* h_pin = nullptr;  // pinned staging of the carried seeds and the encode results (async copies)
};

namespace {

bool stage_ok(bz2mi_unit* u, int want) { return u && u->stage >= want; }

// word copy by a kernel, between device and pinned host memory: the unit's
// small control copies stay on its stream's queue (a DMA-engine copy there
// measured as waiting for work queued on the other streams)
__global__ void copy_words_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
}

// in-place assembly: the previous unit's bits of the first output word
// become the carry (MSB-aligned), as advance_kernel carries a batch's last word
__global__ void carry_in_kernel(bz2mi::StreamDev* __restrict__ st, const uint32_t* __restrict__ out) {
    if (threadIdx.x != 0) return;
    const uint32_t cb = st->carry_bits;
    st->carry = cb ? __builtin_bswap32(out[st->word_base]) & (0xffffffffu << (32 - cb)) : 0u;
}

}  // namespace

extern "C" {

size_t bz2mi_unit_halo(int level, int unit) {
    // the longest raw span of one block: every RLE1 piece of 5 bytes covers
    // 255 input bytes, and the chain's mid-run step looks one piece further
    const size_t S = (size_t)unit * (size_t)level;
    return (S / 5 + 2) * 255 + 64;
}

bz2mi_unit* bz2mi_unit_create(bz2mi_ctx* c) {
    if (!c) {
        fail(BZ2MI_EINVAL, "null context");
        return nullptr;
    }
    if (hipSetDevice(c->device) != hipSuccess) {
        fail(BZ2MI_EDEVICE, "hipSetDevice failed");
        return nullptr;
    }
    auto* u = new bz2mi_unit();
    u->c = c;
    bool ok = dalloc(&u->d_state, (size_t)c->p * bz2mi::kMaxAlpha) == BZ2MI_OK && dalloc(&u->d_sd, 1) == BZ2MI_OK &&
              dalloc(&u->d_vol, 4) == BZ2MI_OK &&
              hipEventCreateWithFlags(&u->ev_in, hipEventDisableTiming) == hipSuccess;
    for (auto& e : u->ev) ok = ok && hipEventCreate(&e) == hipSuccess;
    if (!ok) {
        fail(BZ2MI_EDEVICE, "bz2mi_unit_create: HIP allocation failed");
        bz2mi_unit_destroy(u);
        return nullptr;
    }
    return u;
}

void bz2mi_unit_destroy(bz2mi_unit* u) {
    if (!u) return;
    (void)hipSetDevice(u->c->device);
    for (hipStream_t st : {u->c->stream, u->c->sA, u->c->sM, u->c->sB, u->c->sF})
        if (st) (void)hipStreamSynchronize(st);
    free_front(u->fe);
    free_batch(u->t);
    if (u->d_own) (void)hipFree(u->d_own);
    if (u->d_out) (void)hipFree(u->d_out);
    if (u->d_state) (void)hipFree(u->d_state);
    if (u->d_sd) (void)hipFree(u->d_sd);
    if (u->d_vol) (void)hipFree(u->d_vol);
    if (u->h_pin) (void)hipHostFree(u->h_pin);
    if (u->ev_in) (void)hipEventDestroy(u->ev_in);
    for (auto& e : u->ev)
        if (e) (void)hipEventDestroy(e);
    delete u;
}

int bz2mi_unit_begin(bz2mi_unit* u, const void* d_buf, size_t n_own, size_t n_halo, int flags, void* hip_stream) {
    if (!u || (!d_buf && n_own + n_halo)) return fail(BZ2MI_EINVAL, "null argument");
    if (n_own == 0) return fail(BZ2MI_EINVAL, "empty stream unit");
    bz2mi_ctx* c = u->c;
    HIPCHECK(hipSetDevice(c->device));
    int r;
    u->d_x = (const uint8_t*)d_buf;
    u->n_own = n_own;
    u->n = n_own + n_halo;
    u->ends = (flags & BZ2MI_UNIT_ENDS_STREAM) != 0;
    if (!u->ends && n_halo < bz2mi_unit_halo(c->level, c->unit))
        return fail(BZ2MI_EINVAL, "stream unit: tail halo shorter than bz2mi_unit_halo()");
    u->nb = 0;
    u->stage = 0;
    u->spec_tried = false;
    u->spec_nb = u->spec_exit = u->spliced = u->chained = 0;
    if ((r = ensure_front(u->fe, c->S, u->n))) return r;
    // the bytes were written on the caller's stream (NULL: the null stream)
    HIPCHECK(hipEventRecord(u->ev_in, (hipStream_t)hip_stream));
    HIPCHECK(hipStreamWaitEvent(c->sF, u->ev_in, 0));
    (void)hipGetLastError();
    HIPCHECK(hipEventRecord(u->ev[0], c->sF));
    if ((r = enqueue_front_scan(u->fe, u->d_x, u->n, c->sF))) return r;
    HIPCHECK(hipEventRecord(u->ev[1], c->sF));
    u->stage = 1;
    return BZ2MI_OK;
}

int bz2mi_unit_speculate(bz2mi_unit* u, uint64_t* nblocks) {
    if (!u || u->stage != 1) return fail(BZ2MI_ESTATE, "bz2mi_unit_speculate: unit not begun or already chained");
    bz2mi_ctx* c = u->c;
    if (!u->spec_tried) {
        HIPCHECK(hipSetDevice(c->device));
        u->spec_tried = true;
        HIPCHECK(hipStreamWaitEvent(c->stream, u->ev[1], 0));
        uint64_t nb = 0, ex = 0;
        const int r = run_chain(c, u->fe, u->d_x, u->n, u->n_own, 0, u->ends, &nb, &ex, c->stream);
        if (r == BZ2MI_EINVAL) {
            // the speculative chain's last block runs past the tail halo: no
            // speculation (the chain from the real entry decides); an expected
            // outcome, so its message is not left behind
            (void)hipGetLastError();
            clear_error();
        } else if (r) {
            return r;
        } else {
            // keep its starts [0, nb] (the chain from the entry rewrites d_starts)
            hipLaunchKernelGGL(copy_words_kernel, dim3((unsigned)std::min<uint64_t>((2 * nb + 257) / 256, 64)), dim3(256),
                               0, c->stream, reinterpret_cast<const uint32_t*>(u->fe.d_starts),
                               reinterpret_cast<uint32_t*>(u->fe.d_spec), (int)(2 * (nb + 1)));
            HIPCHECK(hipGetLastError());
            u->spec_nb = nb;
            u->spec_exit = ex;
        }
    }
    if (nblocks) *nblocks = u->spec_nb;
    return BZ2MI_OK;
}

int bz2mi_unit_chain_info(bz2mi_unit* u, uint64_t* out4) {
    if (!u || !out4) return fail(BZ2MI_EINVAL, "null argument");
    out4[0] = u->spec_nb;
    out4[1] = u->spliced;
    out4[2] = u->chained;
    out4[3] = u->spec_tried ? 1 : 0;
    return BZ2MI_OK;
}

int bz2mi_unit_chain(bz2mi_unit* u, uint64_t entry, uint64_t first_block, uint64_t* exit_entry, uint64_t* nblocks) {
    if (!stage_ok(u, 1) || !exit_entry || !nblocks) return fail(BZ2MI_ESTATE, "bz2mi_unit_chain: unit not begun");
    bz2mi_ctx* c = u->c;
    HIPCHECK(hipSetDevice(c->device));
    const uint64_t p0 = entry & ~BZ2MI_ENTRY_MIDRUN;
    u->first_block = first_block;
    if (p0 >= u->n_own) {  // the previous unit's last block covers this one
        u->nb = 0;
        *nblocks = 0;
        *exit_entry = (p0 - u->n_own) | (entry & BZ2MI_ENTRY_MIDRUN);
        u->stage = 2;
        return BZ2MI_OK;
    }
    int r;
    const auto t0 = std::chrono::steady_clock::now();
    HIPCHECK(hipStreamWaitEvent(c->stream, u->ev[1], 0));
    uint64_t nb = 0, ex = 0, spl = 0;
    if (u->spec_nb && p0 == 0) {
        // the speculation was right: its starts are the chain (a block's split
        // does not depend on the bytes before its start, so a mid-run flag on
        // entry 0 changes nothing: the unit's buffer starts a run there)
        nb = spl = u->spec_nb;
        ex = u->spec_exit;
        hipLaunchKernelGGL(copy_words_kernel, dim3((unsigned)std::min<uint64_t>((2 * nb + 257) / 256, 64)), dim3(256), 0,
                           c->stream, reinterpret_cast<const uint32_t*>(u->fe.d_spec),
                           reinterpret_cast<uint32_t*>(u->fe.d_starts), (int)(2 * (nb + 1)));
        HIPCHECK(hipGetLastError());
        // stage_front reads d_starts on stream A: the copy is done first (as
        // run_chain's own path is synchronous on the context stream)
        HIPCHECK(hipStreamSynchronize(c->stream));
    } else if ((r = run_chain(c, u->fe, u->d_x, u->n, u->n_own, entry, u->ends, &nb, &ex, c->stream, u->spec_nb,
                              u->spec_exit, &spl))) {
        return r;
    }
    u->spliced = spl;
    u->chained = nb - spl;
    u->chain_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (nb > (uint64_t)INT32_MAX) return fail(BZ2MI_EINVAL, "stream unit: too many blocks");
    u->nb = nb;
    // the last block of a unit that ends the stream runs to its end
    *exit_entry = u->ends && (ex & ~BZ2MI_ENTRY_MIDRUN) >= u->n - u->n_own ? (u->n - u->n_own) : ex;
    *nblocks = nb;
    const int cnt = (int)nb;
    if ((r = ensure_batch(c, u->t, cnt))) return r;
    Batch& t = u->t;
    // RLE1 emission, CRCs, BWT (stream A); MTF (M); this unit's slot sums (B)
    HIPCHECK(hipEventRecord(u->ev[2], c->sA));
    if ((r = stage_front(c, t, u->fe, u->d_x, u->n, 0, nb, c->sA))) return r;
    if ((r = stage_bwt(c, t, cnt, c->sA))) return r;
    HIPCHECK(hipEventRecord(u->ev[3], c->sA));
    HIPCHECK(hipEventRecord(t.evA, c->sA));
    HIPCHECK(hipStreamWaitEvent(c->sM, t.evA, 0));
    HIPCHECK(hipEventRecord(u->ev[4], c->sM));
    if ((r = stage_mtf(c, t, cnt, c->sM))) return r;
    HIPCHECK(hipEventRecord(u->ev[5], c->sM));
    HIPCHECK(hipEventRecord(t.evM, c->sM));
    // this unit's slot sums right behind its MTF on stream M: stream B stays
    // free for the Huffman coding of units whose seeds are known (a wait for
    // a later unit's MTF queued on B would hold the earlier units' coding back)
    HIPCHECK(hipMemsetAsync(u->d_state, 0, sizeof(uint32_t) * c->p * bz2mi::kMaxAlpha, c->sM));
    if ((r = stage_seed(c, t, cnt, first_block, u->d_state, c->sM))) return r;
    HIPCHECK(hipEventRecord(u->ev[6], c->sM));
    u->stage = 2;
    return BZ2MI_OK;
}

int bz2mi_unit_sums(bz2mi_unit* u, uint32_t* sums) {
    if (!stage_ok(u, 2) || !sums) return fail(BZ2MI_ESTATE, "bz2mi_unit_sums: unit not chained");
    bz2mi_ctx* c = u->c;
    const size_t ne = (size_t)c->p * bz2mi::kMaxAlpha;
    if (u->nb == 0) {
        std::memset(sums, 0, ne * sizeof(uint32_t));
        return BZ2MI_OK;
    }
    HIPCHECK(hipSetDevice(c->device));
    HIPCHECK(hipEventSynchronize(u->ev[6]));
    HIPCHECK(hipMemcpy(sums, u->d_state, ne * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return BZ2MI_OK;
}

int bz2mi_unit_encode(bz2mi_unit* u, const uint32_t* carried, uint64_t* bits, uint32_t* crc) {
    if (!stage_ok(u, 2) || !carried || !bits || !crc) return fail(BZ2MI_ESTATE, "bz2mi_unit_encode: unit not chained");
    bz2mi_ctx* c = u->c;
    if (u->nb == 0) {
        *bits = 0;
        *crc = 0;
        u->bits = 0;
        u->crc = 0;
        u->stage = 3;
        return BZ2MI_OK;
    }
    HIPCHECK(hipSetDevice(c->device));
    int r;
    const int cnt = (int)u->nb;
    Batch& t = u->t;
    hipStream_t s = c->sB;
    const size_t ne = (size_t)c->p * bz2mi::kMaxAlpha;
    // seeds: the carried sums of the earlier units, then this unit's running
    // sums (after its MTF and its own slot sums on stream M)
    // (bz2mi_unit_sums has normally waited for it on the host already; a
    // device-side wait on an event of stream M measured as a wait for
    // everything queued on M later -- the Huffman coding of unit 0 started
    // after the last unit's MTF -- so the stream waits only if it must)
    if (hipEventQuery(u->ev[6]) != hipSuccess) HIPCHECK(hipStreamWaitEvent(s, u->ev[6], 0));
    // pinned staging: a copy from pageable memory is carried out synchronously
    // behind the device's other queued work (measured: unit 0's coding waited
    // for the last unit's MTF)
    if (!u->h_pin) HIPCHECK(hipHostMalloc((void**)&u->h_pin, ne * sizeof(uint32_t) + 256, hipHostMallocDefault));
    std::memcpy(u->h_pin, carried, ne * sizeof(uint32_t));
    hipLaunchKernelGGL(copy_words_kernel, dim3(4), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(u->h_pin),
                       u->d_state, (int)ne);
    HIPCHECK(hipEventRecord(u->ev[7], s));
    if ((r = stage_seed(c, t, cnt, u->first_block, u->d_state, s))) return r;
    if ((r = stage_huffman(c, t, cnt, s))) return r;
    HIPCHECK(hipEventRecord(u->ev[8], s));
    HIPCHECK(hipMemsetAsync(u->d_vol, 0, 4 * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(bz2mi::volume_kernel, dim3(16), dim3(256), 0, s, t.d_lens, t.d_mtflen, t.d_pbits, cnt, u->d_vol);
    // bit count and CRC share (offsets from bit 0, stream CRC from 0)
    HIPCHECK(hipMemsetAsync(u->d_sd, 0, sizeof(bz2mi::StreamDev), s));
    hipLaunchKernelGGL(bz2mi::offsets_dev_kernel, dim3(1), dim3(256), 0, s, t.d_pbits, t.d_crc, cnt, u->d_sd, t.d_offs);
    HIPCHECK(hipGetLastError());
    bz2mi::StreamDev sd{};
    uint64_t total = 0;
    uint8_t* res = u->h_pin + ne * sizeof(uint32_t);  // (its bytes after the seeds: 256 >= 8 + sizeof(sd))
    static_assert(sizeof(bz2mi::StreamDev) + 12 <= 256, "pinned result area");
    hipLaunchKernelGGL(copy_words_kernel, dim3(1), dim3(64), 0, s, reinterpret_cast<const uint32_t*>(t.d_offs + cnt),
                       reinterpret_cast<uint32_t*>(res), 2);
    hipLaunchKernelGGL(copy_words_kernel, dim3(1), dim3(64), 0, s, reinterpret_cast<const uint32_t*>(u->d_sd),
                       reinterpret_cast<uint32_t*>(res + 8), (int)(sizeof(sd) / 4));
    // the front end's segment-table overflow flag (fe_segplan_kernel)
    hipLaunchKernelGGL(copy_words_kernel, dim3(1), dim3(64), 0, s, u->fe.d_nseg + 1,
                       reinterpret_cast<uint32_t*>(res + 8 + sizeof(sd)), 1);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    std::memcpy(&total, res, sizeof(uint64_t));
    std::memcpy(&sd, res + 8, sizeof(sd));
    {
        uint32_t segov = 0;
        std::memcpy(&segov, res + 8 + sizeof(sd), sizeof(segov));
        if (segov) return fail(BZ2MI_EDEVICE, "front end: RLE1 segment table overflow");
    }
    u->bits = total;
    u->crc = sd.crc;
    *bits = total;
    *crc = sd.crc;
    u->stage = 3;
    return BZ2MI_OK;
}

int bz2mi_unit_assemble(bz2mi_unit* u, uint64_t bit_offset, uint32_t crc_before, int flags, void* d_out, size_t cap,
                        size_t* out_bytes, void* hip_stream) {
    if (!stage_ok(u, 3) || !out_bytes || !d_out) return fail(BZ2MI_ESTATE, "bz2mi_unit_assemble: unit not encoded");
    if (((uintptr_t)d_out & 3) != 0) return fail(BZ2MI_EINVAL, "bz2mi_unit_assemble: output not 4-byte aligned");
    bz2mi_ctx* c = u->c;
    const bool first = (flags & BZ2MI_UNIT_FIRST) != 0, last = (flags & BZ2MI_UNIT_LAST) != 0;
    const bool in_place = (flags & BZ2MI_UNIT_IN_PLACE) != 0;
    if (first && bit_offset != 0) return fail(BZ2MI_EINVAL, "bz2mi_unit_assemble: the first unit starts at bit 0");
    HIPCHECK(hipSetDevice(c->device));
    const int cnt = (int)u->nb;
    Batch& t = u->t;
    hipStream_t s = c->sB;
    bz2mi::StreamDev sd{};
    if (first) {  // "BZh<level>" (OutputStream.hpp:126-128)
        sd.carry = (0x425a68u << 8) | (uint32_t)('0' + c->level);
        sd.carry_bits = 32;
    } else if (in_place) {  // from the word holding bit_offset (carry read on the device)
        sd.word_base = bit_offset >> 5;
        sd.carry_bits = (uint32_t)(bit_offset & 31);
    } else {
        sd.carry_bits = (uint32_t)(bit_offset & 7);
    }
    sd.crc = crc_before;
    const uint64_t end = sd.word_base * 32 + sd.carry_bits + u->bits + (last ? 80u : 0u);
    const uint64_t nbytes = (end + 7) / 8;
    const uint64_t cap_words = cap / 4;
    if (((end + 31) / 32) > cap_words) return fail(BZ2MI_ESPACE, "output buffer too small");
    if (cnt == 0) return fail(BZ2MI_EINVAL, "bz2mi_unit_assemble: the unit has no blocks");
    // d_out may still be read or written by work queued on the caller's
    // stream (NULL: the null stream): assembly writes it only after that
    HIPCHECK(hipEventRecord(u->ev_in, (hipStream_t)hip_stream));
    HIPCHECK(hipStreamWaitEvent(s, u->ev_in, 0));
    HIPCHECK(hipEventRecord(u->ev[9], s));
    HIPCHECK(hipMemcpyAsync(u->d_sd, &sd, sizeof(sd), hipMemcpyHostToDevice, s));
    if (in_place && !first && sd.carry_bits)
        hipLaunchKernelGGL(carry_in_kernel, dim3(1), dim3(64), 0, s, u->d_sd, (const uint32_t*)d_out);
    hipLaunchKernelGGL(bz2mi::offsets_dev_kernel, dim3(1), dim3(256), 0, s, t.d_pbits, t.d_crc, cnt, u->d_sd, t.d_offs);
    hipLaunchKernelGGL(bz2mi::assemble_dev_kernel, dim3((unsigned)cnt + 2), dim3(256), 0, s, t.d_payload,
                       c->payload_words, t.d_offs, t.d_crc, cnt, last ? 1 : 0, u->d_sd, (uint32_t*)d_out, cap_words);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(u->ev[10], s));
    HIPCHECK(hipStreamSynchronize(s));
    *out_bytes = (size_t)nbytes;
    return BZ2MI_OK;
}

void* bz2mi_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        fail(BZ2MI_EDEVICE, "hipHostMalloc failed");
        return nullptr;
    }
    return p;
}

void bz2mi_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int bz2mi_unit_begin_host(bz2mi_unit* u, const void* host, size_t n_own, size_t n_halo, int flags) {
    if (!u || (!host && n_own + n_halo)) return fail(BZ2MI_EINVAL, "null argument");
    bz2mi_ctx* c = u->c;
    HIPCHECK(hipSetDevice(c->device));
    const size_t n = n_own + n_halo;
    if (n + 64 > u->own_cap) {
        int r;
        const size_t cap = n + n / 8 + 64;
        if ((r = dalloc(&u->d_own, cap))) return r;
        u->own_cap = cap;
    }
    // on the front-scan stream: begin() orders the scan after it
    HIPCHECK(hipMemcpyAsync(u->d_own, host, n, hipMemcpyHostToDevice, c->sF));
    return bz2mi_unit_begin(u, u->d_own, n_own, n_halo, flags, c->sF);
}

int bz2mi_unit_assemble_host(bz2mi_unit* u, uint64_t bit_offset, uint32_t crc_before, int flags, void* host_out,
                             size_t cap, size_t* out_bytes, void* hip_stream) {
    if (!u || !host_out || !out_bytes) return fail(BZ2MI_EINVAL, "null argument");
    bz2mi_ctx* c = u->c;
    HIPCHECK(hipSetDevice(c->device));
    const size_t need = (size_t)((u->bits + 32 + 80 + 7) / 8) + 64;
    if (need > u->out_cap) {
        int r;
        if ((r = dalloc(&u->d_out, need + need / 8))) return r;
        u->out_cap = need + need / 8;
    }
    int r = bz2mi_unit_assemble(u, bit_offset, crc_before, flags, u->d_out, u->out_cap, out_bytes, hip_stream);
    if (r) return r;
    if (*out_bytes > cap) return fail(BZ2MI_ESPACE, "output buffer too small");
    HIPCHECK(hipMemcpy(host_out, u->d_out, *out_bytes, hipMemcpyDeviceToHost));
    return BZ2MI_OK;
}

int bz2mi_unit_stats(bz2mi_unit* u, uint64_t* out4) {
    if (!u || !out4) return fail(BZ2MI_EINVAL, "null argument");
    out4[0] = out4[1] = out4[2] = 0;
    out4[3] = u->nb;
    if (u->nb == 0 || u->stage < 3) return BZ2MI_OK;
    HIPCHECK(hipSetDevice(u->c->device));
    unsigned long long v[4] = {0, 0, 0, 0};
    HIPCHECK(hipMemcpy(v, u->d_vol, sizeof(v), hipMemcpyDeviceToHost));
    for (int i = 0; i < 3; ++i) out4[i] = v[i];
    return BZ2MI_OK;
}

int bz2mi_unit_timings(bz2mi_unit* u, float* ms6) {
    if (!u || !ms6) return fail(BZ2MI_EINVAL, "null argument");
    auto el = [&](int a, int b) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, u->ev[a], u->ev[b]) != hipSuccess) ms = 0;
        return ms;
    };
    const bool blocks = u->nb > 0 && u->stage >= 2;
    ms6[0] = u->stage >= 1 ? el(0, 1) : 0;
    ms6[1] = u->chain_ms;
    ms6[2] = blocks ? el(2, 3) : 0;
    ms6[3] = blocks ? el(4, 5) : 0;
    ms6[4] = blocks && u->stage >= 3 ? el(7, 8) : 0;
    ms6[5] = blocks && u->stage >= 3 ? el(9, 10) : 0;
    (void)hipGetLastError();
    return BZ2MI_OK;
}

}  // extern "C"
