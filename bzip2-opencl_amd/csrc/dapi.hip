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

template <class T>
int grow(T** p, size_t* cap, size_t count) {
    if (count <= *cap && *p) return BZ2MI_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t c = std::max<size_t>(count, 1);
    hipError_t e = hipMalloc((void**)p, c * sizeof(T));
    if (e != hipSuccess) return bz2mi_set_error(BZ2MI_EDEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
    *cap = c;
    return BZ2MI_OK;
}

}  // namespace

struct bz2mi_dctx {
    int unit = 10000, device = 0, cus = 256;
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
};

namespace {

// inverse-BWT workgroups per XCD (BZ2MI_IBWT_XCD overrides, for experiments)
int ibwt_wg_per_xcd() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("BZ2MI_IBWT_XCD");
        v = (e && atoi(e) > 0) ? atoi(e) : 32;  // measured 8/16/24/32: 101/64/55/58 ms per GiB random, 100/59/45/42 text
    }
    return v;
}

// the whole decode of n bytes at d_in (4-byte aligned) into d_out
int run_decode(bz2mi_dctx* d, const uint8_t* d_in, size_t n, uint8_t* d_out, size_t cap, size_t* out_len,
               hipStream_t s) {
    using namespace bz2mi;
    int r;
    *out_len = 0;
    DCHECK(hipEventRecord(d->ev[0], s));
    // ---- stream header (InputStream::initializeStream :96-115)
    if (n < 4) return bz2mi_set_error(BZ2MI_EFORMAT, n == 0 ? "Insufficient data" : "Invalid BZip2 header");
    // ---- K1: candidates
    const size_t cap_c = n / 8 + 4096;
    if ((r = grow(&d->d_cand, &d->cand_cap, cap_c))) return r;
    DCHECK(hipMemsetAsync(d->d_cnt, 0, 4 * sizeof(uint32_t), s));
    {
        const uint64_t words = (n + 7) / 8;
        hipLaunchKernelGGL(dec_scan_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, d_in, (uint64_t)n,
                           d->d_cand, d->d_cnt, (uint32_t)d->cand_cap);
        DCHECK(hipGetLastError());
    }
    uint32_t ncand = 0;
    DCHECK(hipMemcpyAsync(&ncand, d->d_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    DCHECK(hipStreamSynchronize(s));
    if (ncand > d->cand_cap) {
        // more magic matches than the estimate (crafted input): the scan
        // counted them all, so rescan into a buffer of the exact size
        if ((r = grow(&d->d_cand, &d->cand_cap, ncand))) return r;
        DCHECK(hipMemsetAsync(d->d_cnt, 0, 4 * sizeof(uint32_t), s));
        const uint64_t words = (n + 7) / 8;
        hipLaunchKernelGGL(dec_scan_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, d_in, (uint64_t)n,
                           d->d_cand, d->d_cnt, (uint32_t)d->cand_cap);
        DCHECK(hipGetLastError());
        DCHECK(hipMemcpyAsync(&ncand, d->d_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        DCHECK(hipStreamSynchronize(s));
        if (ncand > d->cand_cap) return bz2mi_set_error(BZ2MI_EFORMAT, "BZip2 stream format error");
    }
    DCHECK(hipEventRecord(d->ev[1], s));
    std::vector<DecCand> cand(ncand);
    if (ncand) DCHECK(hipMemcpy(cand.data(), d->d_cand, ncand * sizeof(DecCand), hipMemcpyDeviceToHost));
    std::sort(cand.begin(), cand.end(), [](const DecCand& a, const DecCand& b) { return a.bitpos < b.bitpos; });
    if (ncand) DCHECK(hipMemcpy(d->d_cand, cand.data(), ncand * sizeof(DecCand), hipMemcpyHostToDevice));
    // ---- K2: every block candidate
    std::vector<uint32_t> ids;
    std::vector<int64_t> id_of(ncand, -1);
    for (uint32_t i = 0; i < ncand; ++i)
        if (cand[i].type == 0) {
            id_of[i] = (int64_t)ids.size();
            ids.push_back(i);
        }
    const uint32_t smax = (uint32_t)(9 * d->unit);
    const uint32_t max_sel = d->unit == 10000 ? (uint32_t)(smax / 50 + 1) : (uint32_t)(smax / 50 + 2);
    const size_t stride = ((size_t)smax + 255) & ~(size_t)255;
    const size_t sym_stride = ((size_t)smax + 2 + 63) & ~(size_t)63;
    const size_t nk = ids.size();
    if ((r = grow(&d->d_ids, &d->ids_cap, nk))) return r;
    if ((r = grow(&d->d_syms, &d->syms_cap, nk * sym_stride))) return r;
    if ((r = grow(&d->d_symmap, &d->symmap_cap, nk * 256))) return r;
    if ((r = grow(&d->d_tabs, &d->tabs_cap, nk * kTabBytes))) return r;
    if ((r = grow(&d->d_info, &d->info_cap, nk))) return r;
    if (nk) {
        DCHECK(hipMemcpyAsync(d->d_ids, ids.data(), nk * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(dec_huff_kernel, dim3((unsigned)nk), dim3(64), (max_sel + 7) / 8 * 4, s, d_in, (uint64_t)n,
                           d->d_cand, d->d_ids, (uint32_t)nk, max_sel, d->d_tabs, d->d_symmap, d->d_info);
        DCHECK(hipGetLastError());
        hipLaunchKernelGGL(dec_sym_kernel, dim3((unsigned)((nk + kDecSymBlocks - 1) / kDecSymBlocks)), dim3(64), 0, s, d_in, (uint64_t)n, d->d_tabs,
                           (uint32_t)nk, smax, d->d_syms, sym_stride, d->d_info);
        DCHECK(hipGetLastError());
    }
    std::vector<DecBlockInfo> info(nk);
    if (nk) DCHECK(hipMemcpyAsync(info.data(), d->d_info, nk * sizeof(DecBlockInfo), hipMemcpyDeviceToHost, s));
    DCHECK(hipEventRecord(d->ev[2], s));
    DCHECK(hipStreamSynchronize(s));
    if (const char* dump = getenv("BZ2MI_DDUMP")) {  // debug: first candidate's info and BWT bytes
        if (FILE* f = fopen(dump, "wb")) {
            if (nk) {
                fwrite(&info[0], sizeof(DecBlockInfo), 1, f);
                std::vector<uint16_t> b(std::min<size_t>(info[0].nsym, sym_stride));
                DCHECK(hipMemcpy(b.data(), d->d_syms, b.size() * 2, hipMemcpyDeviceToHost));
                fwrite(b.data(), 2, b.size(), f);
            }
            fclose(f);
        }
    }
    // ---- the stream structure (InputStream.hpp:96-158), over the candidates
    auto find = [&](uint64_t bit) -> int64_t {
        auto it = std::lower_bound(cand.begin(), cand.end(), bit,
                                   [](const DecCand& c, uint64_t b) { return c.bitpos < b; });
        return (it != cand.end() && it->bitpos == bit) ? (int64_t)(it - cand.begin()) : -1;
    };
    auto header_at = [&](uint64_t byte, int* digit) -> int {
        uint8_t h[4];
        hipError_t e = hipMemcpy(h, d_in + byte, 4, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return -1;
        if (h[0] != 'B' || h[1] != 'Z' || h[2] != 'h' || h[3] < '1' || h[3] > '9') return 0;
        *digit = h[3] - '0';
        return 1;
    };
    std::vector<uint32_t> chain;       // decoded-candidate ids, stream order
    std::vector<uint32_t> chain_crc;   // stored block CRCs
    std::vector<uint32_t> chain_S;     // the block size limit of each block's stream
    std::vector<uint32_t> stream_end;  // chain index where each stream ends
    std::vector<uint32_t> stream_crc;  // stored stream CRCs
    int err_status = -1;               // first structural / decode error after the chain
    std::string err_msg;
    uint64_t byte = 0;
    bool first = true;
    while (byte + 4 <= n) {
        int digit = 0;
        const int h = header_at(byte, &digit);
        if (h < 0) return bz2mi_set_error(BZ2MI_EDEVICE, "hipMemcpy (stream header)");
        if (h == 0) {
            if (first) return bz2mi_set_error(BZ2MI_EFORMAT, "Invalid BZip2 header");
            break;  // trailing bytes after the last stream
        }
        first = false;
        const uint32_t S = (uint32_t)(digit * d->unit);
        uint64_t pos = byte * 8 + 32;
        bool ended = false;
        while (err_status < 0) {
            const int64_t ci = find(pos);
            if (ci < 0) {
                err_status = 0;
                err_msg = pos + 48 > (uint64_t)n * 8 ? "Insufficient data" : "BZip2 stream format error";
                break;
            }
            if (cand[ci].type == 1) {
                stream_end.push_back((uint32_t)chain.size());
                stream_crc.push_back(cand[ci].next32);
                if (pos + 80 > (uint64_t)n * 8) {
                    err_status = 0;
                    err_msg = "Insufficient data";
                    break;
                }
                pos += 80;
                ended = true;
                break;
            }
            const uint32_t k = (uint32_t)id_of[ci];
            if (info[k].status) {
                err_status = (int)info[k].status;
                err_msg = dec_message(info[k].status);
                break;
            }
            if (info[k].end_bit > (uint64_t)n * 8) {
                err_status = 0;
                err_msg = "Insufficient data";
                break;
            }
            chain.push_back(k);
            chain_crc.push_back(info[k].crc);
            chain_S.push_back(S);
            pos = info[k].end_bit;
        }
        if (!ended) break;
        byte = (pos + 7) / 8;
        // the reference's InputStream ends at the first end-of-stream marker
        // (InputStream.hpp:136-143); bzip2 goes on to the next stream
        if (!(d->flags & BZ2MI_DEC_CONCATENATED)) break;
    }
    // ---- K2b (MTF / RLE2) over the blocks of the chain; its errors (block
    // size, origPtr) end the chain at the first failing block
    if (!chain.empty()) {
        if ((r = grow(&d->d_blocks, &d->blocks_cap, chain.size()))) return r;
        if ((r = grow(&d->d_bwt, &d->bwt_cap, nk * stride))) return r;
        // d_merged (the inverse BWT's vector, free until then) is the scratch
        if ((r = grow(&d->d_merged, &d->merged_cap, chain.size() * sym_stride))) return r;
        DCHECK(hipMemcpyAsync(d->d_blocks, chain.data(), chain.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(dec_mtf_kernel, dim3((unsigned)chain.size()), dim3(64), 0, s, d->d_syms, sym_stride,
                           d->d_symmap, d->d_blocks, (uint32_t)chain.size(), smax, d->d_merged, sym_stride,
                           d->d_bwt, stride, d->d_info);
        DCHECK(hipGetLastError());
        DCHECK(hipMemcpyAsync(info.data(), d->d_info, nk * sizeof(DecBlockInfo), hipMemcpyDeviceToHost, s));
        DCHECK(hipStreamSynchronize(s));
        for (size_t i = 0; i < chain.size(); ++i) {
            const DecBlockInfo& bi = info[chain[i]];
            const uint32_t st = bi.status ? bi.status : (bi.len > chain_S[i] ? (uint32_t)kDecSize : 0u);
            if (st) {
                err_status = (int)st;
                err_msg = dec_message(st);
                chain.resize(i);
                chain_crc.resize(i);
                while (!stream_end.empty() && stream_end.back() > i) {
                    stream_end.pop_back();
                    stream_crc.pop_back();
                }
                break;
            }
        }
    }
    DCHECK(hipEventRecord(d->ev[3], s));
    // ---- K3 / K4 over the blocks of the chain
    const size_t nb = chain.size();
    std::vector<uint64_t> olen(nb), ooff(nb + 1, 0);
    std::vector<uint32_t> crc(nb), bad(nb, 0);
    if (nb) {
        if ((r = grow(&d->d_blocks, &d->blocks_cap, nb))) return r;
        if ((r = grow(&d->d_merged, &d->merged_cap, std::max(nb * stride, nb * sym_stride)))) return r;
        if ((r = grow(&d->d_marks, &d->marks_cap, nb * stride))) return r;
        if ((r = grow(&d->d_rle1, &d->rle1_cap, nb * stride))) return r;
        if ((r = grow(&d->d_cstate, &d->cstate_cap, nb * 256))) return r;
        if ((r = grow(&d->d_olen, &d->olen_cap, nb))) return r;
        if ((r = grow(&d->d_ooff, &d->ooff_cap, nb))) return r;
        if ((r = grow(&d->d_crc, &d->crc_cap, nb))) return r;
        if ((r = grow(&d->d_bad, &d->bad_cap, nb))) return r;
        DCHECK(hipMemsetAsync(d->d_bad, 0, nb * sizeof(uint32_t), s));
        DCHECK(hipMemcpyAsync(d->d_blocks, chain.data(), nb * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(dec_ibwt_kernel, dim3((unsigned)std::min<size_t>(nb, (size_t)8 * ibwt_wg_per_xcd())),
                           dim3(kDecIbwtThreads), 0, s, d->d_bwt, stride, d->d_info, d->d_blocks, (uint32_t)nb, d->d_merged, stride, d->d_marks, stride, d->d_rle1,
                           stride, d->d_bad);
        DCHECK(hipGetLastError());
        DCHECK(hipEventRecord(d->ev[4], s));
        hipLaunchKernelGGL(dec_rle1_kernel, dim3((unsigned)nb), dim3(256), 0, s, d->d_rle1, stride, d->d_info,
                           d->d_blocks, (uint32_t)nb, d->d_cstate, d->d_olen, (const uint64_t*)nullptr,
                           (uint8_t*)nullptr, (uint64_t)0, d->d_crc, d->d_crctab, 0);
        DCHECK(hipGetLastError());
        DCHECK(hipMemcpyAsync(olen.data(), d->d_olen, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        DCHECK(hipStreamSynchronize(s));
        for (size_t i = 0; i < nb; ++i) ooff[i + 1] = ooff[i] + olen[i];
        if (ooff[nb] > cap) {
            *out_len = ooff[nb];
            return bz2mi_set_error(BZ2MI_ESPACE, "output buffer too small");
        }
        DCHECK(hipMemcpyAsync(d->d_ooff, ooff.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(dec_rle1_kernel, dim3((unsigned)nb), dim3(256), 0, s, d->d_rle1, stride, d->d_info,
                           d->d_blocks, (uint32_t)nb, d->d_cstate, d->d_olen, d->d_ooff, d_out, (uint64_t)cap, d->d_crc,
                           d->d_crctab, 1);
        DCHECK(hipGetLastError());
        DCHECK(hipMemcpyAsync(crc.data(), d->d_crc, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        DCHECK(hipMemcpyAsync(bad.data(), d->d_bad, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    } else {
        DCHECK(hipEventRecord(d->ev[4], s));
    }
    DCHECK(hipEventRecord(d->ev[5], s));
    DCHECK(hipStreamSynchronize(s));
    // ---- checks in stream order: block CRCs (BlockDecompressor::checkCRC
    // :101-109), stream CRCs (InputStream.hpp:136-143), then the first error
    // the walk stopped at
    size_t si = 0;
    uint32_t scrc = 0;
    for (size_t i = 0; i <= nb; ++i) {
        while (si < stream_end.size() && stream_end[si] == i) {
            if (scrc != stream_crc[si]) return bz2mi_set_error(BZ2MI_EFORMAT, "BZip2 stream CRC error");
            scrc = 0;
            si++;
        }
        if (i == nb) break;
        // (an inconsistent BWT -- `bad` -- yields garbage bytes: the reference
        // would find the same CRC mismatch)
        if ((bad[i] || crc[i] != chain_crc[i]) && !getenv("BZ2MI_DNOCRC")) {
            if (getenv("BZ2MI_DDUMP"))
                fprintf(stderr, "[bz2mi] block %zu: bad %u crc %08x stored %08x len %llu\n", i, bad[i], crc[i],
                        chain_crc[i], (unsigned long long)olen[i]);
            return bz2mi_set_error(BZ2MI_EFORMAT, "BZip2 block CRC error");
        }
        scrc = ((scrc << 1) | (scrc >> 31)) ^ crc[i];
    }
    if (err_status >= 0) return bz2mi_set_error(BZ2MI_EFORMAT, err_msg);
    *out_len = nb ? ooff[nb] : 0;
    float t;
    for (int k = 0; k < 5; ++k) d->ms[k] = hipEventElapsedTime(&t, d->ev[k], d->ev[k + 1]) == hipSuccess ? t : 0.f;
    d->ms[5] = hipEventElapsedTime(&t, d->ev[0], d->ev[5]) == hipSuccess ? t : 0.f;
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
                    (void*)d->d_marks, (void*)d->d_rle1, (void*)d->d_cstate, (void*)d->d_olen, (void*)d->d_ooff,
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

int bz2mi_dset_flags(bz2mi_dctx* d, int flags) {
    if (!d || (flags & ~BZ2MI_DEC_CONCATENATED)) return bz2mi_set_error(BZ2MI_EINVAL, "invalid decoder flags");
    d->flags = flags;
    return BZ2MI_OK;
}

int bz2mi_dlast_timings(bz2mi_dctx* d, float* ms6) {
    if (!d || !ms6) return bz2mi_set_error(BZ2MI_EINVAL, "null argument");
    for (int k = 0; k < 6; ++k) ms6[k] = d->ms[k];
    return BZ2MI_OK;
}

}  // extern "C"
