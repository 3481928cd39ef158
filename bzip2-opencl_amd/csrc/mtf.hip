// Move-to-front + RLE2 (zero-run RUNA/RUNB coding) on the device.
//
// Restates MTFAndRLE2StageEncoder / valueToFront (reference
// kernel.cpp:2514-2533, 2561-2649) with exact sequential semantics, but
// chunk-parallel: one 64-lane wave per block, lane c owns chunk c.
//   1. recency pass: lane c scans its chunk backwards and records the distinct
//      bytes in order of last occurrence (the front of any MTF list after the
//      chunk), plus the chunk's byte set.
//   2. list build: the MTF list at the start of chunk c is the recency lists of
//      chunks c-1, c-2, ... merged (first occurrence wins), followed by the
//      block's remaining symbols in ascending order -- the reference's identity
//      initial list restricted to the symbols in use (symbol map, :2565-2572).
//   3. MTF pass: lane-serial move-to-front over a byte list in LDS, fused
//      search-and-shift on 32-bit words; ranks go to a byte scratch array and
//      the lane records its zero-run boundary state and histogram.
//   4. a wave scan assigns every zero run to the lane where it starts and
//      computes each lane's output offset; lanes then emit RUNA/RUNB digits
//      (bijective base 2, :2585-2606) and rank+1 symbols, and lane 63 the EOB.
// The per-block histogram of the emitted symbols (258 bins) is what the
// reference adds into its persistent frequency array (:2613, :2641-2643).
#include "common.hpp"
#include "kernels.hpp"

namespace bz2mi {

namespace {

constexpr int NL = 64;

struct MtfShared {
    uint32_t mask[NL][8];     // per-lane byte set
    uint32_t present[8];
    uint32_t hist[kMaxAlpha];
};

__device__ __forceinline__ void run_digits(uint32_t r, uint32_t& a, uint32_t& b, uint32_t& nd) {
    uint32_t rep = r - 1;
    for (;;) {
        if ((rep & 1u) == 0) a++;
        else b++;
        nd++;
        if (rep <= 1) break;
        rep = (rep - 2) >> 1;
    }
}

__device__ __forceinline__ void emit_run(uint32_t r, uint16_t* out, uint32_t& o) {
    uint32_t rep = r - 1;
    for (;;) {
        out[o++] = (uint16_t)(rep & 1u);  // RUNA = 0, RUNB = 1
        if (rep <= 1) break;
        rep = (rep - 2) >> 1;
    }
}


// Result of one lane's MTF pass over its chunk (zero-run boundary state).
struct LaneRun {
    uint32_t zl, zt, nz, idig, ia, ib;
    bool seen_nz;
};

// Lane-serial move-to-front over [c0, c1) with the list held in W registers
// (W*4 >= alphabet).  Per symbol, two passes over the list words:
//   search: SWAR zero-byte test of word ^ v*0x01010101; the first word with a
//     match gives the position (fw, byte); stops once every lane has found
//     its symbol;
//   shift: words before fw move up one byte (v_alignbyte with the previous
//     word), word fw is merged up to the match (v_perm with a per-symbol
//     selector), later words stay; stops after the largest fw of the wave.
// The wave-uniform bounds make text (small ranks) cheap; random data costs
// about 11 VALU per list word.
template <int W>
__device__ void mtf_pass(const uint32_t* Lw, const uint8_t* __restrict__ X, uint8_t* __restrict__ R, int c0, int c1,
                         uint32_t* hist, LaneRun& st) {
    uint32_t L[W];
#pragma unroll
    for (int j = 0; j < W; ++j) L[j] = Lw[j];
    uint32_t run = 0;
    const int ntile = (int)uniform((uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max((uint32_t)((c1 - c0 + 15) >> 4)), 63));
    // tiles of 16 symbols: one 16-byte load of X, one 16-byte store of ranks
    for (int tile = 0; tile < ntile; ++tile) {
        const int base = c0 + tile * 16;
        uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;
        if (base < c1) {
            const uint4 xin = *reinterpret_cast<const uint4*>(X + base);
            x0 = xin.x;
            x1 = xin.y;
            x2 = xin.z;
            x3 = xin.w;
        }
        uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, rc = 0;
        for (int q = 0; q < 16; ++q) {
            const bool live = base + q < c1;
            const uint32_t v = x0 & 0xffu;
            x0 >>= 8;
            const uint32_t vv = v * 0x01010101u;
            // ---- search: first word holding v.  Wide lists (random-like data)
            // scan every word, last to first, so the first hit simply wins;
            // narrower ones scan forward and stop once every lane has found.
            int fw = -1;
            uint32_t zf = 0;
            if constexpr (W == 64) {
#pragma unroll
                for (int j = W - 1; j >= 0; --j) {
                    const uint32_t xx = L[j] ^ vv;
                    const uint32_t z = (xx - 0x01010101u) & ~xx & 0x80808080u;
                    fw = z ? j : fw;
                    zf = z ? z : zf;
                }
                if (!live) fw = -1;
            } else {
                bool found = !live;
#pragma unroll
                for (int g = 0; g < W / 8; ++g) {
                    if (__ballot(!found)) {  // wave-uniform early exit
#pragma unroll
                        for (int jj = 0; jj < 8; ++jj) {
                            const int j = g * 8 + jj;
                            const uint32_t xx = L[j] ^ vv;
                            const uint32_t z = (xx - 0x01010101u) & ~xx & 0x80808080u;
                            const bool hit = (z != 0u) && !found;
                            fw = hit ? j : fw;
                            zf = hit ? z : zf;
                            found = found || (z != 0u);
                        }
                    }
                }
            }
            const uint32_t qb = (uint32_t)__builtin_ctz(zf | 0x80000000u) >> 3;  // byte of the match
            // ---- shift: v_perm byte selects (0-3 = previous word, 4-7 = this word):
            // words before fw move up one byte, word fw up to byte qb, later words stay
            constexpr uint32_t keep = 0x07060504u, full = 0x06050403u;
            const uint32_t qmask = qb >= 3 ? 0xffffffffu : ((1u << (8 * (qb + 1))) - 1u);
            const uint32_t selq = (full & qmask) | (keep & ~qmask);
            const int top = (int)__builtin_amdgcn_readlane((int)wave_incl_max((uint32_t)(fw + 1)), 63) - 1;
            uint32_t prev = v << 24;
            uint32_t state = fw >= 0 ? full : keep;
#pragma unroll
            for (int g = 0; g < W / 8; ++g) {
                if (g * 8 <= top) {  // wave-uniform bound: the largest fw
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        const int j = g * 8 + jj;
                        const uint32_t w = L[j];
                        const bool at = j == fw;
                        const uint32_t sel = at ? selq : state;  // full before fw, keep after
                        state = at ? keep : state;
                        L[j] = __builtin_amdgcn_perm(w, prev, sel);
                        prev = w;
                    }
                }
            }
            const uint32_t pos = live ? 4u * (uint32_t)fw + qb : 0u;
            rc |= pos << ((q & 3) * 8);
            if ((q & 3) == 3) {  // (uniform) next source / result dword
                x0 = x1;
                x1 = x2;
                x2 = x3;
                r0 = r1;
                r1 = r2;
                r2 = r3;
                r3 = rc;
                rc = 0;
            }
            if (live) {
                if (pos == 0) {
                    run++;
                } else {
                    if (run > 0) {
                        if (st.seen_nz) run_digits(run, st.ia, st.ib, st.idig);
                        else st.zl = run;
                        run = 0;
                    }
                    st.seen_nz = true;
                    st.nz++;
                    atomicAdd(&hist[pos + 1], 1u);
                }
            }
        }
        if (base < c1) *reinterpret_cast<uint4*>(R + base) = make_uint4(r0, r1, r2, r3);
    }
    if (run > 0) {
        st.zt = run;
        if (!st.seen_nz) st.zl = run;
    }
}

}  // namespace

BZ2MI_PHASE_TABLE(g_mtf_phase)

int mtf_phases(unsigned long long* out) {
#ifdef BZ2MI_PHASES
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mtf_phase), sizeof(unsigned long long) * 16) == hipSuccess ? 16 : -1;
#else
    (void)out;
    return 0;
#endif
}

__global__ __launch_bounds__(64) void mtf_kernel(const uint8_t* __restrict__ bwt, size_t stride,
                                                 const uint32_t* __restrict__ lens, int nblocks,
                                                 uint8_t* __restrict__ ranks, uint8_t* __restrict__ rec,
                                                 uint16_t* __restrict__ mtf_out, size_t mtf_stride,
                                                 uint32_t* __restrict__ mtf_len, uint32_t* __restrict__ alpha_out,
                                                 uint32_t* __restrict__ hist_out,
                                                 uint32_t* __restrict__ present_out) {
    __shared__ MtfShared sh;
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    const int c = threadIdx.x;  // lane == chunk
    const int n = (int)lens[b];
    const uint8_t* X = bwt + (size_t)b * stride;
    uint8_t* R = ranks + (size_t)b * stride;
    // per block: 64 initial MTF lists (256 bytes each) in global scratch
    // (the recency lists live in LDS)
    uint16_t* out = mtf_out + (size_t)b * mtf_stride;
    [[maybe_unused]] const bool stamp = b == nblocks / 2;
    BZ2MI_PHASE(g_mtf_phase, 0, stamp);

    int L = (n + NL - 1) / NL;
    L = (L + 15) & ~15;  // 16-byte tiles
    const int c0 = min(c * L, n);
    const int c1 = min(c0 + L, n);

    // ---- 1. recency lists (backwards scan)
    for (int q = 0; q < 8; ++q) sh.mask[c][q] = 0;
    for (int s = c; s < kMaxAlpha; s += NL) sh.hist[s] = 0;
    int rcnt = 0;
    uint4* myrec = reinterpret_cast<uint4*>(rec + ((size_t)b * NL * 2 + c) * 256);
    uint32_t rb0 = 0, rb1 = 0, rb2 = 0, rb3 = 0;  // 16 pending list bytes
    for (int base = c0 + (((c1 - c0 + 15) >> 4) - 1) * 16; base >= c0; base -= 16) {
        const uint4 xin = *reinterpret_cast<const uint4*>(X + base);
        const uint32_t xw[4] = {xin.x, xin.y, xin.z, xin.w};
#pragma unroll
        for (int q = 15; q >= 0; --q) {
            if (base + q >= c1) continue;
            const uint32_t v = (xw[q >> 2] >> ((q & 3) * 8)) & 0xffu;
            const uint32_t bit = 1u << (v & 31);
            const uint32_t m = sh.mask[c][v >> 5];
            if (!(m & bit)) {
                sh.mask[c][v >> 5] = m | bit;
                const int sl = rcnt & 15;
                const uint32_t add = v << ((sl & 3) * 8);
                rb0 |= sl < 4 ? add : 0u;
                rb1 |= (sl >> 2) == 1 ? add : 0u;
                rb2 |= (sl >> 2) == 2 ? add : 0u;
                rb3 |= (sl >> 2) == 3 ? add : 0u;
                if (sl == 15) {
                    myrec[rcnt >> 4] = make_uint4(rb0, rb1, rb2, rb3);
                    rb0 = rb1 = rb2 = rb3 = 0;
                }
                rcnt++;
            }
        }
    }
    if (rcnt & 15) myrec[rcnt >> 4] = make_uint4(rb0, rb1, rb2, rb3);
    __syncthreads();
    if (c < 8) {
        uint32_t p = 0;
        for (int l = 0; l < NL; ++l) p |= sh.mask[l][c];
        sh.present[c] = p;
    }
    // recency counts are the popcounts of the lane masks
    __syncthreads();
    int k = 0;
    for (int q = 0; q < 8; ++q) k += __popc(sh.present[q]);
    k = (int)uniform((uint32_t)k);

    BZ2MI_PHASE(g_mtf_phase, 1, stamp);
    // ---- 2. initial list of chunk c
    uint32_t seen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t* Lw = (uint32_t*)(rec + ((size_t)b * NL * 2 + NL + c) * 256);
    int len = 0;
    uint32_t word = 0;
    auto push = [&](uint32_t v) {
        word |= v << ((len & 3) * 8);
        if ((len & 3) == 3) {
            Lw[len >> 2] = word;
            word = 0;
        }
        len++;
    };
    for (int cc = c - 1; cc >= 0 && len < k; --cc) {
        const uint4* r4 = reinterpret_cast<const uint4*>(rec + ((size_t)b * NL * 2 + cc) * 256);
        int cnt = 0;
        for (int q = 0; q < 8; ++q) cnt += __popc(sh.mask[cc][q]);
        uint32_t rw[4] = {0, 0, 0, 0};
        for (int j = 0; j < cnt; ++j) {
            if ((j & 15) == 0) {
                const uint4 t4 = r4[j >> 4];
                rw[0] = t4.x;
                rw[1] = t4.y;
                rw[2] = t4.z;
                rw[3] = t4.w;
            }
            const uint32_t v = rw[0] & 0xffu;  // consumed front to back
            rw[0] >>= 8;
            if ((j & 3) == 3) {
                rw[0] = rw[1];
                rw[1] = rw[2];
                rw[2] = rw[3];
            }
            const uint32_t bit = 1u << (v & 31);
            bool had = false;
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q == (int)(v >> 5)) {
                    had = (seen[q] & bit) != 0;
                    seen[q] |= bit;
                }
            if (!had) push(v);
        }
    }
    for (int q = 0; q < 8; ++q) {
        uint32_t rest = sh.present[q] & ~seen[q];
        while (rest) {
            const int z = __ffs(rest) - 1;
            rest &= rest - 1;
            push((uint32_t)(q * 32 + z));
        }
    }
    if (len & 3) Lw[len >> 2] = word;

    __syncthreads();
    BZ2MI_PHASE(g_mtf_phase, 2, stamp);
    // ---- 3. MTF pass (list in registers; W words cover the k symbols in use)
    LaneRun st{0, 0, 0, 0, 0, 0, false};
    if (k <= 32) mtf_pass<8>(Lw, X, R, c0, c1, sh.hist, st);
    else if (k <= 64) mtf_pass<16>(Lw, X, R, c0, c1, sh.hist, st);
    else if (k <= 128) mtf_pass<32>(Lw, X, R, c0, c1, sh.hist, st);
    else mtf_pass<64>(Lw, X, R, c0, c1, sh.hist, st);
    const uint32_t zl = st.zl, zt = st.zt, nz = st.nz, idig = st.idig, ia = st.ia, ib = st.ib;
    const bool seen_nz = st.seen_nz;
    uint32_t run;
    __syncthreads();
    BZ2MI_PHASE(g_mtf_phase, 3, stamp);
    // ---- 4. zero-run ownership and offsets
    const int clen = c1 - c0;
    const uint32_t firstnz = seen_nz ? (uint32_t)(c0 + zl) : (uint32_t)n;
    // next nonzero strictly after this chunk: suffix min over lanes c+1..
    uint32_t nxt = firstnz;
    for (int d = 1; d < NL; d <<= 1) {
        uint32_t y = __shfl_down(nxt, d);
        if (c + d < NL) nxt = nxt < y ? nxt : y;
    }
    uint32_t after = __shfl_down(nxt, 1);
    if (c == NL - 1) after = (uint32_t)n;
    const uint32_t prev_zt = __shfl_up(zt, 1);
    const bool prev_ends_zero = c > 0 && prev_zt > 0;
    uint32_t bdig = 0, ba = 0, bb = 0;
    uint32_t lead_len = 0, tail_len = 0;
    bool own_lead = false;
    if (clen > 0) {
        if (!seen_nz) {
            if (!prev_ends_zero) {  // an all-zero chunk that starts a run
                own_lead = true;
                lead_len = after - (uint32_t)c0;
                run_digits(lead_len, ba, bb, bdig);
            }
        } else {
            if (zl > 0 && !prev_ends_zero) {
                own_lead = true;
                lead_len = zl;
                run_digits(lead_len, ba, bb, bdig);
            }
            if (zt > 0) {
                tail_len = after - (uint32_t)(c1 - zt);
                run_digits(tail_len, ba, bb, bdig);
            }
        }
    }
    const uint32_t cnt = nz + idig + bdig;
    const uint32_t incl = wave_incl_sum(cnt);
    const uint32_t off = incl - cnt;
    const uint32_t total = __shfl(incl, NL - 1);
    const uint32_t runA = wave_sum(ia + ba), runB = wave_sum(ib + bb);

    // ---- 5. emission
    uint32_t o = off;
    if (clen > 0) {
        run = 0;
        int i = c0;
        if (!own_lead && (zl > 0 || !seen_nz)) i = c0 + (int)zl;  // tail of an earlier lane's run
        bool lead = own_lead;
        const int i0 = i;
        for (int base = i0 & ~15; base < c1; base += 16) {  // 16-byte tiles of ranks
            const uint4 rin = *reinterpret_cast<const uint4*>(R + base);
            const uint32_t rw[4] = {rin.x, rin.y, rin.z, rin.w};
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                if (base + q < i0 || base + q >= c1) continue;
                const uint32_t r = (rw[q >> 2] >> ((q & 3) * 8)) & 0xffu;
                if (r == 0) {
                    run++;
                } else {
                    if (run > 0) {
                        emit_run(lead ? lead_len : run, out, o);
                        run = 0;
                    }
                    lead = false;
                    out[o++] = (uint16_t)(r + 1);
                }
            }
        }
        if (run > 0) emit_run(lead ? lead_len : tail_len, out, o);
    }
    __syncthreads();
    BZ2MI_PHASE(g_mtf_phase, 4, stamp);
    const uint32_t eob = (uint32_t)k + 1;
    if (c == NL - 1) {
        out[total] = (uint16_t)eob;
        mtf_len[b] = total + 1;
        alpha_out[b] = eob + 1;
    }
    uint32_t* H = hist_out + (size_t)b * kMaxAlpha;
    for (int s = c; s < kMaxAlpha; s += NL) {
        uint32_t h = sh.hist[s];
        if (s == 0) h += runA;
        if (s == 1) h += runB;
        if ((uint32_t)s == eob) h += 1;
        H[s] = h;
    }
    if (c < 8) present_out[(size_t)b * 8 + c] = sh.present[c];
}

}  // namespace bz2mi
