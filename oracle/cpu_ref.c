/* TEST INFRASTRUCTURE ONLY (oracle/): see cpu_ref.h.
 *
 * A from-scratch C restatement of the reference's compression path.  Every
 * stage cites the reference code it follows (paths relative to the reference
 * tree).  It is the checker for the HIP path and the CPU baseline; nothing in
 * the product links or calls it.
 */
#define _GNU_SOURCE
#include "cpu_ref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ CRC --
 * include/CRC32.hpp:30-92: MSB-first CRC-32, polynomial 0x04c11db7, table
 * driven, register initialised to all ones, complemented on output.  The
 * table is generated rather than listed. */
static uint32_t crc_table[256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;

static void crc_init(void) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i << 24;
        for (int k = 0; k < 8; ++k) c = (c & 0x80000000u) ? (c << 1) ^ 0x04c11db7u : (c << 1);
        crc_table[i] = c;
    }
}

uint32_t cpuref_crc_update(uint32_t crc, const uint8_t* p, size_t n) {
    pthread_once(&crc_once, crc_init);
    for (size_t i = 0; i < n; ++i) crc = (crc << 8) ^ crc_table[((crc >> 24) ^ p[i]) & 0xff];
    return crc;
}

/* ---------------------------------------------------------- bit writer --
 * Packed MSB-first equivalent of the bool-per-bit writers
 * (kernel.cpp:2459-2481, include/BitOutputStream.hpp:101-135). */
typedef struct {
    uint8_t* buf;
    uint64_t n;   /* bits written */
    uint64_t cap; /* capacity in bits */
    int overflow;
} bitw;

static void bw_bit(bitw* w, int b) {
    if (w->n >= w->cap) {
        w->overflow = 1;
        return;
    }
    uint64_t i = w->n >> 3;
    if ((w->n & 7) == 0) w->buf[i] = 0;
    if (b) w->buf[i] |= (uint8_t)(0x80u >> (w->n & 7));
    w->n++;
}

static void bw_bits(bitw* w, int count, uint32_t value) {
    for (int k = count - 1; k >= 0; --k) bw_bit(w, (value >> k) & 1u);
}

static void bw_int(bitw* w, uint32_t v) { bw_bits(w, 32, v); }

static void bw_unary(bitw* w, int v) {
    while (v-- > 0) bw_bit(w, 1);
    bw_bit(w, 0);
}

/* ---------------------------------------------------- RLE1 block split --
 * include/BlockCompressor.hpp:69-154 and OutputStream.hpp:131-142/179-188:
 * a byte is refused once more than S-6 RLE1 bytes have been flushed; runs are
 * cut into pieces of at most 255, a piece of length >= 4 is written as four
 * copies plus (length-4).  The pending run of a full block is flushed into it
 * (finishRLE, :112-118). */
typedef struct {
    uint8_t* blk;
    int len;
    int limit;
    int val;
    int run;
} rle1_state;

static void rle1_flush(rle1_state* s, int v, int run) {
    s->blk[s->len++] = (uint8_t)v;
    if (run > 1) {
        s->blk[s->len++] = (uint8_t)v;
        if (run > 2) {
            s->blk[s->len++] = (uint8_t)v;
            if (run > 3) {
                s->blk[s->len++] = (uint8_t)v;
                s->blk[s->len++] = (uint8_t)(run - 4);
            }
        }
    }
}

static int rle1_put(rle1_state* s, int v) {
    if (s->len > s->limit) return 0;
    if (s->run == 0) {
        s->val = v;
        s->run = 1;
    } else if (s->val == v) {
        if (++s->run > 254) {
            rle1_flush(s, s->val, 255);
            s->run = 0;
        }
    } else {
        rle1_flush(s, s->val, s->run);
        s->val = v;
        s->run = 1;
    }
    return 1;
}

long long cpuref_split(const uint8_t* in, size_t n, int S, uint8_t* blocks, size_t stride,
                       uint64_t* starts, uint32_t* lens, uint32_t* crcs, size_t max_blocks) {
    size_t nb = 0;
    size_t i = 0;
    while (i < n) {
        rle1_state s;
        s.blk = blocks ? blocks + (nb < max_blocks ? nb : 0) * stride : NULL;
        s.len = 0;
        s.limit = S - 6;
        s.run = 0;
        s.val = -1;
        size_t b0 = i;
        if (nb >= max_blocks || !blocks) {
            /* counting mode: run the state machine on a private buffer */
            static __thread uint8_t* tmp = NULL;
            static __thread int tmpcap = 0;
            if (tmpcap < S + 8) {
                free(tmp);
                tmp = (uint8_t*)malloc((size_t)S + 8);
                tmpcap = S + 8;
            }
            s.blk = tmp;
        }
        while (i < n && rle1_put(&s, in[i])) ++i;
        if (s.run > 0) rle1_flush(&s, s.val & 0xff, s.run);
        if (nb < max_blocks) {
            if (starts) starts[nb] = b0;
            if (lens) lens[nb] = (uint32_t)s.len;
            if (crcs) crcs[nb] = ~cpuref_crc_update(0xffffffffu, in + b0, i - b0);
        }
        nb++;
    }
    if (nb > max_blocks) return -(long long)nb;
    return (long long)nb;
}

/* ------------------------------------------------------------------ BWT --
 * kernel.cpp:2429-2456 (DivSufSortBWT on T with the wrap byte T[n]=T[0],
 * kernel.cpp:3113) computes the Burrows-Wheeler transform of the cyclic
 * rotations of the block and returns origPtr, the sorted rank of rotation 0.
 * The order of distinct rotations is unique, so any correct rotation sort
 * reproduces it; this one is prefix doubling with two stable counting sorts
 * per round.  Both sorts start from index order, so equal rotations (periodic
 * blocks only) stay in index order and rotation 0 gets the smallest rank among
 * its equals. */
int cpuref_bwt(const uint8_t* T, int n, uint8_t* bwt) {
    if (n <= 0) return 0;
    if (n == 1) { /* kernel.cpp:2434-2437 */
        bwt[0] = T[0];
        return 0;
    }
    int* sa = (int*)malloc(sizeof(int) * n);
    int* tmp = (int*)malloc(sizeof(int) * n);
    int* rank = (int*)malloc(sizeof(int) * n);
    int* nrank = (int*)malloc(sizeof(int) * n);
    int cntn = n > 256 ? n : 256;
    int* cnt = (int*)malloc(sizeof(int) * (cntn + 1));
    /* round 0: one character */
    memset(cnt, 0, sizeof(int) * 257);
    for (int i = 0; i < n; ++i) cnt[T[i] + 1]++;
    for (int c = 0; c < 256; ++c) cnt[c + 1] += cnt[c];
    for (int i = 0; i < n; ++i) sa[cnt[T[i]]++] = i;
    int groups = 0;
    for (int k = 0; k < n; ++k) {
        if (k > 0 && T[sa[k]] != T[sa[k - 1]]) groups++;
        rank[sa[k]] = groups;
    }
    groups++;
    for (long long h = 1; groups < n && h < n; h <<= 1) {
        /* stable counting sort of 0..n-1 by rank[(i+h) mod n] */
        memset(cnt, 0, sizeof(int) * (groups + 1));
        for (int i = 0; i < n; ++i) cnt[rank[(i + h) % n] + 1]++;
        for (int g = 0; g < groups; ++g) cnt[g + 1] += cnt[g];
        for (int i = 0; i < n; ++i) tmp[cnt[rank[(i + h) % n]]++] = i;
        /* stable counting sort by rank[i] */
        memset(cnt, 0, sizeof(int) * (groups + 1));
        for (int i = 0; i < n; ++i) cnt[rank[i] + 1]++;
        for (int g = 0; g < groups; ++g) cnt[g + 1] += cnt[g];
        for (int k = 0; k < n; ++k) {
            int i = tmp[k];
            sa[cnt[rank[i]]++] = i;
        }
        int g = 0;
        for (int k = 0; k < n; ++k) {
            if (k > 0) {
                int a = sa[k], b = sa[k - 1];
                if (rank[a] != rank[b] || rank[(a + h) % n] != rank[(b + h) % n]) g++;
            }
            nrank[sa[k]] = g;
        }
        groups = g + 1;
        int* t = rank;
        rank = nrank;
        nrank = t;
    }
    int orig = 0;
    for (int k = 0; k < n; ++k) {
        int i = sa[k];
        if (i == 0) orig = k;
        bwt[k] = T[i == 0 ? n - 1 : i - 1];
    }
    free(sa);
    free(tmp);
    free(rank);
    free(nrank);
    free(cnt);
    return orig;
}

/* ------------------------------------------------------------ MTF+RLE2 --
 * kernel.cpp:2561-2649 (MTFAndRLE2StageEncoder) with valueToFront
 * (kernel.cpp:2514-2533). */
static void emit_zero_run(int rep, uint16_t* out, int* j, uint32_t* runA, uint32_t* runB) {
    rep--;
    for (;;) {
        if ((rep & 1) == 0) {
            out[(*j)++] = 0;
            (*runA)++;
        } else {
            out[(*j)++] = 1;
            (*runB)++;
        }
        if (rep <= 1) break;
        rep = (rep - 2) >> 1;
    }
}

int cpuref_mtf(const uint8_t* bwt, int n, const uint8_t* present, uint16_t* mtf,
               uint32_t* hist, int* alpha) {
    uint8_t map[256], list[256];
    int k = 0;
    for (int i = 0; i < 256; ++i) {
        map[i] = 0;
        list[i] = (uint8_t)i;
        if (present[i]) map[i] = (uint8_t)k++;
    }
    memset(hist, 0, sizeof(uint32_t) * 258);
    int eob = k + 1;
    int j = 0, rep = 0;
    uint32_t runA = 0, runB = 0;
    for (int i = 0; i < n; ++i) {
        uint8_t v = map[bwt[i]];
        int pos = 0;
        if (list[0] != v) {
            uint8_t carry = list[0];
            list[0] = v;
            do {
                ++pos;
                uint8_t t = list[pos];
                list[pos] = carry;
                carry = t;
            } while (carry != v);
        }
        if (pos == 0) {
            rep++;
        } else {
            if (rep > 0) {
                emit_zero_run(rep, mtf, &j, &runA, &runB);
                rep = 0;
            }
            mtf[j++] = (uint16_t)(pos + 1);
            hist[pos + 1]++;
        }
    }
    if (rep > 0) emit_zero_run(rep, mtf, &j, &runA, &runB);
    mtf[j++] = (uint16_t)eob;
    hist[eob]++;
    hist[0] += runA;
    hist[1] += runB;
    *alpha = eob + 1;
    return j;
}

/* -------------------------------------------------------------- Huffman --
 * Length-limited code lengths: the in-place allocator of kernel.cpp:2652-2806
 * (jbzip2's HuffmanAllocator, after Moffat & Katajainen), restated. */
static int sig_bits(int x) {
    int n = 0;
    while (x > 0) {
        x >>= 1;
        n++;
    }
    return n;
}

static int ha_first(const int* a, int len, int i, int nodesToMove) {
    const int limit = i;
    int k = len - 2;
    while (i >= nodesToMove && (a[i] % len) > limit) {
        k = i;
        i -= (limit - i + 1);
    }
    if (i < nodesToMove - 1) i = nodesToMove - 1;
    while (k > i + 1) {
        int t = (i + k) >> 1;
        if ((a[t] % len) > limit) k = t;
        else i = t;
    }
    return k;
}

static void ha_parents(int* a, int len) {
    a[0] += a[1];
    for (int head = 0, tail = 1, top = 2; tail < len - 1; tail++) {
        int t;
        if (top >= len || a[head] < a[top]) {
            t = a[head];
            a[head++] = tail;
        } else {
            t = a[top++];
        }
        if (top >= len || (head < tail && a[head] < a[top])) {
            t += a[head];
            a[head++] = tail + len;
        } else {
            t += a[top++];
        }
        a[tail] = t;
    }
}

static int ha_relocate_count(const int* a, int len, int maxLen) {
    int cur = len - 2;
    for (int d = 1; d < maxLen - 1 && cur > 1; d++) cur = ha_first(a, len, cur - 1, 0);
    return cur;
}

static void ha_lengths(int* a, int len) {
    int firstNode = len - 2, nextNode = len - 1;
    for (int d = 1, avail = 2; avail > 0; d++) {
        int lastNode = firstNode;
        firstNode = ha_first(a, len, lastNode - 1, 0);
        for (int i = avail - (lastNode - firstNode); i > 0; i--) a[nextNode--] = d;
        avail = (lastNode - firstNode) << 1;
    }
}

static void ha_lengths_reloc(int* a, int len, int nodesToMove, int insertDepth) {
    int firstNode = len - 2, nextNode = len - 1;
    int d = (insertDepth == 1) ? 2 : 1;
    int left = (insertDepth == 1) ? nodesToMove - 2 : nodesToMove;
    for (int avail = d << 1; avail > 0; d++) {
        int lastNode = firstNode;
        if (firstNode > nodesToMove) firstNode = ha_first(a, len, lastNode - 1, nodesToMove);
        int off = 0;
        if (d >= insertDepth) {
            int cap = 1 << (d - insertDepth);
            off = left < cap ? left : cap;
        } else if (d == insertDepth - 1) {
            off = 1;
            if (a[firstNode] == lastNode) firstNode++;
        }
        for (int i = avail - (lastNode - firstNode + off); i > 0; i--) a[nextNode--] = d;
        left -= off;
        avail = (lastNode - firstNode + off) << 1;
    }
}

static void ha_allocate(int* a, int len, int maxLen) {
    if (len == 2) {
        a[1] = 1;
        a[0] = 1;
        return;
    }
    if (len == 1) {
        a[0] = 1;
        return;
    }
    ha_parents(a, len);
    int r = ha_relocate_count(a, len, maxLen);
    if ((a[0] % len) >= r) ha_lengths(a, len);
    else ha_lengths_reloc(a, len, r, maxLen - sig_bits(r - 1));
}

static int cmp_int(const void* x, const void* y) {
    int a = *(const int*)x, b = *(const int*)y;
    return (a > b) - (a < b);
}

/* kernel.cpp:2835-2857: sort keys (freq << 9) | symbol ascending (they are
 * unique, so the order does not depend on the sorting method), allocate,
 * scatter back. */
static void code_lengths(int alpha, const int* freq, int* lens) {
    int merged[258], sorted[258];
    for (int i = 0; i < alpha; ++i) merged[i] = (freq[i] << 9) | i;
    qsort(merged, alpha, sizeof(int), cmp_int);
    for (int i = 0; i < alpha; ++i) sorted[i] = merged[i] >> 9;
    ha_allocate(sorted, alpha, 20);
    for (int i = 0; i < alpha; ++i) lens[merged[i] & 0x1ff] = sorted[i];
}

static int table_count(int mtfLength) { /* kernel.cpp:2808-2818 */
    if (mtfLength >= 2400) return 6;
    if (mtfLength >= 1200) return 5;
    if (mtfLength >= 600) return 4;
    if (mtfLength >= 200) return 3;
    return 2;
}

/* int32 wrap-around arithmetic, as the reference's int array behaves. */
static inline int32_t wadd(int32_t a, uint32_t b) { return (int32_t)((uint32_t)a + b); }
static inline int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }

/* H3 as the reference behaves on an MI355X (tests/test_refgpu.py): the
 * uninitialised tableFrequencies (kernel.cpp:2902) starts at zero in a lane's
 * first block but is not cleared between the four optimisation passes. */
static int h3_accumulate = 0;
void cpuref_set_h3_accumulate(int on) { h3_accumulate = on; }

long long cpuref_block_payload(int origPtr, const uint8_t* present, const uint16_t* mtf,
                               int mtfLength, int alpha, const uint32_t* seed, uint8_t* out,
                               uint64_t cap_bits, uint8_t* sel_out, uint8_t* len_out) {
    bitw w = {out, 0, cap_bits, 0};
    /* kernel.cpp:3116 */
    bw_bits(&w, 24, (uint32_t)origPtr);
    /* writeSymbolMap, kernel.cpp:2483-2511 */
    int used16[16];
    for (int i = 0; i < 16; ++i) {
        used16[i] = 0;
        for (int j = 0; j < 16; ++j)
            if (present[i * 16 + j]) used16[i] = 1;
    }
    for (int i = 0; i < 16; ++i) bw_bit(&w, used16[i]);
    for (int i = 0; i < 16; ++i)
        if (used16[i])
            for (int j = 0; j < 16; ++j) bw_bit(&w, present[i * 16 + j] != 0);

    /* HuffmanStageEncoder, kernel.cpp:3064-3096 */
    const int T = table_count(mtfLength);
    const int nsel = (mtfLength + 49) / 50;
    static __thread int lens[6][258];
    static __thread int codes[6][258];
    uint8_t* sel = (uint8_t*)malloc((size_t)nsel + 1);
    memset(lens, 0, sizeof(lens));
    memset(codes, 0, sizeof(codes));

    /* generateHuffmanOptimisationSeeds, kernel.cpp:2859-2893 */
    {
        int32_t remaining = mtfLength;
        int lowEnd = -1;
        for (int i = 0; i < T; i++) {
            int32_t target = remaining / (T - i);
            int lowStart = lowEnd + 1;
            int32_t actual = 0;
            while (actual < target && lowEnd < alpha - 1) actual = wadd(actual, seed[++lowEnd]);
            if (lowEnd > lowStart && i != 0 && i != T - 1 && ((T - i) % 2) == 0)
                actual = wsub(actual, (int32_t)seed[lowEnd--]);
            for (int j = 0; j < alpha; j++)
                if (j < lowStart || j > lowEnd) lens[i][j] = 15;
            remaining = wsub(remaining, actual);
        }
    }
    /* 4x optimiseSelectorsAndHuffmanTables, kernel.cpp:2895-2951 */
    static __thread int tf[6][258];
    memset(tf, 0, sizeof(tf));
    for (int it = 3; it >= 0; it--) {
        if (!h3_accumulate) memset(tf, 0, sizeof(tf)); /* H3: zero-initialised per pass (O_ref) */
        int si = 0;
        for (int gs = 0; gs < mtfLength;) {
            int ge = (gs + 50 < mtfLength ? gs + 50 : mtfLength) - 1;
            int cost[6] = {0, 0, 0, 0, 0, 0};
            for (int i = gs; i <= ge; i++)
                for (int t = 0; t < T; t++) cost[t] += lens[t][mtf[i]];
            int best = 0, bestCost = cost[0];
            for (int t = 1; t < T; t++)
                if (cost[t] < bestCost) {
                    bestCost = cost[t];
                    best = t;
                }
            for (int i = gs; i <= ge; i++) tf[best][mtf[i]]++;
            if (it == 0) sel[si++] = (uint8_t)best;
            gs = ge + 1;
        }
        for (int t = 0; t < T; t++) code_lengths(alpha, tf[t], lens[t]);
    }
    /* assignHuffmanCodeSymbols, kernel.cpp:2953-2989 */
    for (int t = 0; t < T; t++) {
        int mn = 32, mx = 0;
        for (int j = 0; j < alpha; ++j) {
            if (lens[t][j] > mx) mx = lens[t][j];
            if (lens[t][j] < mn) mn = lens[t][j];
        }
        int code = 0;
        for (int L = mn; L <= mx; L++) {
            for (int k = 0; k < alpha; k++)
                if ((lens[t][k] & 0xff) == L) codes[t][k] = (L << 24) | code++;
            code <<= 1;
        }
    }
    /* writeSelectorsAndHuffmanTables, kernel.cpp:2991-3041 */
    bw_bits(&w, 3, (uint32_t)T);
    bw_bits(&w, 15, (uint32_t)nsel);
    {
        uint8_t lst[6] = {0, 1, 2, 3, 4, 5};
        for (int i = 0; i < nsel; i++) {
            int v = sel[i], pos = 0;
            while (lst[pos] != v) pos++;
            for (int q = pos; q > 0; q--) lst[q] = lst[q - 1];
            lst[0] = (uint8_t)v;
            bw_unary(&w, pos);
        }
    }
    for (int t = 0; t < T; ++t) {
        int cur = lens[t][0];
        bw_bits(&w, 5, (uint32_t)cur);
        for (int j = 0; j < alpha; j++) {
            int L = lens[t][j];
            uint32_t v = (cur < L) ? 2u : 3u;
            int d = L - cur;
            if (d < 0) d = -d;
            while (d-- > 0) bw_bits(&w, 2, v);
            bw_bit(&w, 0);
            cur = L;
        }
    }
    /* writeBlockData, kernel.cpp:3043-3062 */
    for (int i = 0, si = 0; i < mtfLength; si++) {
        int ge = (i + 50 < mtfLength ? i + 50 : mtfLength) - 1;
        const int* c = codes[sel[si]];
        for (; i <= ge; i++) {
            int m = c[mtf[i]];
            bw_bits(&w, m >> 24, (uint32_t)m & 0xffffffu);
        }
    }
    if (sel_out) memcpy(sel_out, sel, (size_t)nsel);
    if (len_out)
        for (int t = 0; t < 6; ++t)
            for (int j = 0; j < 258; ++j) len_out[t * 258 + j] = (uint8_t)(t < T && j < alpha ? lens[t][j] : 0);
    free(sel);
    if (w.overflow) return -1;
    return (long long)w.n;
}

/* --------------------------------------------------------------- stream -- */
size_t cpuref_bound(size_t n, int level, int unit) {
    size_t S = (size_t)unit * (size_t)level;
    size_t blocks = (n + n / 4) / (S - 5) + 2;
    size_t per = (S + 1) * 20 / 8 + (S / 50 + 2) + 6 * 258 * 5 + 1024;
    return 64 + blocks * per;
}

typedef struct {
    const uint8_t* in;
    const uint64_t* starts;
    const uint32_t* lens;
    uint8_t* blocks;
    size_t stride;
    uint8_t* bwt;
    uint16_t* mtf;     /* stride + 2 per block */
    uint32_t* hist;    /* 258 per block */
    int* mtflen;
    int* alpha;
    int* orig;
    uint8_t* present;  /* 256 per block */
    const uint32_t* seeds;
    uint8_t* payload;  /* payload_stride bytes per block */
    size_t payload_stride;
    long long* pbits;
    long long nb;
    int phase;
    long long next;
    pthread_mutex_t mu;
} job_t;

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        long long b = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (b >= j->nb) break;
        const uint8_t* blk = j->blocks + b * j->stride;
        int n = (int)j->lens[b];
        uint8_t* pres = j->present + b * 256;
        if (j->phase == 0) {
            memset(pres, 0, 256);
            for (int i = 0; i < n; ++i) pres[blk[i]] = 1;
            uint8_t* bw = j->bwt + b * j->stride;
            j->orig[b] = cpuref_bwt(blk, n, bw);
            j->mtflen[b] = cpuref_mtf(bw, n, pres, j->mtf + b * (j->stride + 2), j->hist + b * 258,
                                      &j->alpha[b]);
        } else {
            j->pbits[b] = cpuref_block_payload(j->orig[b], pres, j->mtf + b * (j->stride + 2),
                                               j->mtflen[b], j->alpha[b], j->seeds + b * 258,
                                               j->payload + b * j->payload_stride,
                                               (uint64_t)j->payload_stride * 8, NULL, NULL);
        }
    }
    return NULL;
}

static void run_pool(job_t* j, int threads) {
    j->next = 0;
    if (threads <= 1) {
        worker(j);
        return;
    }
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, j);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
}

static void put_bits_from(bitw* w, const uint8_t* src, uint64_t nbits) {
    /* append nbits MSB-first bits of src; byte-fast when aligned */
    uint64_t i = 0;
    while (i < nbits && (w->n & 7)) {
        bw_bit(w, (src[i >> 3] >> (7 - (i & 7))) & 1);
        i++;
    }
    if (i < nbits && (i & 7) == 0) {
        uint64_t whole = (nbits - i) >> 3;
        if (w->n + whole * 8 <= w->cap) {
            memcpy(w->buf + (w->n >> 3), src + (i >> 3), whole);
            w->n += whole * 8;
            i += whole * 8;
        }
    } else if (i < nbits) {
        /* w aligned, src not: shift */
        uint64_t sh = i & 7;
        while (i + 8 <= nbits && w->n + 8 <= w->cap) {
            uint64_t byte = i >> 3;
            uint8_t v = (uint8_t)((src[byte] << sh) | (src[byte + 1] >> (8 - sh)));
            w->buf[w->n >> 3] = v;
            w->n += 8;
            i += 8;
        }
    }
    for (; i < nbits; ++i) bw_bit(w, (src[i >> 3] >> (7 - (i & 7))) & 1);
}

long long cpuref_compress(const uint8_t* in, size_t n, int level, int p, int unit, uint8_t* out,
                          size_t cap, int threads) {
    if (level < 1 || level > 9 || p < 1 || unit < 10) return -1;
    const int S = unit * level;
    long long nb = cpuref_split(in, n, S, NULL, 0, NULL, NULL, NULL, 0);
    nb = nb < 0 ? -nb : nb;
    size_t stride = (size_t)S + 8;
    uint8_t* blocks = (uint8_t*)malloc(nb * stride + 1);
    uint64_t* starts = (uint64_t*)malloc(sizeof(uint64_t) * (nb + 1));
    uint32_t* lens = (uint32_t*)malloc(sizeof(uint32_t) * (nb + 1));
    uint32_t* crcs = (uint32_t*)malloc(sizeof(uint32_t) * (nb + 1));
    cpuref_split(in, n, S, blocks, stride, starts, lens, crcs, (size_t)nb);

    job_t j;
    memset(&j, 0, sizeof(j));
    pthread_mutex_init(&j.mu, NULL);
    j.in = in;
    j.starts = starts;
    j.lens = lens;
    j.blocks = blocks;
    j.stride = stride;
    j.nb = nb;
    j.bwt = (uint8_t*)malloc(nb * stride + 1);
    j.mtf = (uint16_t*)malloc(sizeof(uint16_t) * nb * (stride + 2) + 2);
    j.hist = (uint32_t*)malloc(sizeof(uint32_t) * 258 * (nb + 1));
    j.mtflen = (int*)malloc(sizeof(int) * (nb + 1));
    j.alpha = (int*)malloc(sizeof(int) * (nb + 1));
    j.orig = (int*)malloc(sizeof(int) * (nb + 1));
    j.present = (uint8_t*)malloc(256 * (nb + 1));
    j.phase = 0;
    run_pool(&j, threads);

    /* H4: block b seeds from the running sum over blocks b' <= b with
     * b' == b (mod p) -- the never-cleared per-slot frequency array of the
     * reference (OutputStream.hpp:93, kernel.cpp:2613,2641-2643). */
    uint32_t* seeds = (uint32_t*)malloc(sizeof(uint32_t) * 258 * (nb + 1));
    for (long long b = 0; b < nb; ++b)
        for (int s = 0; s < 258; ++s)
            seeds[b * 258 + s] = j.hist[b * 258 + s] + (b >= p ? seeds[(b - p) * 258 + s] : 0u);
    j.seeds = seeds;
    j.payload_stride = (size_t)S * 20 / 8 + S / 50 + 8 * 1024;
    j.payload = (uint8_t*)malloc(j.payload_stride * nb + 1);
    j.pbits = (long long*)malloc(sizeof(long long) * (nb + 1));
    j.phase = 1;
    run_pool(&j, threads);

    /* framing: OutputStream.hpp:126-128, :192-213, :163-176 -- the leftover
     * carry of BitOutputStream.hpp:30-99 makes the stream a plain bit
     * concatenation. */
    bitw w = {out, 0, (uint64_t)cap * 8, 0};
    bw_bits(&w, 16, 0x425a);
    bw_bits(&w, 8, 0x68);
    bw_bits(&w, 8, (uint32_t)('0' + level));
    uint32_t streamCRC = 0;
    long long ret = 0;
    for (long long b = 0; b < nb; ++b) {
        if (j.pbits[b] < 0) {
            ret = -2;
            break;
        }
        streamCRC = ((streamCRC << 1) | (streamCRC >> 31)) ^ crcs[b];
        bw_bits(&w, 24, 0x314159);
        bw_bits(&w, 24, 0x265359);
        bw_int(&w, crcs[b]);
        bw_bit(&w, 0);
        put_bits_from(&w, j.payload + b * j.payload_stride, (uint64_t)j.pbits[b]);
    }
    if (ret == 0) {
        bw_bits(&w, 24, 0x177245);
        bw_bits(&w, 24, 0x385090);
        bw_int(&w, streamCRC);
        while (w.n & 7) bw_bit(&w, 0);
        ret = w.overflow ? -2 : (long long)(w.n >> 3);
    }
    free(blocks);
    free(starts);
    free(lens);
    free(crcs);
    free(j.bwt);
    free(j.mtf);
    free(j.hist);
    free(j.mtflen);
    free(j.alpha);
    free(j.orig);
    free(j.present);
    free(seeds);
    free(j.payload);
    free(j.pbits);
    pthread_mutex_destroy(&j.mu);
    return ret;
}

/* ---------------------------------------------------------- stream units --
 * The block chain from `entry` (a block start: the RLE1 state restarts there,
 * BlockCompressor.hpp:120-131) until the next start lies at or past n_own;
 * blocks then go through the same stages as cpuref_compress, with stream block
 * indices first_block.. for the seed slots (H4) and the stream CRC / bit
 * offsets supplied by the caller (OutputStream.hpp:190-240, :202). */
struct cpuref_unit {
    int level, p, S;
    long long nb;
    uint64_t first_block;
    uint32_t* crcs;
    job_t j;
    uint32_t* seeds;
};

#define UNIT_MIDRUN (1ull << 63)

cpuref_unit* cpuref_unit_open(const uint8_t* buf, size_t n_own, size_t n_halo, int ends, int level, int p,
                              int unit, uint64_t entry, uint64_t first_block, uint64_t* exit_entry,
                              uint64_t* nblocks, int threads) {
    if (level < 1 || level > 9 || p < 1 || unit < 10 || n_own == 0 || !exit_entry || !nblocks) return NULL;
    const int S = unit * level;
    const size_t n = n_own + n_halo;
    cpuref_unit* u = (cpuref_unit*)calloc(1, sizeof(cpuref_unit));
    u->level = level;
    u->p = p;
    u->S = S;
    u->first_block = first_block;
    size_t pos = (size_t)(entry & ~UNIT_MIDRUN);
    /* pass 1: count the blocks; pass 2: emit them */
    size_t cap = (n_own + n_own / 4) / (size_t)(S - 5) + 4;
    size_t stride = (size_t)S + 8;
    uint8_t* blocks = (uint8_t*)malloc(cap * stride + 1);
    uint64_t* starts = (uint64_t*)malloc(sizeof(uint64_t) * (cap + 1));
    uint32_t* lens = (uint32_t*)malloc(sizeof(uint32_t) * (cap + 1));
    u->crcs = (uint32_t*)malloc(sizeof(uint32_t) * (cap + 1));
    long long nb = 0;
    int bad = 0;
    while (pos < n_own) {
        if ((size_t)nb >= cap) {
            bad = 1;
            break;
        }
        rle1_state s;
        s.blk = blocks + nb * stride;
        s.len = 0;
        s.limit = S - 6;
        s.run = 0;
        s.val = -1;
        size_t i = pos;
        while (i < n && rle1_put(&s, buf[i])) ++i;
        if (i >= n && !ends) {
            bad = 1; /* the block runs past the halo */
            break;
        }
        if (s.run > 0) rle1_flush(&s, s.val & 0xff, s.run);
        starts[nb] = pos;
        lens[nb] = (uint32_t)s.len;
        u->crcs[nb] = ~cpuref_crc_update(0xffffffffu, buf + pos, i - pos);
        nb++;
        pos = i;
    }
    if (bad) {
        free(blocks);
        free(starts);
        free(lens);
        free(u->crcs);
        free(u);
        return NULL;
    }
    if (pos >= n_own) {
        const int mid = pos > 0 && pos < n && buf[pos] == buf[pos - 1];
        *exit_entry = (uint64_t)(pos - n_own) | (mid ? UNIT_MIDRUN : 0);
    }
    if (nb == 0) *exit_entry = ((entry & ~UNIT_MIDRUN) - n_own) | (entry & UNIT_MIDRUN);
    *nblocks = (uint64_t)nb;
    u->nb = nb;
    job_t* j = &u->j;
    memset(j, 0, sizeof(*j));
    pthread_mutex_init(&j->mu, NULL);
    j->in = buf;
    j->starts = starts;
    j->lens = lens;
    j->blocks = blocks;
    j->stride = stride;
    j->nb = nb;
    j->bwt = (uint8_t*)malloc(nb * stride + 1);
    j->mtf = (uint16_t*)malloc(sizeof(uint16_t) * nb * (stride + 2) + 2);
    j->hist = (uint32_t*)malloc(sizeof(uint32_t) * 258 * (nb + 1));
    j->mtflen = (int*)malloc(sizeof(int) * (nb + 1));
    j->alpha = (int*)malloc(sizeof(int) * (nb + 1));
    j->orig = (int*)malloc(sizeof(int) * (nb + 1));
    j->present = (uint8_t*)malloc(256 * (nb + 1));
    j->phase = 0;
    if (nb) run_pool(j, threads);
    return u;
}

void cpuref_unit_sums(const cpuref_unit* u, uint32_t* sums) {
    memset(sums, 0, sizeof(uint32_t) * 258 * (size_t)u->p);
    for (long long b = 0; b < u->nb; ++b) {
        const int slot = (int)((u->first_block + (uint64_t)b) % (uint64_t)u->p);
        for (int s = 0; s < 258; ++s) sums[slot * 258 + s] += u->j.hist[b * 258 + s];
    }
}

int cpuref_unit_encode(cpuref_unit* u, const uint32_t* carried, uint64_t* bits, uint32_t* crc, int threads) {
    const long long nb = u->nb;
    job_t* j = &u->j;
    free(u->seeds);
    u->seeds = (uint32_t*)malloc(sizeof(uint32_t) * 258 * (nb + 1));
    uint32_t* acc = (uint32_t*)malloc(sizeof(uint32_t) * 258 * (size_t)u->p);
    memcpy(acc, carried, sizeof(uint32_t) * 258 * (size_t)u->p);
    for (long long b = 0; b < nb; ++b) {
        const int slot = (int)((u->first_block + (uint64_t)b) % (uint64_t)u->p);
        for (int s = 0; s < 258; ++s) {
            acc[slot * 258 + s] += j->hist[b * 258 + s];
            u->seeds[b * 258 + s] = acc[slot * 258 + s];
        }
    }
    free(acc);
    j->seeds = u->seeds;
    j->payload_stride = (size_t)u->S * 20 / 8 + u->S / 50 + 8 * 1024;
    free(j->payload);
    free(j->pbits);
    j->payload = (uint8_t*)malloc(j->payload_stride * nb + 1);
    j->pbits = (long long*)malloc(sizeof(long long) * (nb + 1));
    j->phase = 1;
    if (nb) run_pool(j, threads);
    uint64_t tot = 0;
    uint32_t x = 0;
    for (long long b = 0; b < nb; ++b) {
        if (j->pbits[b] < 0) return -2;
        tot += 81 + (uint64_t)j->pbits[b];
        const uint32_t r = (uint32_t)(nb - 1 - b) & 31u;
        x ^= r ? (u->crcs[b] << r) | (u->crcs[b] >> (32 - r)) : u->crcs[b];
    }
    *bits = tot;
    *crc = x;
    return 0;
}

long long cpuref_unit_assemble(const cpuref_unit* u, uint64_t bit_offset, uint32_t crc_before, int flags,
                               uint8_t* out, size_t cap) {
    const job_t* j = &u->j;
    bitw w = {out, 0, (uint64_t)cap * 8, 0};
    if (flags & 1) {
        bw_bits(&w, 16, 0x425a);
        bw_bits(&w, 8, 0x68);
        bw_bits(&w, 8, (uint32_t)('0' + u->level));
    } else {
        for (uint64_t k = 0; k < (bit_offset & 7); ++k) bw_bit(&w, 0);
    }
    uint32_t streamCRC = crc_before;
    for (long long b = 0; b < u->nb; ++b) {
        streamCRC = ((streamCRC << 1) | (streamCRC >> 31)) ^ u->crcs[b];
        bw_bits(&w, 24, 0x314159);
        bw_bits(&w, 24, 0x265359);
        bw_int(&w, u->crcs[b]);
        bw_bit(&w, 0);
        put_bits_from(&w, j->payload + b * j->payload_stride, (uint64_t)j->pbits[b]);
    }
    if (flags & 2) {
        bw_bits(&w, 24, 0x177245);
        bw_bits(&w, 24, 0x385090);
        bw_int(&w, streamCRC);
    }
    const uint64_t nbits = w.n;
    while (w.n & 7) bw_bit(&w, 0);
    if (w.overflow) return -2;
    return (long long)((nbits + 7) >> 3);
}

void cpuref_unit_free(cpuref_unit* u) {
    if (!u) return;
    job_t* j = &u->j;
    free((void*)j->starts);
    free((void*)j->lens);
    free(j->blocks);
    free(j->bwt);
    free(j->mtf);
    free(j->hist);
    free(j->mtflen);
    free(j->alpha);
    free(j->orig);
    free(j->present);
    free(j->payload);
    free(j->pbits);
    free(u->seeds);
    free(u->crcs);
    pthread_mutex_destroy(&j->mu);
    free(u);
}
