/*
 * bm_scan16.c -- 16-lane AVX-512 restatement of the miner's min-scan.
 * TEST INFRASTRUCTURE ONLY (see bm_oracle.h): it exists to make golden
 * answers for ranges too long for the byte-at-a-time oracle (the 2^35-nonce
 * weak-scaling ranges and the 2^40-nonce C4 range), and is itself checked
 * against oracle_search() and hashlib before its answers are used
 * (tests/test_oracle.py, tests/golden/make_golden.py).
 *
 * Reference behaviour restated:
 *   hash.go:11-15   Hash(msg, nonce) = BigEndian.Uint64(sha256(Sprintf("%s %d"))[0:8])
 *   miner.go:45-46  the scan starts from (2^64-1, 2^64-1)
 *   miner.go:59-65  ascending nonces, strict '<' (smallest nonce wins ties);
 *                   bounds inclusive (README:329)
 *
 * How it scans (FIPS 180-4 SHA-256, nothing GPU-specific):
 *   - the whole 64-byte blocks of "msg " are compressed once (midstate);
 *   - [lower, upper] is cut at powers of ten, so every nonce of a piece has
 *     the same digit count and the same final-block layout;
 *   - each of 16 lanes walks its own contiguous run of a piece in ascending
 *     order, its message words kept structure-of-arrays and its decimal
 *     digits stepped in place (with carries), and all 16 are compressed
 *     together with vprord / vpternlogd / vpaddd;
 *   - each lane keeps a strict-'<' minimum; lanes, then threads, merge by
 *     lexicographic (hash, nonce) min, which equals the sequential scan.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "bm_oracle.h"

static const uint32_t K16[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

static const uint32_t IV16[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

#define LANES 16
#define AVX512 __attribute__((target("avx512f")))

static inline uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

/* scalar compression for the midstate */
static void compress1(uint32_t st[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
               ((uint32_t)blk[4 * i + 2] << 8) | (uint32_t)blk[4 * i + 3];
    for (int i = 16; i < 64; ++i)
        w[i] = w[i - 16] + (ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
               (ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10));
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = h + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + K16[i] + w[i];
        uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

#define ROR(x, n) _mm512_ror_epi32((x), (n))
#define XOR3(a, b, c) _mm512_ternarylogic_epi32((a), (b), (c), 0x96)
#define CH(e, f, g) _mm512_ternarylogic_epi32((e), (f), (g), 0xCA)
#define MAJ(a, b, c) _mm512_ternarylogic_epi32((a), (b), (c), 0xE8)
#define ADD(a, b) _mm512_add_epi32((a), (b))

/* 16 compressions of one block each: st[k] (in/out) += F(st, w). */
AVX512 static void compress16(__m512i st[8], const uint32_t* wsoa /* [16][LANES] */) {
    __m512i w[16];
    for (int i = 0; i < 16; ++i) w[i] = _mm512_loadu_si512((const void*)(wsoa + LANES * i));
    __m512i a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int t = 0; t < 64; ++t) {
        __m512i wt;
        if (t < 16) {
            wt = w[t];
        } else {
            const __m512i x15 = w[(t - 15) & 15], x2 = w[(t - 2) & 15];
            const __m512i s0 = XOR3(ROR(x15, 7), ROR(x15, 18), _mm512_srli_epi32(x15, 3));
            const __m512i s1 = XOR3(ROR(x2, 17), ROR(x2, 19), _mm512_srli_epi32(x2, 10));
            wt = ADD(ADD(w[t & 15], s0), ADD(w[(t - 7) & 15], s1));
            w[t & 15] = wt;
        }
        const __m512i t1 = ADD(ADD(h, XOR3(ROR(e, 6), ROR(e, 11), ROR(e, 25))),
                               ADD(CH(e, f, g), ADD(_mm512_set1_epi32((int)K16[t]), wt)));
        const __m512i t2 = ADD(XOR3(ROR(a, 2), ROR(a, 13), ROR(a, 22)), MAJ(a, b, c));
        h = g; g = f; f = e; e = ADD(d, t1); d = c; c = b; b = a; a = ADD(t1, t2);
    }
    st[0] = ADD(st[0], a); st[1] = ADD(st[1], b); st[2] = ADD(st[2], c); st[3] = ADD(st[3], d);
    st[4] = ADD(st[4], e); st[5] = ADD(st[5], f); st[6] = ADD(st[6], g); st[7] = ADD(st[7], h);
}

static int ndigits(uint64_t v) {
    int d = 1;
    while (v >= 10) {
        v /= 10;
        ++d;
    }
    return d;
}

static uint64_t pow10u(int d) {
    uint64_t p = 1;
    for (int i = 0; i < d; ++i) p *= 10;
    return p;
}

typedef struct {
    uint32_t mid[8];   /* state after the whole blocks of "msg " */
    uint8_t tail[64];  /* bytes of "msg " after those blocks */
    uint32_t tail_len; /* r = (len + 1) % 64 */
    uint64_t prefix;   /* len + 1 */
} prefix_t;

static void make_prefix(const uint8_t* msg, size_t len, prefix_t* p) {
    memcpy(p->mid, IV16, sizeof p->mid);
    p->prefix = (uint64_t)len + 1;
    const uint64_t full = p->prefix / 64;
    uint8_t blk[64];
    for (uint64_t b = 0; b < full; ++b) {
        for (int i = 0; i < 64; ++i) {
            const uint64_t pos = b * 64 + (uint64_t)i;
            blk[i] = pos < len ? msg[pos] : (uint8_t)' ';
        }
        compress1(p->mid, blk);
    }
    p->tail_len = (uint32_t)(p->prefix - full * 64);
    for (uint32_t i = 0; i < p->tail_len; ++i) {
        const uint64_t pos = full * 64 + i;
        p->tail[i] = pos < len ? msg[pos] : (uint8_t)' ';
    }
}

/* word k of lane l in the SoA block array */
#define WSOA(arr, k, l) ((arr)[LANES * (k) + (l)])

/* Adds delta (-9..1) to the digit byte at tail-relative position pos. */
static inline void bump(uint32_t* wsoa, int l, uint32_t pos, int32_t delta) {
    WSOA(wsoa, pos >> 2, l) += (uint32_t)delta << (8 * (3 - (pos & 3)));
}

/* Scan [lo, hi] (all nonces with D digits) in 16 lanes. */
AVX512 static void scan_piece(const prefix_t* P, uint64_t lo, uint64_t hi, int D, uint64_t* bh, uint64_t* bn) {
    const uint32_t r = P->tail_len;
    const uint32_t nb = (r + (uint32_t)D + 9 <= 64) ? 1 : 2;
    uint32_t wsoa[2 * 16 * LANES] __attribute__((aligned(64)));
    uint8_t digs[LANES][20];
    uint64_t cnt[LANES], next[LANES], lbh[LANES], lbn[LANES];
    const uint64_t span = hi - lo; /* count - 1 */
    const uint64_t per = span / LANES + 1;
    uint64_t steps = 0;
    for (int l = 0; l < LANES; ++l) {
        const uint64_t off = per * (uint64_t)l;
        cnt[l] = off > span ? 0 : (span - off + 1 < per ? span - off + 1 : per);
        next[l] = lo + (cnt[l] ? off : 0);
        if (cnt[l] > steps) steps = cnt[l];
        lbh[l] = UINT64_MAX;
        lbn[l] = UINT64_MAX;
        /* the lane's first message: tail ‖ digits ‖ 0x80 ‖ 0 ... ‖ bit length */
        uint8_t blk[128];
        memset(blk, 0, sizeof blk);
        memcpy(blk, P->tail, r);
        uint64_t x = next[l];
        for (int k = D - 1; k >= 0; --k) {
            digs[l][k] = (uint8_t)('0' + x % 10);
            x /= 10;
        }
        memcpy(blk + r, digs[l], (size_t)D);
        blk[r + (uint32_t)D] = 0x80;
        const uint64_t bits = (P->prefix + (uint64_t)D) * 8u;
        for (int i = 0; i < 8; ++i) blk[nb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
        for (uint32_t k = 0; k < 16 * nb; ++k)
            WSOA(wsoa, k, l) = ((uint32_t)blk[4 * k] << 24) | ((uint32_t)blk[4 * k + 1] << 16) |
                               ((uint32_t)blk[4 * k + 2] << 8) | (uint32_t)blk[4 * k + 3];
    }
    __m512i mid[8];
    for (int i = 0; i < 8; ++i) mid[i] = _mm512_set1_epi32((int)P->mid[i]);
    __m512i hiv = _mm512_set1_epi32(-1); /* per-lane high word of its best hash */
    for (uint64_t s = 0; s < steps; ++s) {
        __m512i st[8];
        for (int i = 0; i < 8; ++i) st[i] = mid[i];
        compress16(st, wsoa);
        if (nb == 2) compress16(st, wsoa + 16 * LANES);
        /* rare path: a lane whose H0 <= its best high word */
        const __mmask16 m = _mm512_cmple_epu32_mask(st[0], hiv);
        if (m) {
            uint32_t h0[LANES], h1[LANES];
            _mm512_storeu_si512((void*)h0, st[0]);
            _mm512_storeu_si512((void*)h1, st[1]);
            for (int l = 0; l < LANES; ++l) {
                if (!((m >> l) & 1) || s >= cnt[l]) continue;
                const uint64_t h = ((uint64_t)h0[l] << 32) | h1[l];
                if (h < lbh[l]) { /* strict '<' over ascending nonces (miner.go:61) */
                    lbh[l] = h;
                    lbn[l] = next[l];
                }
            }
            uint32_t hv[LANES];
            for (int l = 0; l < LANES; ++l) hv[l] = (uint32_t)(lbh[l] >> 32);
            hiv = _mm512_loadu_si512((const void*)hv);
        }
        /* step every lane's decimal digits by one, in place */
        for (int l = 0; l < LANES; ++l) {
            if (s + 1 >= cnt[l]) continue;
            ++next[l];
            int k = D - 1;
            while (digs[l][k] == '9') {
                digs[l][k] = '0';
                bump(wsoa, l, r + (uint32_t)k, -9);
                --k; /* k >= 0: the piece never crosses a power of ten */
            }
            ++digs[l][k];
            bump(wsoa, l, r + (uint32_t)k, 1);
        }
    }
    for (int l = 0; l < LANES; ++l)
        if (lbh[l] < *bh || (lbh[l] == *bh && lbn[l] < *bn)) {
            *bh = lbh[l];
            *bn = lbn[l];
        }
}

/* [lo, hi] cut at powers of ten */
static void scan_range16(const prefix_t* P, uint64_t lo, uint64_t hi, uint64_t* bh, uint64_t* bn) {
    *bh = UINT64_MAX;
    *bn = UINT64_MAX;
    if (lo > hi) return;
    uint64_t cur = lo;
    for (;;) {
        const int D = ndigits(cur);
        const uint64_t top = D >= 20 ? UINT64_MAX : pow10u(D) - 1;
        const uint64_t end = top < hi ? top : hi;
        scan_piece(P, cur, end, D, bh, bn);
        if (end == hi) break;
        cur = end + 1;
    }
}

typedef struct {
    const prefix_t* P;
    uint64_t lo, hi, h, n;
} job16_t;

typedef struct {
    job16_t* jobs;
    uint64_t njobs;
    uint64_t next; /* work queue head (atomic) */
} queue16_t;

static void* worker16(void* p) {
    queue16_t* q = (queue16_t*)p;
    for (;;) {
        const uint64_t i = __atomic_fetch_add(&q->next, 1, __ATOMIC_RELAXED);
        if (i >= q->njobs) return NULL;
        job16_t* j = &q->jobs[i];
        scan_range16(j->P, j->lo, j->hi, &j->h, &j->n);
    }
}

int oracle_search_x16(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, int nthreads,
                      uint64_t* oh, uint64_t* on) {
    __builtin_cpu_init();
    if (!__builtin_cpu_supports("avx512f")) return -2;
    if (nthreads < 1) nthreads = 1;
    *oh = UINT64_MAX;
    *on = UINT64_MAX;
    if (lower > upper) return 0;
    prefix_t P;
    make_prefix(msg, len, &P);
    /* many more pieces than threads, taken from a queue, so threads finish together */
    const uint64_t span = upper - lower;
    uint64_t npieces = (uint64_t)nthreads * 64;
    if (npieces > span / 4096 + 1) npieces = span / 4096 + 1;
    job16_t* jobs = (job16_t*)calloc((size_t)npieces, sizeof(job16_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return -1;
    }
    const uint64_t q = span / npieces, rem = span % npieces;
    uint64_t cur = lower;
    for (uint64_t i = 0; i < npieces; ++i) {
        const uint64_t piece = q + (i < rem ? 1 : 0) + (i == 0 ? 1 : 0);
        jobs[i].P = &P;
        jobs[i].lo = cur;
        jobs[i].hi = cur + (piece - 1);
        cur = jobs[i].hi + 1; /* may wrap only after the last piece */
    }
    jobs[npieces - 1].hi = upper;
    queue16_t queue = {jobs, npieces, 0};
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, worker16, &queue);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    for (uint64_t i = 0; i < npieces; ++i)
        if (jobs[i].h < *oh || (jobs[i].h == *oh && jobs[i].n < *on)) {
            *oh = jobs[i].h;
            *on = jobs[i].n;
        }
    free(jobs);
    free(th);
    return 0;
}
