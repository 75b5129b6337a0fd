/*
 * bm_oracle.c -- CPU restatement of the reference hot path.  TEST
 * INFRASTRUCTURE ONLY (see bm_oracle.h): never linked into the product.
 *
 * Reference behaviour restated here:
 *   hash.go:11-15   Hash(msg, nonce) = BigEndian.Uint64(sha256(Sprintf("%s %d"))[0:8])
 *   miner.go:45-46  min_hash = min_nonce = 2^64-1 before the scan
 *   miner.go:59-65  ascending scan, `if current_hash < min_hash` (strict)
 *
 * SHA-256 is written from FIPS 180-4 directly (Go's crypto/sha256 is the
 * same standard function).  An optional OpenSSL path hashes the very same
 * byte string with the system libcrypto, which is only a speed knob.
 */
#include "bm_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef BM_ORACLE_OPENSSL
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include <openssl/sha.h>
#endif

static const uint32_t K256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

static const uint32_t IV256[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                  0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

static inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void sha256_compress(uint32_t st[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
               ((uint32_t)blk[4 * i + 2] << 8) | (uint32_t)blk[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[i] + w[i];
        uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void oracle_sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
    uint32_t st[8];
    memcpy(st, IV256, sizeof st);
    size_t off = 0;
    for (; off + 64 <= len; off += 64) sha256_compress(st, data + off);
    uint8_t blk[128];
    size_t rem = len - off;
    memset(blk, 0, sizeof blk);
    if (rem) memcpy(blk, data + off, rem);
    blk[rem] = 0x80;
    size_t nblk = (rem + 1 + 8 <= 64) ? 1 : 2;
    uint64_t bits = (uint64_t)len * 8u;
    for (int i = 0; i < 8; ++i) blk[nblk * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_compress(st, blk);
    if (nblk == 2) sha256_compress(st, blk + 64);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

/* Go's %d on a uint64: unsigned decimal, no padding, "0" for zero. */
static size_t u64_to_dec(uint64_t v, char* dst) {
    char tmp[24];
    size_t n = 0;
    do {
        tmp[n++] = (char)('0' + (v % 10u));
        v /= 10u;
    } while (v);
    for (size_t i = 0; i < n; ++i) dst[i] = tmp[n - 1 - i];
    return n;
}

size_t oracle_format(const uint8_t* msg, size_t len, uint64_t nonce, uint8_t* buf, size_t cap) {
    if (len + 1 + 20 > cap) return 0;
    if (len) memcpy(buf, msg, len);
    buf[len] = ' ';
    return len + 1 + u64_to_dec(nonce, (char*)buf + len + 1);
}

static uint64_t be64(const uint8_t* d) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | d[i];
    return v;
}

static uint64_t hash_with(uint8_t* buf, size_t cap, const uint8_t* msg, size_t len, uint64_t nonce,
                          int use_openssl) {
    uint8_t dig[32];
    size_t n = oracle_format(msg, len, nonce, buf, cap);
#ifdef BM_ORACLE_OPENSSL
    if (use_openssl == 2) {
        /* hash.go:11-15 allocates per call: sha256.New() a digest, fmt.Sprintf
         * the "%s %d" string, []byte(...) its copy, Sum(nil) the 32-byte
         * slice.  The same four heap objects here, each malloc'd and freed per
         * nonce, and the decimal digits through printf's %llu as Sprintf's %d */
        (void)n;
        SHA256_CTX* c = (SHA256_CTX*)malloc(sizeof *c);
        char* s = (char*)malloc(cap);
        if (len) memcpy(s, msg, len);
        s[len] = ' ';
        const int k = snprintf(s + len + 1, cap - len - 1, "%llu", (unsigned long long)nonce);
        const size_t m = len + 1 + (size_t)k;
        uint8_t* b = (uint8_t*)malloc(m);
        memcpy(b, s, m);
        SHA256_Init(c);
        SHA256_Update(c, b, m);
        uint8_t* sum = (uint8_t*)malloc(32);
        SHA256_Final(sum, c);
        const uint64_t h = be64(sum);
        free(sum);
        free(b);
        free(s);
        free(c);
        return h;
    }
    if (use_openssl) {
        /* low-level API: OpenSSL 3's one-shot SHA256() re-fetches the EVP
         * provider on every call, which is ~10x slower than the block code */
        SHA256_CTX c;
        SHA256_Init(&c);
        SHA256_Update(&c, buf, n);
        SHA256_Final(dig, &c);
        return be64(dig);
    }
#else
    (void)use_openssl;
#endif
    oracle_sha256(buf, n, dig);
    return be64(dig);
}

uint64_t oracle_hash(const uint8_t* msg, size_t len, uint64_t nonce) {
    size_t cap = len + 32;
    uint8_t stackbuf[256];
    uint8_t* buf = cap <= sizeof stackbuf ? stackbuf : (uint8_t*)malloc(cap);
    uint64_t h = hash_with(buf, cap, msg, len, nonce, 0);
    if (buf != stackbuf) free(buf);
    return h;
}

void oracle_hash_many(const uint8_t* msg, size_t len, const uint64_t* nonces, size_t n, uint64_t* out) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_hash(msg, len, nonces[i]);
}

/* miner.go:45-46 init + :59-65 strict-'<' ascending scan, inclusive bound. */
static void scan_range(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, int use_openssl,
                       uint64_t* oh, uint64_t* on) {
    uint64_t min_hash = UINT64_MAX, min_nonce = UINT64_MAX;
    if (lower <= upper) {
        size_t cap = len + 32;
        uint8_t* buf = (uint8_t*)malloc(cap);
        uint64_t i = lower;
        for (;;) {
            uint64_t h = hash_with(buf, cap, msg, len, i, use_openssl);
            if (h < min_hash) {
                min_nonce = i;
                min_hash = h;
            }
            if (i == upper) break; /* inclusive upper, no wrap at 2^64-1 */
            ++i;
        }
        free(buf);
    }
    *oh = min_hash;
    *on = min_nonce;
}

void oracle_search(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, uint64_t* oh,
                   uint64_t* on) {
    scan_range(msg, len, lower, upper, 0, oh, on);
}

void oracle_search_excl(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, uint64_t* oh,
                        uint64_t* on) {
    if (upper <= lower) {
        *oh = UINT64_MAX;
        *on = UINT64_MAX;
        return;
    }
    scan_range(msg, len, lower, upper - 1, 0, oh, on);
}

typedef struct {
    const uint8_t* msg;
    size_t len;
    uint64_t lo, hi;
    int use_openssl;
    uint64_t h, n;
} job_t;

static void* job_main(void* p) {
    job_t* j = (job_t*)p;
    scan_range(j->msg, j->len, j->lo, j->hi, j->use_openssl, &j->h, &j->n);
    return NULL;
}

int oracle_search_mt(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, int nthreads,
                     int use_openssl, uint64_t* oh, uint64_t* on) {
    if (nthreads < 1) nthreads = 1;
    if (lower > upper) {
        *oh = UINT64_MAX;
        *on = UINT64_MAX;
        return 0;
    }
    uint64_t span = upper - lower; /* count - 1, never overflows */
    if ((uint64_t)nthreads > span) nthreads = (int)span + 1;
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return -1;
    }
    /* Contiguous near-equal pieces whose sizes sum to span+1 (which may be
     * 2^64 and so is never formed): q or q+1 each, plus one extra on piece 0. */
    uint64_t q = span / (uint64_t)nthreads, r = span % (uint64_t)nthreads;
    uint64_t cur = lower;
    for (int t = 0; t < nthreads; ++t) {
        uint64_t piece = q + ((uint64_t)t < r ? 1 : 0) + (t == 0 ? 1 : 0);
        jobs[t].msg = msg;
        jobs[t].len = len;
        jobs[t].lo = cur;
        jobs[t].hi = cur + (piece - 1);
        jobs[t].use_openssl = use_openssl;
        cur = jobs[t].hi + 1; /* may wrap only after the last piece */
    }
    jobs[nthreads - 1].hi = upper;
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, job_main, &jobs[t]);
    uint64_t bh = UINT64_MAX, bn = UINT64_MAX;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        /* lexicographic (hash, nonce) merge == sequential strict-'<' scan */
        if (jobs[t].h < bh || (jobs[t].h == bh && jobs[t].n < bn)) {
            bh = jobs[t].h;
            bn = jobs[t].n;
        }
    }
    free(jobs);
    free(th);
    *oh = bh;
    *on = bn;
    return 0;
}
