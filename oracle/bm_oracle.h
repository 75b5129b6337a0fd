/*
 * bm_oracle.h -- CPU oracle for the nonce-search hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libbtcminer.so, the
 * Python package's compute path) links, loads or calls this code.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / the timed CPU baseline.
 *
 * It restates, in plain C:
 *   - bitcoin.Hash(msg, nonce)  @ /root/reference/project2/bitcoin/hash.go:11-15
 *       SHA-256 of fmt.Sprintf("%s %d", msg, nonce), big-endian first 8 bytes.
 *   - the miner's min-scan       @ /root/reference/project2/bitcoin/miner/miner.go:45-46,59-65
 *       start (2^64-1, 2^64-1), ascending nonces, strict '<' update, so the
 *       smallest nonce wins ties.  Bounds are INCLUSIVE [lower, upper] per the
 *       spec (project2/README.md:329, "0 <= n <= N"); miner.go:59 uses an
 *       exclusive upper, the *_excl helper reproduces that literally.
 *
 * Pinned by the reference's only result-bearing data, the known answers at
 * project2/README.md:331-335, and by golden vectors generated with Python
 * hashlib (tests/golden/make_golden.py).  The reference Go code cannot be
 * built here (no Go toolchain; the miner sources do not compile).
 */
#ifndef BM_ORACLE_H
#define BM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One SHA-256 over an arbitrary byte string (FIPS 180-4, scalar). */
void oracle_sha256(const uint8_t* data, size_t len, uint8_t out[32]);

/* bitcoin.Hash(msg, nonce): hash.go:11-15. */
uint64_t oracle_hash(const uint8_t* msg, size_t len, uint64_t nonce);

/* Formats "<msg> <decimal nonce>" into buf (cap bytes); returns its length
 * or 0 when it does not fit.  Mirrors fmt.Sprintf("%s %d") in hash.go:13. */
size_t oracle_format(const uint8_t* msg, size_t len, uint64_t nonce, uint8_t* buf, size_t cap);

/* Inclusive min-scan over [lower, upper] (miner.go:45-46, 59-65).
 * lower > upper yields (2^64-1, 2^64-1), like the loop running zero times. */
void oracle_search(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper,
                   uint64_t* out_hash, uint64_t* out_nonce);

/* The literal miner.go:59 loop: for i := Lower; i < Upper; i++ (exclusive). */
void oracle_search_excl(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper,
                        uint64_t* out_hash, uint64_t* out_nonce);

/* Multi-threaded inclusive search: [lower, upper] cut into nthreads contiguous
 * pieces, each scanned as above, merged by lexicographic (hash, nonce) min,
 * which equals the sequential strict-'<' scan.
 * use_openssl != 0 hashes with OpenSSL's SHA256() (SHA-NI) instead of the
 * scalar restatement: same bytes, same answer, faster (used for goldens over
 * 2^32 nonces and as the CPU baseline).  use_openssl = 2 does the same with
 * hash.go:11-15's per-call allocation shape: a fresh heap digest
 * (sha256.New), a fresh formatted string (fmt.Sprintf, the nonce through
 * printf's %llu), its []byte copy, and a fresh 32-byte sum (Sum(nil)), all
 * freed per nonce -- bench.py's cpu_baseline.go_shape leg.  Returns 0 on
 * success. */
int oracle_search_mt(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper,
                     int nthreads, int use_openssl,
                     uint64_t* out_hash, uint64_t* out_nonce);

/* The same inclusive search with 16 lanes of AVX-512 per thread
 * (bm_scan16.c): midstate, digits stepped in place, 16 compressions at a
 * time.  Only for golden answers over ranges of 2^32..2^40 nonces; checked
 * against oracle_search() by tests/test_oracle.py.  Returns 0, or -2 when the
 * CPU lacks AVX-512F. */
int oracle_search_x16(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, int nthreads,
                      uint64_t* out_hash, uint64_t* out_nonce);

/* Hash a list of nonces (scalar restatement). */
void oracle_hash_many(const uint8_t* msg, size_t len, const uint64_t* nonces, size_t n,
                      uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif
