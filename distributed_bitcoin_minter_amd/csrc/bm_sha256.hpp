// bm_sha256.hpp -- SHA-256 constants shared by host and device code, and the
// host-side compression used ONLY to fold the constant message prefix into a
// midstate before a launch (the per-nonce work is on the GPU).
//
// FIPS 180-4 SHA-256; the reference reaches it through Go's crypto/sha256 in
// bitcoin.Hash (/root/reference/project2/bitcoin/hash.go:11-15).
#pragma once
#include <cstdint>

namespace bm {

#if defined(__HIPCC__) || defined(__HIP__)
#define BM_HD __host__ __device__
#else
#define BM_HD
#endif

constexpr uint32_t kK256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

constexpr uint32_t kIV256[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

// K[t] + W[t] of the constant padding block that follows a message of K
// whole 64-byte blocks plus a last block whose last byte is at P >= 55:
// W0 = 0x80000000 when P = 63 (the 0x80 byte spilled over), W15 = the
// message length in bits, 8 * (64K + P + 1), W1..W14 = 0, W16..W63 expanded
// at compile time.  The folded padding-block kernels (bm_kernels.hpp:
// search_kernel_padc, K = 0, whose entering state is the IV; search_kernel_padk,
// K = 1..kMaxPadPrefixBlocks, after a midstate) use these as literal operands instead of 64
// kernarg SGPRs; the launcher checks a segment against them at run time.
struct KW64 {
    uint32_t v[64];
};
constexpr uint32_t crotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
constexpr KW64 pad_kw_const(int P, int K = 0) {
    uint32_t w[64] = {};
    w[0] = P == 63 ? 0x80000000u : 0u;
    w[15] = 8u * (uint32_t)(64 * K + P + 1);
    for (int t = 16; t < 64; ++t) {
        const uint32_t x = w[t - 15], y = w[t - 2];
        w[t] = (crotr(y, 17) ^ crotr(y, 19) ^ (y >> 10)) + w[t - 7] + (crotr(x, 7) ^ crotr(x, 18) ^ (x >> 3)) +
               w[t - 16];
    }
    KW64 r{};
    for (int t = 0; t < 64; ++t) r.v[t] = kK256[t] + w[t];
    return r;
}
template <int P, int K = 0>
inline constexpr KW64 kPadKW = pad_kw_const(P, K);
// search_kernel_padk<P, K>: K = 1..15 prefix blocks, i.e. "msg nonce" up to
// 64 * 15 + 64 = 1,024 bytes -- every message an LSP packet can carry (about
// 1,000 bytes, README:61; the reference's readers take 1,500-byte datagrams,
// lsp/client_impl.go:172).  Longer messages run the generic kernel.
constexpr int kMaxPadPrefixBlocks = 15;

namespace host {

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

inline uint32_t load_be32(const uint8_t* p) {
    return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}

// Message schedule of one block (w[0..15] given) -> w[16..63].
inline void expand(uint32_t w[64]) {
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
}

inline void compress(uint32_t st[8], const uint32_t block_words[16]) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = block_words[i];
    expand(w);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kK256[i] + w[i];
        uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

inline void compress_bytes(uint32_t st[8], const uint8_t block[64]) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) w[i] = load_be32(block + 4 * i);
    compress(st, w);
}

}  // namespace host
}  // namespace bm
