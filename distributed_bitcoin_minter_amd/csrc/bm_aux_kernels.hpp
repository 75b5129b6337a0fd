// bm_aux_kernels.hpp -- the small kernels around the search kernel:
//   reduce_partials : second pass, lexicographic min of the per-workgroup
//                     partials of one search on one device -> 16 bytes.
//   lane_partials_min : the search kernel's workgroup reduction over given
//                     partials (bm_reduce_gpu, a test entry for the tie rule).
//   hash_kernel     : batched bitcoin.Hash (hash.go:11-15) for arbitrary
//                     nonces, used by bm_hash_gpu (parity tests, the Hash
//                     mirror).  Not on the search hot path.
#pragma once
#include "bm_kernels.hpp"

namespace bm {

constexpr int kReduceThreads = 1024;

__global__ __launch_bounds__(kReduceThreads) void reduce_partials(const Partial* __restrict__ part, uint32_t n,
                                                                  Partial* __restrict__ out) {
    uint64_t h = ~0ull, nn = ~0ull;
    for (uint32_t i = threadIdx.x; i < n; i += kReduceThreads) {
        const Partial p = part[i];
        if (lex_less(p.hash, p.nonce, h, nn)) {
            h = p.hash;
            nn = p.nonce;
        }
    }
    if (block_min<kReduceThreads>(h, nn)) *out = Partial{h, nn};
}

// Test entry of the reductions (bm_reduce_gpu): one partial per lane
// (beyond n: the empty (2^64-1, 2^64-1)), the search kernel's block_min
// (ds_swizzle butterflies, readlane, LDS), one partial per workgroup.
__global__ __launch_bounds__(kBlock) void lane_partials_min(const Partial* __restrict__ in, uint32_t n,
                                                            Partial* __restrict__ out) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    uint64_t h = ~0ull, nn = ~0ull;
    if (i < n) {
        h = in[i].hash;
        nn = in[i].nonce;
    }
    if (block_min<kBlock>(h, nn)) out[blockIdx.x] = Partial{h, nn};
}

constexpr int kHashThreads = 64;

// One lane per nonce.  The lane assembles its (at most two) final blocks in
// its own 128-byte LDS row with byte stores at run-time offsets, then reads
// them back as big-endian words and compresses from the prefix midstate.
__global__ __launch_bounds__(kHashThreads) void hash_kernel(const HashArgs A, const uint64_t* __restrict__ nonces,
                                                            uint64_t* __restrict__ out) {
    __shared__ uint32_t rows[kHashThreads][32];
    const uint64_t i = (uint64_t)blockIdx.x * kHashThreads + threadIdx.x;
    if (i >= A.n) return;
    uint32_t* row32 = rows[threadIdx.x];
    uint8_t* row = reinterpret_cast<uint8_t*>(row32);
#pragma unroll
    for (int k = 0; k < 32; ++k) row32[k] = 0;

    const uint64_t nonce = nonces[i];
    int D = 1;
    for (uint64_t x = nonce; x >= 10; x /= 10) ++D;
    const uint32_t tl = A.tail_len;
    for (uint32_t k = 0; k < tl; ++k) row[k] = A.tail[k];
    uint64_t x = nonce;
    for (int k = D - 1; k >= 0; --k) {
        row[tl + k] = (uint8_t)('0' + (uint32_t)(x % 10u));
        x /= 10u;
    }
    row[tl + D] = 0x80;
    const int nb = (tl + D + 9 <= 64) ? 1 : 2;
    const uint64_t bits = (A.total_prefix + (uint64_t)D) * 8u;
    row32[nb * 16 - 2] = __builtin_bswap32((uint32_t)(bits >> 32));
    row32[nb * 16 - 1] = __builtin_bswap32((uint32_t)bits);

    uint32_t st[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) st[k] = A.mid[k];
    for (int b = 0; b < nb; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = __builtin_bswap32(row32[b * 16 + k]);
        sha_compress(st, w);
    }
    out[i] = ((uint64_t)st[0] << 32) | st[1];
}

}  // namespace bm
