// bm_common.h -- launch descriptor shared by the host launcher and the
// gfx950 kernels.  Passed BY VALUE as the kernel argument, so every field is
// wave-uniform and lives in SGPRs (kernarg segment, s_load).
#pragma once
#include <cstdint>

namespace bm {

#ifndef BM_BLOCK  // threads per workgroup of the search kernels (a build knob for A/B)
#define BM_BLOCK 256
#endif
constexpr int kBlock = BM_BLOCK;  // 4 waves
static_assert(kBlock % 64 == 0 && kBlock >= 64 && kBlock <= 1024, "whole waves");

struct Partial {  // 16-byte result, ordered lexicographically (hash, nonce)
    uint64_t hash;
    uint64_t nonce;
};

struct SearchArgs {
    uint32_t mid[8];     // SHA-256 state before the varying block(s)
    uint32_t tmpl[32];   // varying block words (digit bytes = '0')
    uint32_t padkw[64];  // K[t] + W[t] of the constant padding block (pad mode)
    uint64_t vlo, vhi;   // inclusive range of v; nonce = nonce_base + v
    uint64_t nonce_base;
    uint64_t t0, t_end;  // task range [t0, t_end); task t covers v in [t*S, t*S + S)
    uint32_t chunk_m;    // tasks per lane per dequeued chunk (a chunk = 64*chunk_m tasks)
    uint32_t S;          // nonces per task = 10^ms
    uint32_t ms;         // digits iterated by the inner loop (all in one word)
    uint32_t nd;         // digits of v placed in the varying block(s)
    uint32_t part_off;   // first partial slot written by this launch
    uint32_t pad_;
};

struct HashArgs {
    uint32_t mid[8];    // state after the whole 64-byte blocks of "msg "
    uint8_t tail[64];   // remaining bytes of "msg " (tail_len < 64)
    uint32_t tail_len;
    uint32_t pad_;
    uint64_t total_prefix;  // L + 1 (bytes of "msg ")
    uint64_t n;             // nonces to hash
};

}  // namespace bm
