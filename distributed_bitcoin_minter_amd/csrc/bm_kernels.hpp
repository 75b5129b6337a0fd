// bm_kernels.hpp -- gfx950 (CDNA4) kernels for the nonce search.
//
// Replaces the reference's per-nonce bitcoin.Hash call inside the miner's
// min-scan (/root/reference/project2/bitcoin/hash.go:11-15 and
// bitcoin/miner/miner.go:58-65) with one integer-VALU-bound kernel:
//
//   * Each lane owns a "task": S = 10^ms consecutive values of v whose
//     high digits (the task index t) are constant.  The task's digits are
//     formatted once per task (64-bit divide-by-10 chain) and added into the
//     template words.
//   * The ms low digits sit in ONE 32-bit message word (word LW of the last
//     block) and are identical in all 64 lanes at every inner iteration, so
//     they are kept in SGPRs and stepped on the scalar unit.
//   * Rounds 0..LW-1 of the last block depend only on task-constant words and
//     are computed once per task; the schedule terms that do not depend on
//     word LW are loop-invariant and hoisted out of the inner loop.
//   * Words after LW are compile-time constants (zeros / the 0x80 pad byte),
//     so the schedule sheds their terms at compile time (template P = byte
//     position of the last digit).
//   * Rotations are v_alignbit_b32, Sigma/sigma xors and Ch/Maj are single
//     v_bitop3_b32 (gfx950), sums fold into v_add3_u32.
//   * The running minimum is compared on the first state word only; the
//     exact 64-bit compare, the range check and the update run on the rare
//     path (a new low is seen ~ln(n) times per lane).
//   * Ties: a lane scans its nonces in ascending order with a strict '<', and
//     every reduction above it is a lexicographic (hash, nonce) min, which
//     equals the reference's sequential strict-'<' scan.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "bm_common.h"
#include "bm_sha256.hpp"

namespace bm {

#define BM_DEV __device__ __forceinline__

template <int B, int E, class F>
BM_DEV void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

BM_DEV uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }

// 3-input bitwise ops as one v_bitop3_b32; constant operands fold in C instead
// (the intrinsic is opaque to constant folding).
BM_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    if (__builtin_constant_p(a) && __builtin_constant_p(b) && __builtin_constant_p(c)) return a ^ b ^ c;
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
BM_DEV uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    if (__builtin_constant_p(e) && __builtin_constant_p(f) && __builtin_constant_p(g)) return (e & f) ^ (~e & g);
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
BM_DEV uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    if (__builtin_constant_p(a) && __builtin_constant_p(b) && __builtin_constant_p(c))
        return (a & b) ^ (a & c) ^ (b & c);
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
BM_DEV uint32_t bsig0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
BM_DEV uint32_t bsig1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
BM_DEV uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
BM_DEV uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }

// Round T on a rotating register file: entering round T, role r (a=0..h=7)
// lives in s[(r - T) & 7], so no values move between rounds.
template <int T>
BM_DEV void sha_round(uint32_t (&s)[8], uint32_t w) {
    uint32_t& a = s[(0 - T) & 7];
    uint32_t& b = s[(1 - T) & 7];
    uint32_t& c = s[(2 - T) & 7];
    uint32_t& d = s[(3 - T) & 7];
    uint32_t& e = s[(4 - T) & 7];
    uint32_t& f = s[(5 - T) & 7];
    uint32_t& g = s[(6 - T) & 7];
    uint32_t& h = s[(7 - T) & 7];
    const uint32_t t1 = h + bsig1(e) + ch(e, f, g) + (kK256[T] + w);
    d += t1;
    h = t1 + bsig0(a) + maj(a, b, c);
}

#ifndef BM_PAD_ADD3S  // generic padding block: the K+W kernarg inside one v_add3 (A/B knob)
#define BM_PAD_ADD3S 1
#endif

// a + s + b as ONE v_add3_u32 reading the wave-uniform s from its SGPR.
// Written in C, LLVM adds s on its own first (v_add_u32 v, s, v: an SGPR
// operand makes it a slow-class op), then v_add3 -- two slow ops where one
// slow v_add3 plus one fast v_add_u32 of the third term does.
BM_DEV uint32_t add3_sgpr(uint32_t a, uint32_t s, uint32_t b) {
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(s), "v"(b));
    return r;
}

// Same round with K[T] + W[T] supplied pre-added (constant padding block):
// a compile-time literal (search_kernel_padc) or a kernarg SGPR.
template <int T, bool KW_SGPR = false>
BM_DEV void sha_round_kw(uint32_t (&s)[8], uint32_t kw) {
    uint32_t& a = s[(0 - T) & 7];
    uint32_t& b = s[(1 - T) & 7];
    uint32_t& c = s[(2 - T) & 7];
    uint32_t& d = s[(3 - T) & 7];
    uint32_t& e = s[(4 - T) & 7];
    uint32_t& f = s[(5 - T) & 7];
    uint32_t& g = s[(6 - T) & 7];
    uint32_t& h = s[(7 - T) & 7];
    uint32_t t1;
    if constexpr (KW_SGPR && BM_PAD_ADD3S)
        t1 = add3_sgpr(h, kw, ch(e, f, g)) + bsig1(e);
    else
        t1 = h + bsig1(e) + ch(e, f, g) + kw;
    d += t1;
    h = t1 + bsig0(a) + maj(a, b, c);
}

// Rounds [R0, R1) of one block; w is the 16-word schedule window holding
// W[t] at w[t & 15] (the raw block words on entry when R0 <= 16).
template <int R0, int R1>
BM_DEV void sha_rounds(uint32_t (&s)[8], uint32_t (&w)[16]) {
    static_for<R0, R1>([&](auto I) {
        constexpr int t = decltype(I)::value;
        if constexpr (t >= 16)
            w[t & 15] = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
        sha_round<t>(s, w[t & 15]);
    });
}

// sigma0 in plain shifts, for wave-uniform arguments (the compiler keeps it
// on the scalar unit).
BM_DEV uint32_t ssig0_uniform(uint32_t x) {
    return ((x >> 7) | (x << 25)) ^ ((x >> 18) | (x << 14)) ^ (x >> 3);
}

#ifndef BM_PIN  // SALU sigma0(J) + VGPR copies of launch constants in the inner loop (A/B knob)
#define BM_PIN 1
#endif

// sigma0 of a wave-uniform word on the scalar unit.  Written in C, LLVM turns
// the rotates into v_alignbit reading the SGPR (two slow VALU ops per nonce);
// here they stay SALU (its own issue port), and only the final xor with the
// per-lane part is a VALU op.
BM_DEV uint32_t ssig0_salu(uint32_t x) {
    uint32_t r, t0, t1, t2;
    asm("s_lshr_b32 %1, %4, 7\n\t"
        "s_lshl_b32 %2, %4, 25\n\t"
        "s_or_b32 %1, %1, %2\n\t"
        "s_lshr_b32 %2, %4, 18\n\t"
        "s_lshl_b32 %3, %4, 14\n\t"
        "s_or_b32 %2, %2, %3\n\t"
        "s_xor_b32 %1, %1, %2\n\t"
        "s_lshr_b32 %2, %4, 3\n\t"
        "s_xor_b32 %0, %1, %2"
        : "=s"(r), "=&s"(t0), "=&s"(t1), "=&s"(t2)
        : "s"(x)
        : "scc");
    return r;
}

// A launch constant (kernarg SGPR) copied once into a VGPR, so the inner
// loop's ops that use it read no SGPR and stay in the fast class.
BM_DEV uint32_t vgpr_copy(uint32_t x) {
    uint32_t r;
    asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
}

// Inner-loop rounds [R0, 64) of the last block, with two shortcuts
// (BM_FOLD, A/B-able):
//  * sigma0(W[V]) enters W[V+15]; V is the word that varies per nonce.  There
//    W[V] = wl + J with disjoint bits (J only fills the low nibbles of '0'
//    digit bytes), and sigma0 is linear over GF(2), so sigma0(W[V]) =
//    sigma0(wl) ^ sigma0(J): a per-task value (hoisted) ^ a wave-uniform one
//    (scalar unit).  s0v is that xor.
//  * round 63 folds the midstate word `h0_add` into its K constant, so the 'a'
//    it produces is H0 = st[0] + a64 itself (e64 is never needed).
// Returns H0; s is left as it entered round 63, so s[1] = a63 (H1 - st[1]).
template <int R0, int V>
BM_DEV uint32_t sha_rounds_h0(uint32_t (&s)[8], uint32_t (&w)[16], uint32_t s0v, uint32_t h0_add) {
    static_assert(R0 <= V && V >= 1 && V <= 15, "varying word");
    static_for<R0, 63>([&](auto I) {
        constexpr int t = decltype(I)::value;
        if constexpr (t >= 16) {
            uint32_t s0;
            if constexpr (t - 15 == V)
                s0 = s0v;
            else
                s0 = ssig0(w[(t - 15) & 15]);
            w[t & 15] = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + s0 + w[t & 15];
        }
        sha_round<t>(s, w[t & 15]);
    });
    w[15] = ssig1(w[13]) + w[8] + ssig0(w[0]) + w[15];  // W[63]
    const uint32_t a = s[1], b = s[2], c = s[3], e = s[5], f = s[6], g = s[7], h = s[0];  // roles at round 63
    const uint32_t t1 = h + bsig1(e) + ch(e, f, g) + (kK256[63] + h0_add) + w[15];
    return t1 + bsig0(a) + maj(a, b, c);
}

// Full compression: st = st + F(st, block).
BM_DEV void sha_compress(uint32_t (&st)[8], uint32_t (&w)[16]) {
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = st[i];
    sha_rounds<0, 64>(s, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] += s[i];
}

// Compile-time value of last-block word k > LW, or -1 when it is runtime
// (the bit-length word of a non-padding layout).
template <int P, bool PADB>
constexpr int64_t tail_word(int k) {
    constexpr int LW = P / 4;
    if (k == LW + 1 && (P % 4) == 3 && P != 63) return 0x80000000ll;  // 0x80 spilled into the next word
    if (!PADB && k == 15) return -1;  // 8 * message length
    return 0;                         // zeros (and word 14: length < 2^32 bits)
}

// Add the digits of task t into the words: v's digit i (0 = least
// significant) lives at byte 64*(NBV-1) + P - i of the varying region.
// Digits i in [ms, nd) come from t; digits below ms are the inner loop's.
template <int P, int NBV>
BM_DEV void add_task_digits(uint32_t (&W)[16 * NBV], uint64_t t, uint32_t ms, uint32_t nd) {
    uint64_t x = t;
    static_for<1, 20>([&](auto I) {
        constexpr int i = decltype(I)::value;
        constexpr int pos = 64 * (NBV - 1) + P - i;
        if constexpr (pos >= 0) {
            if (i >= (int)ms && i < (int)nd) {  // wave-uniform
                const uint64_t q = x / 10u;
                const uint32_t d = (uint32_t)(x - q * 10u);
                x = q;
                W[pos >> 2] += d << (8 * (3 - (pos & 3)));
            }
        }
    });
}

// Lexicographic (hash, nonce) compare.
BM_DEV bool lex_less(uint64_t h1, uint64_t n1, uint64_t h2, uint64_t n2) {
    return h1 < h2 || (h1 == h2 && n1 < n2);
}

template <int XOR>
BM_DEV uint64_t swizzle_xor_u64(uint64_t v) {
    // ds_swizzle bitmask mode: lane' = lane ^ XOR within each 32-lane half
    constexpr int pat = (XOR << 10) | 0x1F;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)v, pat);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(v >> 32), pat);
    return ((uint64_t)hi << 32) | lo;
}

BM_DEV uint64_t readlane_u64(uint64_t v, int lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// Wave-wide lexicographic min: ds_swizzle xor butterflies inside each 32-lane
// half, then the two halves via readlane.  Result valid in every lane.
BM_DEV void wave_min(uint64_t& h, uint64_t& n) {
    static_for<0, 5>([&](auto I) {
        constexpr int x = 1 << decltype(I)::value;
        const uint64_t oh = swizzle_xor_u64<x>(h), on = swizzle_xor_u64<x>(n);
        if (lex_less(oh, on, h, n)) {
            h = oh;
            n = on;
        }
    });
    const uint64_t h0 = readlane_u64(h, 0), n0 = readlane_u64(n, 0);
    const uint64_t h1 = readlane_u64(h, 32), n1 = readlane_u64(n, 32);
    if (lex_less(h1, n1, h0, n0)) {
        h = h1;
        n = n1;
    } else {
        h = h0;
        n = n0;
    }
}

// Workgroup min of (h, n) -> thread 0 returns true with the result.
template <int NT>
BM_DEV bool block_min(uint64_t& h, uint64_t& n) {
    constexpr int NWAVE = NT / 64;
    __shared__ Partial sh[NWAVE];
    wave_min(h, n);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[wave] = Partial{h, n};
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 1; i < NWAVE; ++i)
            if (lex_less(sh[i].hash, sh[i].nonce, h, n)) {
                h = sh[i].hash;
                n = sh[i].nonce;
            }
        return true;
    }
    return false;
}

BM_DEV uint64_t readfirstlane_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// The search kernel for one layout.  P = byte index (0..63) of the last
// digit inside the last varying block; NBV = 2 when each task also
// re-compresses the block before it (high digits there).
//
// Work distribution: each wave dequeues chunks of 64*m consecutive tasks
// from a per-launch counter (one returning atomic per chunk, lane 0), lane l
// taking tasks base + l, base + 64 + l, ...  Chunks come out of the counter in
// increasing order, so every lane still visits its nonces in ascending order
// (required for the strict-'<' tie rule), and the launch drains within one
// chunk whatever the residency or clock of each CU.
// Occupancy request per layout: 8 waves/SIMD (64 VGPR, <= 80 SGPR) keeps
// every 1-block inner loop spill-free; the layouts that carry a second
// compression or a per-task block re-compression in registers get a larger
// register budget (tools/check_inner.py verifies no spill lands in a loop).
#ifndef BM_FOLD  // sha_rounds_h0's shortcuts in the inner loop (0 = plain rounds, for A/B)
#define BM_FOLD 1
#endif
#ifndef BM_WAVES_MAIN  // waves/SIMD of the 1-block layouts (most of every search)
#define BM_WAVES_MAIN 7
#endif
#ifndef BM_WAVES_PAD
#define BM_WAVES_PAD 5
#endif
#ifndef BM_WAVES_NBV2
#define BM_WAVES_NBV2 7
#endif
// NBV = 2 layouts kept at 6 waves/SIMD.  Until round 6 that was P = 4, 13
// and 14, whose inner loops spilled at 7 (72 VGPRs).  Round 6: at 7, P = 13
// and 14 compile with no scratch, readlane or memory op in the inner loop
// (tools/check_inner.py), and measured +0.25% / +0.57% against 6 (-0.3% on
// an unchanged control layout; profiles/r06/ab_nbv2_tight.log), so they run
// at 7 now; P = 4 measured -0.8% at 7 and keeps 6.  BM_NBV2_TIGHT=0 gives
// P = 4 7 too (the A/B knob).
#ifndef BM_NBV2_TIGHT
#define BM_NBV2_TIGHT 1
#endif
constexpr bool nbv2_tight(int P) { return BM_NBV2_TIGHT && P == 4; }
constexpr int search_waves(int P, int NBV) {
    return (NBV == 1 && P >= 55) ? BM_WAVES_PAD
                                 : (NBV == 2 ? (nbv2_tight(P) ? 6 : BM_WAVES_NBV2) : BM_WAVES_MAIN);
}
#ifndef BM_LDS_BEST  // a lane's running best (hash, nonce) kept in LDS, not in VGPRs (A/B knob)
#define BM_LDS_BEST 0
#endif
// BM_CLOCK_PROBE=1: workgroup 0 stamps the clock counters of each launch, so
// bm_launch_stat_t.clock_ghz reports the live shader clock.  Off by default:
// although the inner loop is unchanged, the C2 kernel measured 0.35-0.67%
// slower with it (profiles/r02/ab_probe*.log); build with
// EXTRA_HIPFLAGS=-DBM_CLOCK_PROBE=1 to measure clocks.
#ifndef BM_CLOCK_PROBE
#define BM_CLOCK_PROBE 0
#endif
// The stamps sit 128 B after the launch's dequeue counter (counter[0]): a line
// of their own, away from the one every wave's atomics hit.
constexpr int kClockSlot = 16;
#ifndef BM_KATTR  // occupancy request of the search kernels (a build knob; see Makefile)
#define BM_KATTR __attribute__((amdgpu_waves_per_eu(search_waves(P, NBV), 8)))
#endif

// PADK >= 0 (the padding-block layouts of a message of PADK whole blocks
// plus the varying one): the padding block's K + W are compile-time
// constants instead of 64 kernargs (kPadKW<P, PADK>; the launcher checks the
// segment's pad_w against them), and for PADK = 0 the entering state is the
// IV, also folded.  PADK = -1: the generic kernel, everything from kernargs.
template <int P, int NBV, int PADK>
BM_DEV void search_body(const SearchArgs& A, Partial* __restrict__ part, unsigned long long* __restrict__ counter) {
    static_assert(P >= 0 && P < 64 && (NBV == 1 || (NBV == 2 && P <= 18)), "layout");
    constexpr int LW = P / 4;                      // last-block word holding the last digit
    constexpr int BOFF = 16 * (NBV - 1);           // word offset of the last block
    constexpr bool PADB = (NBV == 1) && (P >= 55); // a constant padding block follows
    constexpr bool PADC = PADK >= 0;               // its constants folded
    static_assert(!PADC || (PADB && PADK <= kMaxPadPrefixBlocks), "PADK is a padding-block layout");
    // Word LW holds only the last digit (P%4 == 0): a task's second digit is
    // stepped by an outer loop in word LW-1 (round LW-1 redone per step), so
    // tasks stay 100 nonces long instead of 10.
    constexpr bool TWOW = (P % 4 == 0) && (LW >= 1);
    // sha_rounds_h0's shortcuts (sigma0 split of word LW, H0 folded into
    // round 63); the padding-block layouts keep the plain rounds, and so do
    // the four whose inner loop would otherwise touch scratch
    // (tools/check_inner.py).
    constexpr bool kFold = BM_FOLD && !PADB && LW >= 1 && !(NBV == 1 && (P == 53 || P == 54)) &&
                           !(NBV == 2 && P >= 17);
    // BM_PIN (SALU sigma0 of the uniform digits, launch constants in VGPRs):
    // not for P >= 48, where the extra VGPRs push the inner loop into scratch
    constexpr bool kPin = BM_PIN && kFold && !(NBV == 1 && P >= 48);

    // Inner-loop digit steps: digit i (< ms) of the inner counter sits at
    // bit 8*(3 - P%4 + i) of word LW.
    constexpr uint32_t inc0 = 1u << (8 * (3 - P % 4));
    constexpr uint32_t inc1 = (P % 4) >= 1 ? 1u << (8 * (4 - P % 4)) : 0u;
    constexpr uint32_t inc2 = (P % 4) >= 2 ? 1u << (8 * (5 - P % 4)) : 0u;
    constexpr uint32_t inc3 = (P % 4) >= 3 ? 1u << (8 * (6 - P % 4)) : 0u;

    uint64_t best_h = ~0ull, best_n = ~0ull;
    uint32_t bh = 0xFFFFFFFFu;  // high word of best_h
#if BM_LDS_BEST
    // The full 64-bit best and its nonce are touched only on the rare path
    // (a new low); in LDS they cost no VGPRs, so no spill slots and no scratch
    // stores on that path.  Only bh stays in a register for the compare.
    __shared__ uint64_t lbest_h[kBlock], lbest_n[kBlock];
    lbest_h[threadIdx.x] = ~0ull;
    lbest_n[threadIdx.x] = ~0ull;
#endif

    const uint32_t S = A.S;
    // TWOW: S in {10, 100} = n_out x 10; otherwise one pass of S inner steps
    const uint32_t n_in = TWOW ? 10u : S;
    const uint32_t n_out = TWOW ? S / 10u : 1u;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t ntask = A.t_end - A.t0;
    const uint64_t chunk = 64ull * A.chunk_m;

    // clock probe: workgroup 0 (which dequeues until the counter runs dry, so
    // it spans the launch) stamps the shader-clock and constant-rate counters
    // next to the launch's dequeue counter; the host turns them into the
    // launch's average clock (bm_launch_stat_t.clock_ghz)
    if (BM_CLOCK_PROBE && blockIdx.x == 0 && threadIdx.x == 0) {
        counter[kClockSlot + 0] = __builtin_amdgcn_s_memtime();
        counter[kClockSlot + 1] = __builtin_amdgcn_s_memrealtime();
    }
    for (;;) {
        uint64_t base = 0;
        if (lane == 0) base = atomicAdd(counter, (unsigned long long)chunk);
        base = readfirstlane_u64(base);
        if (base >= ntask) break;
        for (uint32_t i = 0; i < A.chunk_m; ++i) {
            const uint64_t tt = base + 64ull * i + lane;
            if (tt >= ntask) break;
            const uint64_t t = A.t0 + tt;

            // ---- per task: words, block before (NBV=2), rounds 0..LW-1 ----
            uint32_t W[16 * NBV];
            static_for<0, 16 * NBV>([&](auto K) { W[decltype(K)::value] = A.tmpl[decltype(K)::value]; });
            add_task_digits<P, NBV>(W, t, A.ms, A.nd);

            uint32_t st[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) st[q] = PADK == 0 ? kIV256[q] : A.mid[q];
            if constexpr (NBV == 2) {
                uint32_t wa[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) wa[k] = W[k];
                sha_compress(st, wa);
            }

            uint32_t wb[16];
            static_for<0, 16>([&](auto K) {
                constexpr int k = decltype(K)::value;
                if constexpr (k <= LW) {
                    wb[k] = W[BOFF + k];
                } else {
                    constexpr int64_t c = tail_word<P, PADB>(k);
                    if constexpr (c < 0)
                        wb[k] = (kPin && NBV == 1) ? vgpr_copy(A.tmpl[BOFF + k]) : A.tmpl[BOFF + k];
                    else
                        wb[k] = (uint32_t)c;
                }
            });
            // rounds before the varying word(s): once per task
            constexpr int R0 = TWOW ? LW - 1 : LW;
            uint32_t s00[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) s00[q] = st[q];
            sha_rounds<0, R0>(s00, wb);

            const uint64_t vbase = t * (uint64_t)S;
            for (uint32_t jo = 0; jo < n_out; ++jo) {
                // ---- outer step (TWOW only): digit 1 = lowest byte of word LW-1 ----
                uint32_t wo[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) wo[k] = wb[k];
                uint32_t s0[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) s0[q] = s00[q];
                if constexpr (TWOW) {
                    wo[LW - 1] = wb[LW - 1] + jo;
                    sha_rounds<LW - 1, LW>(s0, wo);
                }
                const uint32_t wl = wo[LW];
                const uint32_t s0wl = ssig0(wl);  // sigma0 of word LW's task part (kFold)
                // BM_PIN: the round-63 constant and h1's midstate word as VGPRs
                const uint32_t h0_add = (kPin && NBV == 1) ? vgpr_copy(st[0]) : st[0];
                const uint32_t h1_add = (kPin && NBV == 1) ? vgpr_copy(st[1]) : st[1];

                // ---- inner loop over the uniform low digit(s) of word LW ----
                uint32_t J = 0, c0 = 0, c1 = 0, c2 = 0;
                for (uint32_t j = 0; j < n_in; ++j) {
                    uint32_t w[16];
#pragma unroll
                    for (int k = 0; k < 16; ++k) w[k] = wo[k];
                    w[LW] = wl + J;
                    uint32_t x[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) x[q] = s0[q];

                    uint32_t h0, h1;
                    if constexpr (kFold) {
                        const uint32_t s0J = kPin ? ssig0_salu(J) : ssig0_uniform(J);
                        h0 = sha_rounds_h0<LW, LW>(x, w, s0wl ^ s0J, h0_add);
                        h1 = h1_add + x[1];
                    } else if constexpr (PADB) {
                        sha_rounds<LW, 64>(x, w);
                        uint32_t y[8];
#pragma unroll
                        for (int q = 0; q < 8; ++q) y[q] = st[q] + x[q];
                        uint32_t z[8];
#pragma unroll
                        for (int q = 0; q < 8; ++q) z[q] = y[q];
                        static_for<0, 64>([&](auto I) {
                            constexpr int tt2 = decltype(I)::value;
                            if constexpr (PADC) {
                                constexpr uint32_t kw = kPadKW<P, (PADK > 0 ? PADK : 0)>.v[tt2];
                                sha_round_kw<tt2>(z, kw);
                            } else {
                                sha_round_kw<tt2, true>(z, A.padkw[tt2]);
                            }
                        });
                        h0 = y[0] + z[0];
                        h1 = y[1] + z[1];
                    } else {
                        sha_rounds<LW, 64>(x, w);
                        h0 = st[0] + x[0];
                        h1 = st[1] + x[1];
                    }

                    if (__builtin_expect(h0 <= bh, 0)) {
                        const uint64_t h = ((uint64_t)h0 << 32) | h1;
                        const uint64_t v = vbase + (uint64_t)jo * n_in + j;
#if BM_LDS_BEST
                        if (h < lbest_h[threadIdx.x] && v >= A.vlo && v <= A.vhi) {
                            lbest_h[threadIdx.x] = h;
                            lbest_n[threadIdx.x] = A.nonce_base + v;
                            bh = h0;
                        }
#else
                        if (h < best_h && v >= A.vlo && v <= A.vhi) {
                            best_h = h;
                            best_n = A.nonce_base + v;
                            bh = h0;
                        }
#endif
                    }

                    // step the uniform decimal counter held in word LW
                    J += inc0;
                    if (++c0 == 10u) {
                        c0 = 0;
                        J += inc1 - 10u * inc0;
                        if (++c1 == 10u) {
                            c1 = 0;
                            J += inc2 - 10u * inc1;
                            if (++c2 == 10u) {
                                c2 = 0;
                                J += inc3 - 10u * inc2;
                            }
                        }
                    }
                }
            }
        }
    }

    if (BM_CLOCK_PROBE && blockIdx.x == 0 && threadIdx.x == 0) {
        counter[kClockSlot + 2] = __builtin_amdgcn_s_memtime();
        counter[kClockSlot + 3] = __builtin_amdgcn_s_memrealtime();
    }
#if BM_LDS_BEST
    best_h = lbest_h[threadIdx.x];
    best_n = lbest_n[threadIdx.x];
#endif
    if (block_min<kBlock>(best_h, best_n)) part[A.part_off + blockIdx.x] = Partial{best_h, best_n};
}

template <int P, int NBV>
__global__ __launch_bounds__(kBlock) BM_KATTR void search_kernel(
    const SearchArgs A, Partial* __restrict__ part, unsigned long long* __restrict__ counter) {
    search_body<P, NBV, -1>(A, part, counter);
}

// The padding-block layouts (P >= 55) of a one-block message, with their
// constants folded (search_body's PADK = 0: IV and padding K + W); NBV is 1
// (a parameter only so the occupancy attribute reads as for search_kernel).
template <int P, int NBV = 1>
__global__ __launch_bounds__(kBlock) BM_KATTR void search_kernel_padc(
    const SearchArgs A, Partial* __restrict__ part, unsigned long long* __restrict__ counter) {
    static_assert(NBV == 1 && P >= 55, "padding-block layouts only");
    search_body<P, 1, 0>(A, part, counter);
}

// The same after K = 1..15 whole prefix blocks (messages whose "msg nonce"
// ends at byte 64K + P, P >= 55: L + D between about 119 and 1,023): the
// midstate comes from kernargs, the padding block's K + W are literals
// (W15 = 8 * (64K + P + 1)), so the 64 kernarg words the generic kernel
// keeps in SGPRs -- more than the file holds at this occupancy, hence its
// v_readlane refills in the inner loop -- are gone.
template <int P, int K, int NBV = 1>
__global__ __launch_bounds__(kBlock) BM_KATTR void search_kernel_padk(
    const SearchArgs A, Partial* __restrict__ part, unsigned long long* __restrict__ counter) {
    static_assert(NBV == 1 && P >= 55 && K >= 1 && K <= kMaxPadPrefixBlocks, "padding-block layouts only");
    search_body<P, 1, K>(A, part, counter);
}

}  // namespace bm
