// plan_fuzz.cpp -- host-only fuzz of the launch planner (csrc/bm_plan.cpp),
// built with AddressSanitizer + UBSan by tests/test_plan_sanitize.py:
//
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all
//       -I distributed_bitcoin_minter_amd/csrc -I include
//       tools/plan_fuzz.cpp distributed_bitcoin_minter_amd/csrc/bm_plan.cpp
//
// For random (msg length 0..700, range anywhere in u64 incl. the ends) it
// checks that the segments tile [lower, upper] in ascending order with one
// digit count each, that every layout is one the kernel table instantiates,
// and that replaying a segment the way search_kernel does (template words +
// digits of v, compressed from the midstate, + the padding block) gives
// SHA-256("msg nonce") computed directly (hash.go:13 message).
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "bm_plan.hpp"
#include "bm_sha256.hpp"

namespace {

uint64_t direct_hash(const std::vector<uint8_t>& msg, uint64_t nonce) {
    std::string s(msg.begin(), msg.end());
    s += ' ';
    s += std::to_string(nonce);
    std::vector<uint8_t> b(s.begin(), s.end());
    const uint64_t bits = (uint64_t)b.size() * 8;
    b.push_back(0x80);
    while (b.size() % 64 != 56) b.push_back(0);
    for (int i = 7; i >= 0; --i) b.push_back((uint8_t)(bits >> (8 * i)));
    uint32_t st[8];
    std::memcpy(st, bm::kIV256, sizeof st);
    for (size_t off = 0; off < b.size(); off += 64) bm::host::compress_bytes(st, b.data() + off);
    return ((uint64_t)st[0] << 32) | st[1];
}

uint64_t replay(const bm_segment_t& s, uint64_t v) {
    uint32_t w[32];
    std::memcpy(w, s.tmpl, sizeof w);
    uint64_t x = v;
    for (int i = 0; i < s.nd; ++i) {
        const int pos = 64 * (s.nbv - 1) + s.p - i;
        w[pos >> 2] += (uint32_t)(x % 10) << (8 * (3 - (pos & 3)));
        x /= 10;
    }
    uint32_t st[8];
    std::memcpy(st, s.mid, sizeof st);
    for (int b = 0; b < s.nbv; ++b) bm::host::compress(st, w + 16 * b);
    if (s.pad_block) bm::host::compress(st, s.pad_w);
    return ((uint64_t)st[0] << 32) | st[1];
}

int fail(const char* what, size_t L, uint64_t lo, uint64_t hi) {
    std::printf("FAIL %s L=%zu lo=%llu hi=%llu\n", what, L, (unsigned long long)lo, (unsigned long long)hi);
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
    std::mt19937_64 rng(0x5EED);
    size_t nseg_total = 0;
    for (int it = 0; it < iters; ++it) {
        const size_t L = rng() % 701;
        std::vector<uint8_t> msg(L);
        for (auto& c : msg) c = (uint8_t)(rng() & 0xFF);
        uint64_t lo, hi;
        switch (it % 4) {
            case 0: lo = rng() >> (rng() % 64); hi = lo + (rng() % 100000); break;
            case 1: lo = UINT64_MAX - (rng() % 1000000); hi = UINT64_MAX; break;
            case 2: lo = rng() % 1000; hi = rng() >> (rng() % 64); break;
            default: lo = rng(); hi = rng(); break;
        }
        if (hi < lo && it % 4 != 3) std::swap(lo, hi);
        std::vector<bm_segment_t> segs;
        const int mw = (it % 7 == 0) ? 0 : bm::kDefaultMaxWindows;
        if (bm::plan_segments(msg.data(), L, lo, hi, segs, mw) != BM_OK) return fail("status", L, lo, hi);
        nseg_total += segs.size();
        if (lo > hi) {
            if (!segs.empty()) return fail("empty range planned", L, lo, hi);
            continue;
        }
        uint64_t cur = lo;
        for (size_t i = 0; i < segs.size(); ++i) {
            const bm_segment_t& s = segs[i];
            const uint64_t a = s.nonce_base + s.vlo, b = s.nonce_base + s.vhi;
            if (a != cur || b < a) return fail("tiling", L, lo, hi);
            if (bm::decimal_digits(a) != s.digits || bm::decimal_digits(b) != s.digits)
                return fail("digit count", L, lo, hi);
            if (!(s.nbv == 1 || (s.nbv == 2 && s.p <= 18)) || s.p < 0 || s.p > 63) return fail("layout", L, lo, hi);
            if (s.nd < 20 && s.vhi >= bm::kPow10[s.nd]) return fail("v range", L, lo, hi);
            const uint64_t vs[3] = {s.vlo, s.vhi, s.vlo + (s.vhi - s.vlo) / 2};
            for (uint64_t v : vs)
                if (replay(s, v) != direct_hash(msg, s.nonce_base + v)) return fail("sha", L, lo, hi);
            if (b == UINT64_MAX) {
                if (i + 1 != segs.size()) return fail("past 2^64-1", L, lo, hi);
            } else {
                cur = b + 1;
            }
        }
        if (segs.empty() || segs.back().nonce_base + segs.back().vhi != hi) return fail("end", L, lo, hi);
    }
    std::printf("ok %d plans, %zu segments\n", iters, nseg_total);
    return 0;
}
