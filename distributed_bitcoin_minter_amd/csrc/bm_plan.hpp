// bm_plan.hpp -- host-side launch planner for the nonce search.
//
// Splits an inclusive nonce range into launches ("segments") inside which
//   * every nonce has the same decimal digit count D, so the message
//     "msg <nonce>" (hash.go:13) has a fixed length, fixed SHA-256 block
//     count and fixed padding;
//   * every message byte before the varying SHA-256 block(s) is constant and
//     is folded into a midstate on the host.
// See DESIGN.md §3 for the layout and the reasoning behind each split.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "btcminer.h"

namespace bm {

extern const uint64_t kPow10[20];

// Number of decimal digits of v (1..20), Go's %d width for a uint64.
int decimal_digits(uint64_t v);

// Default cap on launches per digit-count segment before the planner
// switches to re-compressing the high-digit block per task (nbv = 2).
constexpr int kDefaultMaxWindows = 64;

// Returns BM_OK or a BM_E* code; appends to segs.
int plan_segments(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper,
                  std::vector<bm_segment_t>& segs, int max_windows = kDefaultMaxWindows);

// Split [lower, upper] into n contiguous near-equal inclusive pieces (fewer
// if the range is shorter than n).  Never overflows, also for the full
// 2^64 range.
struct Piece {
    uint64_t lo, hi;
};
std::vector<Piece> split_range(uint64_t lower, uint64_t upper, int n);

// The multi-GPU range partitioner: one contiguous piece per slot (device or
// rank), exactly n pieces.  shares empty (or not n of them): split_range's
// near-equal pieces, padded with empty ones.  Else (every share >= 1) piece
// i holds the nonces [lower + B_i, lower + B_{i+1} - 1], B_i = floor(count *
// (s_0 + ... + s_{i-1}) / S) with S the sum of the shares: sizes in
// proportion to the shares, computed in 128-bit integers so every slot of a
// process group derives the same pieces.  An empty piece has lo > hi.
std::vector<Piece> slot_pieces(uint64_t lower, uint64_t upper, int n, const std::vector<uint32_t>& shares);

}  // namespace bm
