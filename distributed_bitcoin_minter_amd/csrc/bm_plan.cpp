// bm_plan.cpp -- see bm_plan.hpp.
//
// Message layout (hash.go:13, Sprintf("%s %d")): bytes [0, L) = msg,
// byte L = ' ', bytes [L+1, L+1+D) = the D decimal digits of the nonce,
// then SHA-256 padding: 0x80, zeros, 64-bit big-endian bit length.
#include "bm_plan.hpp"

#include <algorithm>
#include <cstring>

#include "bm_sha256.hpp"

namespace bm {

const uint64_t kPow10[20] = {1ull,
                             10ull,
                             100ull,
                             1000ull,
                             10000ull,
                             100000ull,
                             1000000ull,
                             10000000ull,
                             100000000ull,
                             1000000000ull,
                             10000000000ull,
                             100000000000ull,
                             1000000000000ull,
                             10000000000000ull,
                             100000000000000ull,
                             1000000000000000ull,
                             10000000000000000ull,
                             100000000000000000ull,
                             1000000000000000000ull,
                             10000000000000000000ull};

int decimal_digits(uint64_t v) {
    int d = 1;
    while (d < 20 && v >= kPow10[d]) ++d;
    return d;
}

namespace {

// Build one segment.  vb = first varying block; blk = block of the last digit.
void emit(const uint8_t* msg, size_t L, int D, int nbv, int nd, uint64_t nonce_base, uint64_t vlo,
          uint64_t vhi, std::vector<bm_segment_t>& segs) {
    const uint64_t pabs = L + (uint64_t)D;  // index of the last digit byte
    const uint64_t blk = pabs / 64;
    const int P = (int)(pabs % 64);
    const uint64_t vb = blk - (uint64_t)(nbv - 1);
    const bool pad_block = (nbv == 1) && (P >= 55);
    const uint64_t total_bytes = L + 1 + (uint64_t)D;

    // Decimal string of a representative nonce: its high digits (those not
    // owned by v) are the same for every nonce of the segment.
    char digs[21];
    {
        uint64_t x = nonce_base + vlo;
        for (int i = D - 1; i >= 0; --i) {
            digs[i] = (char)('0' + x % 10);
            x /= 10;
        }
    }
    auto byte_at = [&](uint64_t pos) -> uint8_t {
        if (pos < L) return msg[pos];
        if (pos == L) return ' ';
        if (pos <= pabs) {
            int di = (int)(pos - L - 1);         // 0 = most significant digit
            if (di >= D - nd) return '0';        // owned by v: the kernel adds it
            return (uint8_t)digs[di];            // constant high digit
        }
        if (pos == pabs + 1) return 0x80;
        return 0;
    };

    bm_segment_t s;
    std::memset(&s, 0, sizeof s);
    s.p = P;
    s.nbv = nbv;
    s.pad_block = pad_block ? 1 : 0;
    s.digits = D;
    s.nd = nd;
    s.max_inner = std::min(nd, P % 4 + 1);
    s.vlo = vlo;
    s.vhi = vhi;
    s.nonce_base = nonce_base;

    // Midstate over the constant blocks [0, vb).
    uint32_t st[8];
    for (int i = 0; i < 8; ++i) st[i] = kIV256[i];
    uint8_t block[64];
    for (uint64_t b = 0; b < vb; ++b) {
        for (int i = 0; i < 64; ++i) block[i] = byte_at(b * 64 + (uint64_t)i);
        host::compress_bytes(st, block);
    }
    std::memcpy(s.mid, st, sizeof st);

    // Template words of the varying block(s).
    uint8_t region[128];
    const int rbytes = 64 * nbv;
    for (int i = 0; i < rbytes; ++i) region[i] = byte_at(vb * 64 + (uint64_t)i);
    const uint64_t bits = total_bytes * 8;
    if (!pad_block) {
        for (int i = 0; i < 8; ++i) region[rbytes - 1 - i] = (uint8_t)(bits >> (8 * i));
    } else {
        uint8_t pad[64];
        std::memset(pad, 0, sizeof pad);
        if (P == 63) pad[0] = 0x80;  // the 0x80 did not fit after the last digit
        for (int i = 0; i < 8; ++i) pad[63 - i] = (uint8_t)(bits >> (8 * i));
        for (int i = 0; i < 16; ++i) s.pad_w[i] = host::load_be32(pad + 4 * i);
    }
    for (int i = 0; i < rbytes / 4; ++i) s.tmpl[i] = host::load_be32(region + 4 * i);
    segs.push_back(s);
}

}  // namespace

int plan_segments(const uint8_t* msg, size_t L, uint64_t lower, uint64_t upper,
                  std::vector<bm_segment_t>& segs, int max_windows) {
    if (L > BM_MAX_MSG_LEN || (L && !msg) || max_windows < 0) return BM_EINVAL;
    if (lower > upper) return BM_OK;  // empty: the loop of miner.go:59 runs zero times
    for (int D = 1; D <= 20; ++D) {
        const uint64_t dlo = D == 1 ? 0 : kPow10[D - 1];
        const uint64_t dhi = D == 20 ? UINT64_MAX : kPow10[D] - 1;
        const uint64_t a = std::max(lower, dlo), b = std::min(upper, dhi);
        if (a > b) continue;
        const uint64_t pabs = L + (uint64_t)D;
        const uint64_t blk = pabs / 64;
        const uint64_t first = L + 1;  // first digit byte
        const int nlast = (int)(pabs - std::max<uint64_t>(first, 64 * blk) + 1);  // digits in last block
        const int h = D - nlast;  // digits in earlier blocks
        if (h == 0) {
            emit(msg, L, D, 1, D, 0, a, b, segs);
            continue;
        }
        // nlast <= 19 here, so 10^nlast fits.
        const uint64_t unit = kPow10[nlast];
        const uint64_t nwin = b / unit - a / unit + 1;
        if (nwin <= (uint64_t)max_windows) {
            // One launch per value of the high digits: they join the midstate.
            uint64_t x = a;
            for (;;) {
                const uint64_t base = (x / unit) * unit;
                const uint64_t wend = (base > UINT64_MAX - (unit - 1)) ? UINT64_MAX : base + (unit - 1);
                const uint64_t y = std::min(b, wend);
                emit(msg, L, D, 1, nlast, base, x - base, y - base, segs);
                if (y == b) break;
                x = y + 1;
            }
        } else {
            // Too many windows: each task re-compresses the block holding the
            // high digits once and then sweeps only the last block per nonce.
            emit(msg, L, D, 2, D, 0, a, b, segs);
        }
    }
    return BM_OK;
}

std::vector<Piece> split_range(uint64_t lower, uint64_t upper, int n) {
    std::vector<Piece> out;
    if (lower > upper || n < 1) return out;
    const uint64_t span = upper - lower;  // count - 1 (count may be 2^64)
    if ((uint64_t)(n - 1) > span) n = (int)(span + 1);
    // count = n*q + (r+1) with 1 <= r+1 <= n: the first r+1 pieces get q+1.
    const uint64_t q = span / (uint64_t)n, r = span % (uint64_t)n;
    uint64_t cur = lower;
    for (int i = 0; i < n; ++i) {
        const uint64_t size_m1 = (uint64_t)i <= r ? q : q - 1;
        Piece p{cur, cur + size_m1};
        out.push_back(p);
        if (i != n - 1) cur = p.hi + 1;
    }
    out.back().hi = upper;
    return out;
}

std::vector<Piece> slot_pieces(uint64_t lower, uint64_t upper, int n, const std::vector<uint32_t>& shares) {
    const Piece empty{1, 0};
    if (n < 1) return {};
    if (shares.size() != (size_t)n || lower > upper) {
        std::vector<Piece> out = split_range(lower, upper, n);
        out.resize((size_t)n, empty);
        return out;
    }
    std::vector<Piece> out((size_t)n, empty);
    unsigned __int128 total = 0;
    for (int i = 0; i < n; ++i) total += shares[(size_t)i];
    const unsigned __int128 count = (unsigned __int128)(upper - lower) + 1;  // up to 2^64
    unsigned __int128 prefix = 0, b0 = 0;
    for (int i = 0; i < n; ++i) {
        prefix += shares[(size_t)i];
        const unsigned __int128 b1 = (i == n - 1) ? count : count * prefix / total;
        if (b1 > b0) out[(size_t)i] = Piece{lower + (uint64_t)b0, lower + (uint64_t)(b1 - 1)};
        b0 = b1;
    }
    return out;
}

}  // namespace bm
