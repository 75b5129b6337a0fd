"""CPU tests of the host-side launch planner (bm_plan_segments).

The GPU kernel consumes each segment as: template words + the digits of v
added at byte 64*(nbv-1) + p - i, compressed from the segment's midstate
(plus the constant padding block), and assumes the words after the last
digit word are the compile-time constants of bm_kernels.hpp:tail_word().
These tests replay exactly that on the CPU (pure-Python SHA-256) and check
it against hashlib's SHA-256 of "msg nonce" (hash.go:13), so a layout bug is
caught here, without a GPU.
"""
import hashlib
import random

import pytest

from distributed_bitcoin_minter_amd import plan_segments
from sharef import IV, compress

U64 = (1 << 64) - 1


def ref_hash(msg, n):
    return int.from_bytes(hashlib.sha256(msg + b" " + str(n).encode()).digest()[:8], "big")


def kernel_replay(seg, v):
    words = list(seg.tmpl)[: 16 * seg.nbv]
    for i in range(seg.nd):
        pos = 64 * (seg.nbv - 1) + seg.p - i
        words[pos >> 2] += ((v // 10 ** i) % 10) << (8 * (3 - (pos & 3)))
    st = list(seg.mid)
    for b in range(seg.nbv):
        st = compress(st, words[16 * b: 16 * b + 16])
    if seg.pad_block:
        st = compress(st, list(seg.pad_w))
    return (st[0] << 32) | st[1]


def tail_word(p, pad):
    """Mirror of bm_kernels.hpp tail_word<P, PADB>(k): None = runtime."""
    lw = p // 4

    def f(k):
        if k == lw + 1 and p % 4 == 3 and p != 63:
            return 0x80000000
        if not pad and k == 15:
            return None
        return 0
    return f


def check_plan(msg, lo, hi, rng, samples=6):
    segs = plan_segments(msg, lo, hi)
    # segments tile [lo, hi] in ascending order
    cur = lo
    for s in segs:
        a, b = s.nonce_base + s.vlo, s.nonce_base + s.vhi
        assert a == cur and a <= b
        assert len(str(a)) == len(str(b)) == s.digits
        cur = b + 1
    assert cur - 1 == hi
    for s in segs:
        assert s.nbv in (1, 2) and 0 <= s.p < 64
        assert s.pad_block == (1 if (s.nbv == 1 and s.p >= 55) else 0)
        if s.nbv == 2:
            assert s.p <= 18
        assert s.vhi < 10 ** s.nd
        # compile-time words of the kernel match the template
        tw = tail_word(s.p, bool(s.pad_block))
        base = 16 * (s.nbv - 1)
        for k in range(s.p // 4 + 1, 16):
            exp = tw(k)
            if exp is not None:
                assert s.tmpl[base + k] == exp, (s.p, k)
        # the inner-loop digits all sit in the last-digit word
        for i in range(s.max_inner):
            assert (s.p - i) // 4 == s.p // 4
        vs = {s.vlo, s.vhi, (s.vlo + s.vhi) // 2}
        for _ in range(samples):
            vs.add(rng.randint(s.vlo, s.vhi))
        for v in vs:
            assert kernel_replay(s, v) == ref_hash(msg, s.nonce_base + v), (len(msg), s.nonce_base + v)
    return segs


RANGES = [(0, 9999), (0, 2 ** 32 - 1), (9990, 10009), (U64 - 2 ** 32 + 1, U64), (10 ** 19 - 5, 10 ** 19 + 5),
          (0, U64), (123456789, 123456789), (5, 5)]


@pytest.mark.parametrize("L", [0, 1, 7, 8, 30, 44, 45, 46, 53, 54, 55, 56, 57, 62, 63, 64, 65, 100, 110, 118, 119,
                               120, 121, 127, 128, 183, 600])
def test_plan_layout_matches_sha256(L):
    rng = random.Random(L)
    msg = bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz ,.-") for _ in range(L))
    for lo, hi in RANGES:
        check_plan(msg, lo, hi, rng)


def test_plan_every_layout_reachable():
    """Across message lengths 0..127 the planner emits every layout the
    kernel table instantiates (NBV=1: P 0..63; NBV=2: P 0..18)."""
    seen = set()
    for L in range(128):
        msg = b"x" * L
        for lo, hi in [(0, U64)]:
            for s in plan_segments(msg, lo, hi):
                seen.add((s.nbv, s.p))
    assert {(1, p) for p in range(64)} <= seen
    # NBV=2 shows up when the high digits straddle a block boundary over
    # more than 64 windows; with 10^17..10^19-nonce windows that never
    # happens, so P 17/18 (instantiated for safety) are unreachable.
    for L in range(40, 64):
        for s in plan_segments(b"y" * L, 0, U64):
            seen.add((s.nbv, s.p))
    assert {(2, p) for p in range(17)} <= seen
    assert all(p <= 16 for nbv, p in seen if nbv == 2)


def test_plan_empty_and_bad_args():
    assert plan_segments(b"msg", 10, 9) == []
    from distributed_bitcoin_minter_amd._lib import BtcMinerError
    with pytest.raises(BtcMinerError):
        plan_segments(b"x" * ((1 << 20) + 1), 0, 1)


def test_plan_c3_single_window():
    """C3 (120-B msg, 20-digit nonces near 2^64): the 7 high digits in the
    second block are constant over the range, so one launch with them in the
    midstate and 1 compression per nonce."""
    msg = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]
    segs = plan_segments(msg, U64 - (2 ** 32 - 1), U64)
    assert len(segs) == 1
    s = segs[0]
    assert (s.nbv, s.p, s.pad_block, s.digits, s.nd) == (1, 12, 0, 20, 13)


try:
    from hypothesis import HealthCheck, given, settings, strategies as st
except ImportError:  # pragma: no cover - hypothesis is in the image
    given = None

if given is not None:
    @settings(max_examples=200, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow])
    @given(msg=st.binary(min_size=0, max_size=200),
           lo=st.one_of(st.integers(0, 10 ** 6), st.integers(0, U64),
                        st.sampled_from([10 ** k - 3 for k in range(1, 20)])),
           width=st.one_of(st.integers(0, 50), st.integers(0, 10 ** 12), st.integers(0, U64)))
    def test_plan_property_random_bytes_and_ranges(msg, lo, width):
        """Any raw-byte message (Go's %s carries bytes unchanged) and any
        inclusive range, clipped at 2^64-1: the segments tile the range in
        ascending order, keep the kernel's compile-time words, and replay to
        hashlib's SHA-256 of "msg nonce" at sampled nonces."""
        hi = min(U64, lo + width)
        check_plan(msg, lo, hi, random.Random(len(msg) ^ lo), samples=2)


def _padc_kw_table(K=0):
    """pad_kw_const(P, K) for P = 55..63 from bm_sha256.hpp (the constants
    search_kernel_padc (K = 0) and search_kernel_padk<P, K> fold), printed by
    a tiny C++ program."""
    import os
    import subprocess
    import tempfile
    from conftest import ROOT
    src = ('#include <cstdio>\n#include "bm_sha256.hpp"\nint main() {\n'
           f'  for (int p = 55; p < 64; ++p) {{ const bm::KW64 k = bm::pad_kw_const(p, {K});\n'
           '    for (int t = 0; t < 64; ++t) std::printf("%u ", k.v[t]); std::printf("\\n"); }\n'
           '  static_assert(bm::kPadKW<60>.v[15] == bm::kK256[15] + 8u * 61u, "compile-time table");\n'
           '  static_assert(bm::kPadKW<60, 2>.v[15] == bm::kK256[15] + 8u * (128u + 61u), "K = 2");\n}\n')
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "kw.cpp"), os.path.join(d, "kw")
        open(c, "w").write(src)
        subprocess.check_call(["g++", "-std=c++17", "-O1", "-I",
                               os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc"), c, "-o", exe])
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.splitlines()
    return {55 + i: [int(x) for x in ln.split()] for i, ln in enumerate(out)}


@pytest.mark.parametrize("Kp", [0, 1, 2])
def test_padc_constants_are_the_padding_block_of_a_one_block_message(Kp):
    """search_kernel_padc (Kp = 0 prefix blocks) and search_kernel_padk<P, Kp>
    fold K[t] + W[t] of the padding block of a message whose last byte sits
    at P >= 55 of block Kp (bm_sha256.hpp pad_kw_const(P, Kp)).  Here those 64
    words are rebuilt from standard SHA-256 padding (FIPS 180-4: 0x80, zeros,
    the 64-bit bit length) and the block schedule, and the full hash (the
    message blocks from the IV, then the padding block with them) equals
    hashlib's."""
    from sharef import K
    rot = lambda x, n: ((x >> n) | (x << (32 - n))) & 0xFFFFFFFF
    table = _padc_kw_table(Kp)
    for P in range(55, 64):
        msg = bytes(0x41 + i % 26 for i in range(64 * Kp + P + 1))   # last byte at P of block Kp
        padded = msg + b"\x80" + b"\0" * ((55 - len(msg)) % 64) + (8 * len(msg)).to_bytes(8, "big")
        assert len(padded) == 64 * (Kp + 2)
        last = 64 * (Kp + 1)
        w = [int.from_bytes(padded[last + 4 * i: last + 4 + 4 * i], "big") for i in range(16)]
        assert w[1:15] == [0] * 14 and w[0] == (0x80000000 if P == 63 else 0) and w[15] == 8 * (64 * Kp + P + 1)
        for t in range(16, 64):
            s0 = rot(w[t - 15], 7) ^ rot(w[t - 15], 18) ^ (w[t - 15] >> 3)
            s1 = rot(w[t - 2], 17) ^ rot(w[t - 2], 19) ^ (w[t - 2] >> 10)
            w.append((w[t - 16] + s0 + w[t - 7] + s1) & 0xFFFFFFFF)
        assert table[P] == [(K[t] + w[t]) & 0xFFFFFFFF for t in range(64)], P
        st = list(IV)
        for b in range(Kp + 1):
            st = compress(st, [int.from_bytes(padded[64 * b + 4 * i: 64 * b + 4 * i + 4], "big") for i in range(16)])
        st = compress(st, w[:16])
        assert b"".join(x.to_bytes(4, "big") for x in st) == hashlib.sha256(msg).digest()
