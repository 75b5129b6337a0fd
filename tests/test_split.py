"""The multi-GPU range partitioner (bm::slot_pieces via bm_split_range, pure
CPU) and its Python mirror (dist.slot_pieces): exact tiling of [lower, upper]
in slot order, sizes in proportion to the shares within one nonce, identical
pieces from the library and the mirror (so every rank of a group, and the
bench's one-GPU rehearsal, cut the same pieces), and the near-equal default.
Results never depend on the split (the lexicographic min);
the GPU side is in tests/test_gpu_multi.py."""
import random

import pytest

from conftest import U64
from distributed_bitcoin_minter_amd import _lib
from distributed_bitcoin_minter_amd.dist import shares_from_rates, slot_pieces, split_range


def _cases():
    rng = random.Random(0x5EED)
    out = [(0, U64, [1, 1]), (0, U64, [3, 5, 7]), (0, 2 ** 35 - 1, [65536, 61000, 65000, 64000, 65536, 60000, 63000,
                                                                  65536]),
           (5, 9, [1, 1, 1, 1, 1, 1, 1, 1]), (7, 7, [2, 9]), (U64 - 3, U64, [1, 1000]), (0, 99, [1, 1, 98])]
    for _ in range(300):
        n = rng.randint(1, 9)
        lo = rng.choice([0, rng.randint(0, 2 ** 40), rng.randint(0, U64)])
        hi = min(U64, lo + rng.choice([0, rng.randint(0, 50), rng.randint(0, 2 ** 36), U64]))
        out.append((lo, hi, [rng.choice([1, rng.randint(1, 70000), rng.randint(1, 2 ** 32 - 1)]) for _ in range(n)]))
    return out


def _check_tiling(lo, hi, pieces):
    cur = lo
    for p in pieces:
        if p is None:
            continue
        assert p[0] == cur and p[0] <= p[1]
        cur = p[1] + 1
    assert cur == hi + 1


@pytest.mark.parametrize("lo,hi,shares", _cases())
def test_weighted_pieces_tile_in_proportion(lo, hi, shares):
    got = _lib.split_range(lo, hi, len(shares), shares)
    assert got == slot_pieces(lo, hi, len(shares), shares)
    _check_tiling(lo, hi, got)
    count, total = hi - lo + 1, sum(shares)
    for p, s in zip(got, shares):
        size = 0 if p is None else p[1] - p[0] + 1
        assert abs(size * total - count * s) <= 2 * total  # within about one nonce (floor at both ends)


def test_default_is_the_near_equal_split():
    rng = random.Random(7)
    for _ in range(200):
        n = rng.randint(1, 9)
        lo = rng.randint(0, U64)
        hi = min(U64, lo + rng.choice([0, 3, rng.randint(0, 10 ** 9), U64]))
        want = split_range(lo, hi, n)
        assert _lib.split_range(lo, hi, n) == want + [None] * (n - len(want))
        assert slot_pieces(lo, hi, n) == want + [None] * (n - len(want))
        assert slot_pieces(lo, hi, n, [1] * (n + 1)) == want + [None] * (n - len(want))  # wrong count: default


def test_weak_scaling_pieces_with_shares():
    """bench.py's weak-scaling range [0, 8*2^32-1] over 8 GPUs whose rates
    differ by a few percent: pieces follow the rates, tile the range, and the
    fastest GPU gets the largest piece."""
    rates = [54.9, 53.1, 54.2, 52.8, 55.0, 54.4, 53.7, 54.0]
    sh = shares_from_rates(rates)
    assert max(sh) == 65536 and min(sh) >= 1
    pieces = _lib.split_range(0, 8 * 2 ** 32 - 1, 8, sh)
    _check_tiling(0, 8 * 2 ** 32 - 1, pieces)
    sizes = [b - a + 1 for a, b in pieces]
    assert sizes.index(max(sizes)) == rates.index(max(rates))
    for s, r in zip(sizes, rates):
        assert abs(s / (8 * 2 ** 32) - r / sum(rates)) < 1e-4


def test_invalid_arguments():
    with pytest.raises(_lib.BtcMinerError):
        _lib.split_range(0, 10, 2, [1, 0])  # every share >= 1
    with pytest.raises(_lib.BtcMinerError):
        _lib.split_range(0, 10, 0)
    assert _lib.split_range(10, 5, 3, [1, 2, 3]) == [None, None, None]  # empty range


def test_calibrated_rates_ignore_one_outlier_step():
    """rank-mode calibration takes each rank's median over its
    warmup steps after the first, and holds a rank at 0.85 of the fastest
    unless two of its steps agree it is slower.  One injected outlier step
    (a clock ramp, a late code-object load) leaves the shares within 2% of the
    steady rates; a rank that is persistently 20% slower keeps its rate."""
    from distributed_bitcoin_minter_amd.dist import calibrated_rates, shares_from_rates
    steady = [54.0, 53.2, 55.1, 54.6]
    steps = [[r * (1 + 0.001 * k) for k in range(4)] for r in steady]
    steps[1][2] = 20.0          # one transient step on rank 1
    steps[3][0] = 90.0          # one absurdly fast step on rank 3
    rates, info = calibrated_rates(steps)
    want = shares_from_rates(steady)
    got = shares_from_rates(rates)
    assert all(abs(g - w) <= 0.02 * w for g, w in zip(got, want)), (got, want)
    assert info["clamped"] == [] and info["spread"][1] > 0.6 and info["spread"][0] < 0.01
    # a persistently slow rank: its steps agree, so its rate stands
    slow = [[43.0, 43.2, 43.1], [54.0, 54.1, 53.9]]
    rates, info = calibrated_rates(slow)
    assert info["clamped"] == [] and abs(rates[0] - 43.1) < 1e-9
    # a rank low in two steps that disagree (46 vs 30): held at 0.85 of the fastest
    rates, info = calibrated_rates([[46.0, 30.0], [54.0, 54.0]])
    assert info["clamped"] == [0] and abs(rates[0] - 0.85 * 54.0) < 1e-9
    # one step per rank (warmup 2): the median is that step; a single low
    # step cannot agree with another, so below 0.85 of the fastest it is held
    assert calibrated_rates([[50.0], [54.0]])[0] == [50.0, 54.0]
    assert calibrated_rates([[40.0], [54.0]])[0] == [0.85 * 54.0, 54.0]
