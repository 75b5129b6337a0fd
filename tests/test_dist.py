"""Multi-rank sharding (distributed_bitcoin_minter_amd/dist.py) on CPU with
gloo, world_size 2 and 4: each rank scans its piece (with the CPU oracle
standing in for the per-rank GPU search), one all_gather of 16-byte
partials, lexicographic min == the single-process scan.

torch is imported only inside the spawned workers: the pytest process
keeps a single HIP runtime (/opt/rocm's) for the GPU tests."""
import multiprocessing as mp
import os
import random
import socket

import pytest

from conftest import ROOT, U64
from distributed_bitcoin_minter_amd.dist import lex_min, rank_piece, split_range


def test_split_range_tiles_exactly():
    rng = random.Random(0x5EED)
    cases = [(0, U64, 8), (0, 0, 8), (5, 9, 8), (U64 - 3, U64, 2), (0, 2 ** 40 - 1, 8)]
    cases += [(a, a + rng.randint(0, 10 ** 6), rng.randint(1, 9)) for a in [rng.randint(0, 2 ** 63) for _ in range(50)]]
    for lo, hi, n in cases:
        p = split_range(lo, hi, n)
        assert p[0][0] == lo and p[-1][1] == hi and len(p) == min(n, hi - lo + 1)
        for (a, b), (c, d) in zip(p, p[1:]):
            assert b + 1 == c and a <= b
        sizes = [b - a + 1 for a, b in p]
        assert max(sizes) - min(sizes) <= 1


def test_lex_min_tie_goes_to_smallest_nonce():
    assert lex_min([(5, 9), (5, 3), (7, 1)]) == (5, 3)
    assert lex_min([]) == (U64, U64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, msg, lo, hi, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from conftest import Oracle
    from distributed_bitcoin_minter_amd.dist import combine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    oracle = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
    piece = rank_piece(lo, hi, rank, world)
    part = oracle.search(msg, *piece) if piece else (U64, U64)
    res = combine(part)
    q.put((rank, res))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_combine_equals_single_scan(oracle, world):
    msg, lo, hi = b"bradfitz", 0, 99_999
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, msg, lo, hi, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = oracle.search(msg, lo, hi)
    assert all(res == expect for _, res in out), out
