"""Multi-rank sharding on CPU: the range split (dist.split_range, the mirror of
bm::split_range), the lexicographic combine, and the torchrun-style
rendezvous (distributed_bitcoin_minter_amd/rendezvous.py: files on the node,
no torch) at world sizes 2, 4 and 8.  On CPU each rank's scan is the oracle;
the same workers run the HIP search in the -m gpu variant (every rank on
GPU 0), so no N>1 test is left without the real kernels."""
import json
import os
import random
import socket
import subprocess
import sys

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


def test_split_range_weak_scaling_pieces():
    """bench.py's weak-scaling ranges [0, N*2^32-1] split into exactly the
    per-GPU pieces [r*2^32, (r+1)*2^32-1] the goldens are keyed on."""
    for n in (1, 2, 4, 8):
        assert split_range(0, n * 2 ** 32 - 1, n) == [(r * 2 ** 32, (r + 1) * 2 ** 32 - 1) for r in range(n)]


def test_lex_min_tie_goes_to_smallest_nonce():
    assert lex_min([(5, 9), (5, 3), (7, 1)]) == (5, 3)
    assert lex_min([]) == (U64, U64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# One rank: rendezvous (node files), a broadcast of rank 0's bytes (the
# RCCL unique id's path), its piece scanned (oracle on CPU, HIP on GPU),
# gather + lexicographic min, max over ranks.
_RANK = r"""
import json, os, sys
root, mode, msg_hex, lo, hi = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
sys.path[:0] = [root, os.path.join(root, "tests")]
from distributed_bitcoin_minter_amd.dist import lex_min, rank_piece
from distributed_bitcoin_minter_amd.rendezvous import Rendezvous
msg = bytes.fromhex(msg_hex)
if mode == "gpu":
    from distributed_bitcoin_minter_amd import Context
    ctx = Context(devices=[0])
    scan = ctx.search
else:
    from conftest import Oracle
    scan = Oracle(os.path.join(root, "oracle", "liboracle.so")).search
with Rendezvous(timeout_s=120) as rz:
    token = rz.broadcast_bytes(os.urandom(128) if rz.rank == 0 else None)
    piece = rank_piece(lo, hi, rz.rank, rz.world)
    part = scan(msg, *piece) if piece else (2**64 - 1, 2**64 - 1)
    res = lex_min(tuple(p) for p in rz.all_gather(list(part)))
    mx = rz.all_max(float(rz.rank))
    rz.barrier()
print(json.dumps({"rank": rz.rank, "token": token.hex(), "res": list(res), "max": mx, "piece": piece}))
"""


def _run_ranks(world, mode, msg, lo, hi):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(world))
        procs.append(subprocess.Popen([sys.executable, "-c", _RANK, ROOT, mode, msg.hex(), str(lo), str(hi)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, e[-3000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    return outs


def _check(outs, world, want, lo, hi):
    assert len({o["token"] for o in outs}) == 1  # rank 0's bytes reached every rank
    assert all(o["max"] == world - 1 for o in outs)
    assert all(tuple(o["res"]) == want for o in outs), outs
    pieces = [tuple(o["piece"]) for o in sorted(outs, key=lambda o: o["rank"]) if o["piece"]]
    assert pieces == split_range(lo, hi, world)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rendezvous_combine_equals_single_scan(oracle, world):
    msg, lo, hi = b"bradfitz", 0, 99_999
    _check(_run_ranks(world, "cpu", msg, lo, hi), world, oracle.search(msg, lo, hi), lo, hi)


def test_rendezvous_range_shorter_than_world(oracle):
    msg, lo, hi = b"msg", 1, 2  # 2 nonces over 4 ranks: ranks 2, 3 scan nothing
    outs = _run_ranks(4, "cpu", msg, lo, hi)
    assert [o["piece"] for o in sorted(outs, key=lambda o: o["rank"])] == [[1, 1], [2, 2], None, None]
    assert all(tuple(o["res"]) == oracle.search(msg, lo, hi) for o in outs)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_rendezvous_ranks_on_gpu(oracle, world):
    """The same ranks with the HIP search (every rank on GPU 0): a window
    across the 9->10 digit boundary, split over the ranks."""
    msg, lo, hi = b"bradfitz", 999_000_000, 1_000_999_999
    _check(_run_ranks(world, "gpu", msg, lo, hi), world, oracle.search(msg, lo, hi, threads=8), lo, hi)


def _gloo_worker(rank, world, port, msg, lo, hi, q):
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
    q.put((rank, combine(part)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_torch_gloo_combine_equals_single_scan(oracle, world):
    """dist.combine, the torch.distributed form of the combine (one
    all_gather_into_tensor of 2 x u64 per rank; RCCL under the "nccl" backend,
    tests/test_dist_gpu.py), over gloo at world sizes 2 and 4, with the oracle
    as each rank's scan: the lexicographic min equals one scan of the range,
    including partials >= 2^63 (two's-complement transport)."""
    import multiprocessing as mp
    for msg, lo, hi in ((b"bradfitz", 0, 99_999), (b"bradfitz", U64 - 5000, U64)):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, msg, lo, hi, q)) for r in range(world)]
        for p in procs:
            p.start()
        out = [q.get(timeout=120) for _ in procs]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert all(res == oracle.search(msg, lo, hi) for _, res in out), out


def test_rendezvous_key_separates_elastic_restarts(tmp_path, monkeypatch):
    """a torchrun elastic restart keeps the agent (the parent pid)
    and the master address and port, so the rendezvous directory is also keyed
    by the run id and the restart count: a restarted group never meets the
    failed attempt's files."""
    from distributed_bitcoin_minter_amd.rendezvous import Rendezvous
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29500")
    monkeypatch.delenv("BTCMINER_RDZV_DIR", raising=False)
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    import tempfile
    monkeypatch.setattr(tempfile, "tempdir", str(tmp_path))
    paths = []
    for run_id, restart in (("abc", "0"), ("abc", "1"), ("xyz/1", "0")):
        monkeypatch.setenv("TORCHELASTIC_RUN_ID", run_id)
        monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", restart)
        with Rendezvous(timeout_s=10) as rz:
            paths.append(rz.path)
            assert rz.all_gather(7) == [7]
    assert len(set(paths)) == 3 and all(os.path.dirname(p) == str(tmp_path) for p in paths)
