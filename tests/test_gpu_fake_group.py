"""The library's world > 1 group paths with live rank processes on ONE GPU.

Real RCCL refuses two ranks on one GPU, and every box of this pool has one, so
until round 5 the status-carrying allgather between live ranks, BM_EPEER, the
peer timeout and bench.py's joined-group line had never run (ADVICE r4,
medium).  Here the SAME library objects are linked against
tests/fake_rccl/fake_rccl.cpp (test infrastructure: the eleven RCCL calls the
library makes, with the allgather done on the host in stream order through
shared memory; `make -C distributed_bitcoin_minter_amd/csrc fakerccl`), and
2-3 rank processes share GPU 0.  What this pins is the library's own logic
above RCCL: slot staging, the status word, the peer timeout and its abort,
leave, the rank pieces, and bench.py's N > 1 line with an RCCL combine.  RCCL's
transport over xGMI is not emulated; the driver's 8-GPU node runs that, and
test_rank_group_epeer_two_gpus (test_gpu_multi.py) there.
"""
import glob
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, load_golden

pytestmark = pytest.mark.gpu

FAKE_LIB = os.path.join(ROOT, "tests", "fake_rccl", "libbtcminer_fakerccl.so")
C2 = next(c for c in load_golden("full_range.json")["cases"] if c["config"] == "C2")


def _need_fake():
    if not os.path.exists(FAKE_LIB):
        pytest.skip("tests/fake_rccl/libbtcminer_fakerccl.so not built (make -C distributed_bitcoin_minter_amd/csrc "
                    "fakerccl)")


def _port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cleanup_shm(before):
    for p in set(glob.glob("/dev/shm/fakerccl-*")) - before:
        try:
            os.unlink(p)
        except OSError:
            pass


_RANK_GROUP = r"""
import json, os, sys, time
sys.path.insert(0, sys.argv[1])
from distributed_bitcoin_minter_amd import _lib
_lib.load()   # BTCMINER_LIB: the library linked against the fake RCCL
from distributed_bitcoin_minter_amd import BtcMinerError, Context, rccl_unique_id
from distributed_bitcoin_minter_amd.rendezvous import Rendezvous
msg = b"bradfitz"
shares = json.loads(sys.argv[2])
out = {}

def attempt(c, lo, hi):
    try:
        return list(c.search(msg, lo, hi))
    except BtcMinerError as e:
        return e.status

with Rendezvous(timeout_s=120) as rz:
    uid = rz.broadcast_bytes(rccl_unique_id() if rz.rank == 0 else None)
    with Context(devices=[0], rank=rz.rank, world=rz.world) as c:
        t = time.time()
        c.join(uid, timeout_ms=60_000)
        out["join_s"] = round(time.time() - t, 3)
        c.set_peer_timeout(60_000)
        c.set_timing(True)
        out["ok"] = attempt(c, 0, 9999)
        st = c.last_stats()
        out["stats"] = [st.rccl_nranks, st.rccl_rank, st.dev_rccl_device[0], st.rccl_version, st.combine_used,
                        st.nonces]
        out["ag_ms"], out["init_ms"] = st.rccl_allgather_ms, st.rccl_init_ms
        out["big"] = attempt(c, 999_000_000, 1_000_999_999)
        out["c2"] = attempt(c, 0, 2**32 - 1)
        c.set_split(shares)                       # the same shares on every rank
        out["split"] = attempt(c, 0, 9999)
        out["split_nonces"] = c.last_stats().nonces
        c.set_split(None)
        if rz.rank == 1:
            c.set_test_fault(0)                   # this rank fails before the combine
        out["fault"] = attempt(c, 0, 9999)
        c.set_test_fault(-1)
        out["after"] = attempt(c, 0, 9999)        # the group survived
        if rz.rank == 0:                          # the others never come to this search
            c.set_peer_timeout(2000)
            t = time.time()
            out["timeout"] = attempt(c, 0, 9999)
            out["timeout_s"] = round(time.time() - t, 3)
            out["still"] = attempt(c, 0, 9999)    # the communicator is gone until leave()
        rz.barrier()
        c.leave()
        out["local"] = attempt(c, 0, 9999)        # this rank's own piece again
        out["local_combine"] = c.last_stats().combine_used
        rz.barrier()
print(json.dumps(dict(out, rank=rz.rank, world=rz.world)))
"""


@pytest.mark.parametrize("world,shares", [(2, [1, 3]), (3, [1, 3, 4])])
def test_fake_group_on_one_gpu(oracle, world, shares):
    """world rank processes on GPU 0 joined through the fake RCCL: every rank
    returns the whole range's answer (== oracle, == the C2 golden over 2^32),
    RCCL's view says `world` ranks, the weighted split cuts the pieces the
    partitioner promises, a rank that fails before the combine returns its own
    status while every other rank gets BM_EPEER, the group then answers again,
    a rank whose peers never come gets BM_ETIMEDOUT after its peer timeout
    (and again until leave()), and after leave() each rank returns its own
    piece's partial."""
    _need_fake()
    from distributed_bitcoin_minter_amd import _lib
    from distributed_bitcoin_minter_amd._lib import (BM_COMBINED_LOCAL, BM_COMBINED_RCCL, BM_EINTERNAL, BM_EPEER,
                                                     BM_ETIMEDOUT)
    before = set(glob.glob("/dev/shm/fakerccl-*"))
    port = _port()
    procs = []
    try:
        for r in range(world):
            env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                       WORLD_SIZE=str(world), BTCMINER_LIB=FAKE_LIB)
            procs.append(subprocess.Popen([sys.executable, "-c", _RANK_GROUP, ROOT, json.dumps(shares)], env=env,
                                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        outs = []
        for p in procs:
            o, e = p.communicate(timeout=240)
            assert p.returncode == 0, e[-3000:]
            outs.append(json.loads(o.strip().splitlines()[-1]))
    finally:
        for p in procs:  # never leave a rank holding the GPU
            if p.poll() is None:
                p.kill()
                p.wait()
        _cleanup_shm(before)
    outs.sort(key=lambda o: o["rank"])
    small = [1419516646206828, 9898]
    big = list(oracle.search(b"bradfitz", 999_000_000, 1_000_999_999, threads=8))
    pieces = _lib.split_range(0, 9999, world)
    wpieces = _lib.split_range(0, 9999, world, shares)
    for r, o in enumerate(outs):
        assert o["ok"] == small and o["big"] == big and o["c2"] == [C2["hash"], C2["nonce"]], o
        n = pieces[r][1] - pieces[r][0] + 1
        assert o["stats"] == [world, r, 0, 1, BM_COMBINED_RCCL, n], o["stats"]  # version 1: the fake ran
        assert o["ag_ms"] > 0 and o["init_ms"] > 0, o
        assert o["split"] == small and o["split_nonces"] == wpieces[r][1] - wpieces[r][0] + 1, o
        assert o["fault"] == (BM_EINTERNAL if r == 1 else BM_EPEER), o
        assert o["after"] == small, o
        assert o["local"] == list(oracle.search(b"bradfitz", *pieces[r])) and o["local_combine"] == BM_COMBINED_LOCAL
    assert outs[0]["timeout"] == BM_ETIMEDOUT and 1.5 < outs[0]["timeout_s"] < 30, outs[0]
    assert outs[0]["still"] == BM_ETIMEDOUT, outs[0]


def test_bench_torchrun_joined_group_line():
    """bench.py's N > 1 torchrun path with the group JOINED (the driver's
    8-GPU launch shape, which RCCL never let run on this pool): 2 ranks on
    GPU 0 through the fake RCCL.  The line combines over the group's
    allgather, carries the RCCL block (the fake's version 1, the init and the
    allgather's event pair), the rank rates' split, the start skew and a C4
    step combined over the group, every answer == its golden; and it says it
    is no scaling measurement because both ranks share one GPU -- for that
    reason only."""
    _need_fake()
    before = set(glob.glob("/dev/shm/fakerccl-*"))
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0", BTCMINER_LIB=FAKE_LIB)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "2"]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=300)
    except subprocess.TimeoutExpired:
        import signal
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        pytest.fail(f"bench did not finish in 300 s: {err[-2000:]}")
    finally:
        _cleanup_shm(before)
    assert p.returncode == 0, err[-3000:]
    line = json.loads(out.strip().splitlines()[-1])
    cfg = line["config"]
    assert line["result_ok"] is True and "RCCL allgather" in cfg["parallelism"], cfg["parallelism"]
    ranks = sorted(cfg["ranks"], key=lambda r: r["rank"])
    assert [r["combine"] for r in ranks] == ["rccl", "rccl"] and [r["rccl_rank"] for r in ranks] == [0, 1]
    assert line["rccl_nranks"] == [2] and all(r["allgather_ms"] > 0 for r in ranks), ranks
    rc = line["rccl"]
    assert rc["version"] == 1 and rc["version_str"] == "0.0.1" and rc["init_ms"] > 0, rc
    assert 0 < rc["allgather_ms_min"] <= rc["allgather_ms_max"], rc
    assert cfg["split"]["mode"].startswith("measured rank rates") and len(cfg["split"]["shares"]) == 2
    # the median over the warmup steps after the first (here one), with its spread
    assert "median of warmup steps 2..2" in cfg["split"]["mode"] and len(cfg["split"]["spread"]) == 2
    assert line["start_skew_ms"] >= 0 and all("start_offset_ms" in r for r in ranks)
    assert line["scaling_valid"] is False and line["scaling_invalid"] == [
        "1 distinct GPUs (PCI bus ids) under 2 ranks / devices"], line["scaling_invalid"]
    c4 = line["c4"]
    assert c4["result_ok"] is True and c4["combine"] == "rccl" and c4["nonces"] == 2 ** 40, c4
    assert sum(r["nonces"] for r in c4["ranks"]) == 2 ** 40 and all(r["allgather_ms"] > 0 for r in c4["ranks"])
    # the one-process C4 block; HIP_VISIBLE_DEVICES=0 leaves rank 0
    # one of the two devices a one-process context would need: skipped, and why
    one = line["c4_one_process"]
    assert "rank 0 sees 1 of 2 devices" in one["skipped"], one


_RANK_DIES = r"""
import json, os, sys, time
sys.path.insert(0, sys.argv[1])
from distributed_bitcoin_minter_amd import _lib
_lib.load()
from distributed_bitcoin_minter_amd import BtcMinerError, Context, rccl_unique_id
from distributed_bitcoin_minter_amd.rendezvous import Rendezvous
rz = Rendezvous(timeout_s=120)
uid = rz.broadcast_bytes(rccl_unique_id() if rz.rank == 0 else None)
c = Context(devices=[0], rank=rz.rank, world=rz.world)
c.join(uid, timeout_ms=60_000)
first = list(c.search(b"bradfitz", 0, 9999))
rz.barrier()
if rz.rank == 1:
    os._exit(3)                      # dies inside the group: no leave, no close
c.set_peer_timeout(2000)
t = time.time()
try:
    c.search(b"bradfitz", 0, 9999)
    status = 0
except BtcMinerError as e:
    status = e.status
waited = time.time() - t
t = time.time()
c.close()                            # teardown must not wait on the dead peer
print(json.dumps({"first": first, "status": status, "waited": round(waited, 3),
                  "close_s": round(time.time() - t, 3)}), flush=True)
os._exit(0)                          # no rendezvous goodbye: the peer is gone
"""


def test_fake_group_peer_dies():
    """A rank of a joined group dies (exits without leaving) after a search:
    the survivor's next search returns BM_ETIMEDOUT after its peer timeout
    instead of waiting for ever, and closing its context returns promptly
    (the communicator is aborted, never waited on)."""
    _need_fake()
    from distributed_bitcoin_minter_amd._lib import BM_ETIMEDOUT
    import shutil
    import tempfile
    before = set(glob.glob("/dev/shm/fakerccl-*"))
    port = _port()
    rdzv = tempfile.mkdtemp(prefix="btcminer-rdzv-dies-")  # the ranks exit without the rendezvous goodbye
    procs = []
    try:
        for r in range(2):
            env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                       WORLD_SIZE="2", BTCMINER_LIB=FAKE_LIB, BTCMINER_RDZV_DIR=rdzv)
            procs.append(subprocess.Popen([sys.executable, "-c", _RANK_DIES, ROOT], env=env, stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True))
        outs = [p.communicate(timeout=180) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        _cleanup_shm(before)
        shutil.rmtree(rdzv, ignore_errors=True)
    assert procs[1].returncode == 3, outs[1][1][-2000:]
    assert procs[0].returncode == 0, outs[0][1][-3000:]
    o = json.loads(outs[0][0].strip().splitlines()[-1])
    assert o["first"] == [1419516646206828, 9898] and o["status"] == BM_ETIMEDOUT, o
    assert 1.5 < o["waited"] < 30 and o["close_s"] < 10, o
