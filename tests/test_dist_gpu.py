"""The one-process-per-GPU combine over torch.distributed's "nccl" backend
(RCCL on ROCm), as bench.py --gpus N runs it, exercised at world size 1 on the
box's one GPU: init_process_group("nccl", device_id=cuda:0), a search through
the C ABI, then dist.combine's all_gather_into_tensor of the 16-byte partial
on the device.  The result must equal the direct search and the oracle's scan.
(World sizes 2 and 4 of the same code run on gloo in tests/test_dist.py; the
8-GPU run is the driver's.)"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import json, os, sys
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["BM_ROOT"])
from distributed_bitcoin_minter_amd import Context
from distributed_bitcoin_minter_amd.dist import combine, rank_piece
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
lo, hi = 999_000_000, 1_000_999_999
piece = rank_piece(lo, hi, dist.get_rank(), dist.get_world_size())
with Context(devices=[0]) as ctx:
    part = ctx.search(b"bradfitz", *piece)
    got = combine(part, device=dev)
    direct = ctx.search(b"bradfitz", lo, hi)
dist.destroy_process_group()
print(json.dumps({"got": list(got), "direct": list(direct)}))
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_nccl_combine_world1(oracle):
    env = dict(os.environ, BM_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    want = oracle.search(b"bradfitz", 999_000_000, 1_000_999_999, threads=8)
    assert tuple(out["got"]) == tuple(out["direct"]) == want
