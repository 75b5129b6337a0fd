#!/usr/bin/env python3
"""Diagnostic: rank 0 of a 2-rank group joins alone with a join timeout
(bm_ctx_join_rank's non-blocking init, then abort).  Run with
BTCMINER_TRACE=1 under an outer `timeout`; prints which step returns."""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_bitcoin_minter_amd import BtcMinerError, Context, rccl_unique_id  # noqa: E402

faulthandler.dump_traceback_later(int(os.environ.get("PROBE_DUMP_S", "40")), exit=False)
t = time.monotonic()
with Context(devices=[0], rank=0, world=2) as c:
    try:
        c.join(rccl_unique_id(), timeout_ms=int(os.environ.get("PROBE_TIMEOUT_MS", "3000")))
        print("joined?!", flush=True)
    except BtcMinerError as e:
        print(f"join failed after {time.monotonic() - t:.1f} s: {e}", flush=True)
    print("search", c.search(b"msg", 0, 3), f"{time.monotonic() - t:.1f} s", flush=True)
print(f"closed after {time.monotonic() - t:.1f} s", flush=True)
