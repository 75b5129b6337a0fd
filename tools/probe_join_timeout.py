#!/usr/bin/env python3
"""Diagnostic: rank 0 of a 2-rank group joins alone with a join timeout
(bm_ctx_join_rank's non-blocking init on a worker thread), twice, then
searches its own piece and closes.  The first join times out with its worker
still inside RCCL's bootstrap; the second must not start another worker (it
waits on the pending one, then times out too).  Prints the OS thread count
after each step.  Run with BTCMINER_TRACE=1 under an outer `timeout`."""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_bitcoin_minter_amd import BtcMinerError, Context, rccl_unique_id  # noqa: E402


def threads():
    return len(os.listdir("/proc/self/task"))


faulthandler.dump_traceback_later(int(os.environ.get("PROBE_DUMP_S", "60")), exit=False)
timeout_ms = int(os.environ.get("PROBE_TIMEOUT_MS", "3000"))
t = time.monotonic()
with Context(devices=[0], rank=0, world=2) as c:
    uid = rccl_unique_id()
    print(f"threads before join {threads()}", flush=True)
    for k in (1, 2):
        t1 = time.monotonic()
        try:
            c.join(uid, timeout_ms=timeout_ms)
            print("joined?!", flush=True)
        except BtcMinerError as e:
            print(f"join {k} failed after {time.monotonic() - t1:.1f} s: {e}", flush=True)
        print(f"threads after join {k} {threads()}", flush=True)
    print("search", c.search(b"msg", 0, 3), f"{time.monotonic() - t:.1f} s", flush=True)
print(f"closed after {time.monotonic() - t:.1f} s", flush=True)
