#!/usr/bin/env python3
"""Probe: does the driver's hwmon gfx clock (freq1_input) under the C2 search
agree with the PMC clock (GRBM_GUI_ACTIVE / 8 XCDs / duration)?  Samples every
card's freq1_input while C2 runs 30 times; the busy card is the one whose
clock rises."""
import glob
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import Context  # noqa: E402

paths = sorted(glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*/freq1_input"))
samples = {p: [] for p in paths}
stop = threading.Event()


def sampler(period):
    while not stop.is_set():
        t = time.perf_counter()
        for p in paths:
            try:
                samples[p].append(int(open(p).read()))
            except OSError:
                pass
        stop.wait(max(0.0, period - (time.perf_counter() - t)))


c = json.load(open(os.path.join(ROOT, "tests/golden/full_range.json")))["cases"]
c2 = next(x for x in c if x["config"] == "C2")
with Context(devices=[0]) as ctx:
    ctx.set_timing(True)
    ctx.search(b"bradfitz", 0, 2 ** 32 - 1)
    th = threading.Thread(target=sampler, args=(0.01,), daemon=True)
    th.start()
    t = time.perf_counter()
    for _ in range(30):
        assert ctx.search(b"bradfitz", 0, 2 ** 32 - 1) == (c2["hash"], c2["nonce"])
    dt = time.perf_counter() - t
    stop.set()
    th.join()
out = {"seconds": round(dt, 3), "GHs": round(30 * 2 ** 32 / dt / 1e9, 3)}
for p, v in samples.items():
    if v:
        out[p.split("/")[4]] = {"n": len(v), "mean_GHz": round(sum(v) / len(v) / 1e9, 4),
                                "min": min(v) / 1e9, "max": max(v) / 1e9}
print(json.dumps(out, indent=1))
