#!/usr/bin/env python3
"""BASELINE config C5 with every process native: the C++ bitcoin server
(examples/bm_server), C++ GPU miners (examples/bm_miner, one bm_ctx each, over
the C ABI) and C++ request clients (examples/bm_client), all on lsp.hpp, under
lspnet 10% read and write drop at every endpoint.

    python tools/bench_c5_native.py [--max-nonce-bits 34] [--chunk-bits 32] [--miners 4]
                                    [--clients 16] [--drop 10] [--epoch-ms 50] [--gpus 1]

This process only starts programs and reads their output: it opens no GPU.
Miner i runs on device i % --gpus.  Before the clock starts, one warm-up
client per miner asks for 2^33 nonces, so every miner has loaded its code
objects.  Client i then asks for msg "client-%02d" over [0, 2^bits - 1].
Prints one JSON line: GH/s = all clients' nonces / wall time from the first
client's start to the last client's exit.  Every "Result <hash> <nonce>" line
is checked against the full CPU scans in tests/golden/c5_clients.json.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-nonce-bits", type=int, default=34)
    ap.add_argument("--chunk-bits", type=int, default=32)
    ap.add_argument("--miners", type=int, default=4)
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--drop", type=int, default=10)
    ap.add_argument("--epoch-ms", type=int, default=50)
    ap.add_argument("--epoch-limit", type=int, default=100)
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--window", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--timeout", type=float, default=240.0)
    a = ap.parse_args()

    lsp_flags = ["--epoch-millis", str(a.epoch_ms), "--epoch-limit", str(a.epoch_limit),
                 "--window-size", str(a.window)]
    drops = ["--drop-read", str(a.drop), "--drop-write", str(a.drop)]
    srv = subprocess.Popen([os.path.join(EX, "bm_server"), "0", "--chunk", str(1 << a.chunk_bits), "--depth",
                            str(a.depth), "-v", *lsp_flags, *drops],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    procs = [srv]
    try:
        first = srv.stdout.readline().split()
        assert first[:1] == ["port"], first
        hostport = f"127.0.0.1:{first[1]}"
        joined = []
        lost = []

        def watch():  # the server's -v log: joins and losses
            for ln in srv.stderr:
                if "joined" in ln:
                    joined.append(ln)
                elif "lost" in ln:
                    lost.append(ln)
        threading.Thread(target=watch, daemon=True).start()

        logs = [tempfile.TemporaryFile() for _ in range(a.miners)]
        miners = [subprocess.Popen([os.path.join(EX, "bm_miner"), hostport, "--device", str(i % a.gpus),
                                    *lsp_flags, *drops], stdout=subprocess.DEVNULL, stderr=logs[i])
                  for i in range(a.miners)]
        procs += miners
        t_end = time.monotonic() + 60
        while len(joined) < a.miners:
            dead = [m.returncode for m in miners if m.poll() is not None]
            if dead or time.monotonic() > t_end:
                for f in logs:
                    f.seek(0)
                    print(f.read().decode(errors="replace")[-2000:], file=sys.stderr)
                raise SystemExit(f"only {len(joined)} of {a.miners} miners joined (exited: {dead})")
            time.sleep(0.01)

        def clients(msgs, top):
            return [subprocess.Popen([os.path.join(EX, "bm_client"), hostport, m, str(top), *lsp_flags, *drops],
                                     stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for m in msgs]

        warm = clients([f"warmup-{i}" for i in range(a.miners)], (1 << 33) - 1)
        for c in warm:
            c.communicate(timeout=a.timeout)

        top = (1 << a.max_nonce_bits) - 1
        msgs = [f"client-{i:02d}" for i in range(a.clients)]
        t0 = time.perf_counter()
        cs = clients(msgs, top)
        procs += cs
        outs = [c.communicate(timeout=a.timeout)[0] for c in cs]
        wall = time.perf_counter() - t0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()

    got = {}
    for m, o in zip(msgs, outs):
        f = o.split()
        got[m] = (int(f[1]), int(f[2])) if len(f) == 3 and f[0] == "Result" else None
    total = a.clients * (top + 1)
    out = {"config": "C5", "native": "bm_server + bm_miner (C ABI) + bm_client, all C++ on lsp.hpp",
           "clients": a.clients, "miners": a.miners, "gpus": a.gpus, "drop_pct": a.drop, "epoch_ms": a.epoch_ms,
           "window": a.window, "depth": a.depth, "max_nonce": top, "chunk": 1 << a.chunk_bits,
           "seconds": round(wall, 3), "GHs": round(total / wall / 1e9, 3),
           "all_answered": all(v is not None for v in got.values()), "miners_lost": len(lost)}
    gpath = os.path.join(ROOT, "tests", "golden", "c5_clients.json")
    if os.path.exists(gpath):
        gold = json.load(open(gpath))
        if gold["upper"] == top:
            out["golden_checked"] = sum(1 for m in msgs if m in gold["clients"])
            out["golden_ok"] = all(tuple(gold["clients"][m]) == got[m] for m in msgs if m in gold["clients"])
    print(json.dumps(out), flush=True)
    return 0 if out["all_answered"] and out.get("golden_ok", True) else 1


if __name__ == "__main__":
    raise SystemExit(main())
