#!/usr/bin/env python3
"""A/B the search kernels of several libbtcminer builds on the GPU.

    python tools/ab_bench.py distributed_bitcoin_minter_amd/libbtcminer*.so
    python tools/ab_bench.py BTCMINER_STREAMS=2 BTCMINER_STREAMS=1,BTCMINER_CHUNK=200

Each library runs in its own process (BTCMINER_LIB): C2 ("bradfitz",
[0, 2^32-1]) and C3 (120-B msg, [2^64-2^32, 2^64-1]), checked against the
goldens, best-of-N wall time and per-launch HIP-event times.  No torch."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(reps):
    sys.path.insert(0, ROOT)
    from distributed_bitcoin_minter_amd import Context
    gold = {c["config"]: c for c in json.load(open(os.path.join(ROOT, "tests/golden/full_range.json")))["cases"]}
    out = {"lib": os.environ.get("AB_TAG") or os.path.basename(os.environ.get("BTCMINER_LIB", "default"))}
    bpc = int(os.environ.get("AB_BPC", "0"))
    with Context(devices=[0]) as ctx:
        ctx.set_timing(True)
        if bpc:
            ctx.set_blocks_per_cu(bpc)
        for cfg in ("C2", "C3"):
            c = gold[cfg]
            msg = bytes.fromhex(c["msg_hex"])
            best = None
            for _ in range(reps):
                r = ctx.search(msg, c["lower"], c["upper"])
                assert r == (c["hash"], c["nonce"]), (cfg, r)
                st = ctx.last_stats()
                if best is None or st.wall_ms < best[0]:
                    launches = sorted(((st.launch[i].nonces, st.launch[i].ms, st.launch[i].p, st.launch[i].grid)
                                       for i in range(st.recorded)), reverse=True)[:3]
                    best = (st.wall_ms, st.kernel_ms, launches)
            n = c["upper"] - c["lower"] + 1
            dom = best[2][0]
            out[cfg] = {"wall_ms": round(best[0], 3), "GHs": round(n / best[0] / 1e6, 3),
                        "dom_GHs": round(dom[0] / dom[1] / 1e6, 3) if dom[1] > 0 else None, "dom": dom,
                        "top": best[2]}
    print(json.dumps(out), flush=True)


def main():
    if os.environ.get("AB_CHILD"):
        return one(int(os.environ.get("AB_REPS", "5")))
    for arg in sys.argv[1:]:
        # a library path, or KEY=VALUE[,KEY=VALUE...]: the default library
        # under those environment knobs (BTCMINER_STREAMS, BTCMINER_CHUNK, ...)
        if "=" in arg:
            extra = dict(kv.split("=", 1) for kv in arg.split(","))
            lib = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "libbtcminer.so")
        else:
            extra, lib = {}, arg
        env = dict(os.environ, BTCMINER_LIB=os.path.abspath(lib), AB_CHILD="1", AB_TAG=arg, **extra)
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, timeout=300)
        if r.returncode != 0:
            print(json.dumps({"lib": lib, "rc": r.returncode}), flush=True)
            if r.returncode not in (0, 1):
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
