#!/usr/bin/env python3
"""BASELINE config C5: LSP server + 4 GPU miners + 16 concurrent clients under
lspnet 10% packet drop (read and write, every endpoint).

    python tools/bench_c5.py [--max-nonce-bits 34] [--chunk-bits 32] [--miners 4]
                             [--clients 16] [--drop 10] [--epoch-ms 50] [--depth 2] [--window 1]
                             [--slots 1] [--target-ms 300]

Client i asks for msg "client-%02d" over [0, 2^bits - 1].  The server cuts
every request into 2^chunk_bits-nonce jobs and spreads them
over the miners with its fair-share scheduler; each miner is miner.run over
its own bm_ctx (device i % visible GPUs: on a one-GPU box all four share it).
Prints one JSON line: whole-system GH/s = all clients' nonces / wall time from
the first request to the last answer, the same figure for the bare library
on the same GPUs, and the checks: every answer re-hashes to itself
(bm_hash_gpu), two clients' answers equal one whole-range bm_search_gpu call,
and every answer equals the full CPU scan in tests/golden/c5_clients.json.

--slots S makes each miner one context over S device slots (round 6: a
miner that drives several GPUs, as the Go shim's bm_ctx_create(0) does; on a
one-GPU box the S slots share GPU 0, so each call pays S pieces' fixed costs
on one GPU), and --target-ms is the server's per-miner job sizing
(server.chunk_for; 0 = every job one --chunk): the pair measures what
rate-sized jobs buy such a miner end to end.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_bitcoin_minter_amd import Context, Miner, client, device_count, lsp, lspnet, miner  # noqa: E402
from distributed_bitcoin_minter_amd.server import BitcoinServer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-nonce-bits", type=int, default=34)
    ap.add_argument("--chunk-bits", type=int, default=32)
    ap.add_argument("--miners", type=int, default=4)
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--drop", type=int, default=10)
    ap.add_argument("--epoch-ms", type=int, default=50)
    ap.add_argument("--epoch-limit", type=int, default=100)
    ap.add_argument("--depth", type=int, default=2, help="jobs queued per miner (server.DEFAULT_DEPTH)")
    ap.add_argument("--window", type=int, default=1, help="LSP WindowSize (params.go default 1)")
    ap.add_argument("--slots", type=int, default=1, help="device slots per miner (a multi-GPU miner's context)")
    ap.add_argument("--target-ms", type=int, default=300, help="server job sizing target (0: fixed chunks)")
    a = ap.parse_args()

    ndev = max(1, device_count())
    p = lsp.Params(EpochLimit=a.epoch_limit, EpochMillis=a.epoch_ms, WindowSize=a.window)
    lspnet.seed(0x5EED)
    srv = lsp.NewServer(0, p)
    bs = BitcoinServer(srv, chunk=1 << a.chunk_bits, depth=a.depth, target_ms=a.target_ms)
    hostport = f"127.0.0.1:{srv.port}"
    threads = [threading.Thread(target=bs.serve, daemon=True)]
    gminers = [Miner(devices=[i % ndev] * a.slots) for i in range(a.miners)]
    for m in gminers:
        m.search("warmup", 0, 1 << 20)  # code objects loaded before the clock starts
        threads.append(threading.Thread(target=miner.run, args=(hostport, p), kwargs={"searcher": m}, daemon=True))
    for t in threads:
        t.start()
    while bs.stats["joins"] < a.miners:
        time.sleep(0.01)

    lspnet.SetReadDropPercent(a.drop)
    lspnet.SetWriteDropPercent(a.drop)
    top = (1 << a.max_nonce_bits) - 1
    msgs = [f"client-{i:02d}" for i in range(a.clients)]
    got = {}
    done_at = {}

    def ask(i):
        got[i] = client.request(hostport, msgs[i], top, p)
        done_at[i] = time.perf_counter()

    cth = [threading.Thread(target=ask, args=(i,)) for i in range(a.clients)]
    t0 = time.perf_counter()
    for t in cth:
        t.start()
    for t in cth:
        t.join()
    wall = time.perf_counter() - t0
    lspnet.ResetDropPercent()
    stats = dict(bs.stats)
    bs.close()

    total = a.clients * (top + 1)
    out = {"config": "C5", "clients": a.clients, "miners": a.miners, "gpus": ndev, "drop_pct": a.drop,
           "epoch_ms": a.epoch_ms, "window": a.window, "depth": a.depth, "max_nonce": top, "chunk": 1 << a.chunk_bits,
           "slots_per_miner": a.slots, "target_ms": a.target_ms, "seconds": round(wall, 3),
           "GHs": round(total / wall / 1e9, 3), "server_stats": stats,
           "all_answered": all(got.get(i) is not None for i in range(a.clients))}
    with Context(devices=list(range(min(ndev, a.miners)))) as ctx:
        out["rehash_ok"] = all(ctx.hash_many(msgs[i].encode(), [got[i][1]]) == [got[i][0]]
                               for i in range(a.clients) if got.get(i))
        t = time.perf_counter()
        direct = [ctx.search(msgs[i].encode(), 0, top) for i in (0, a.clients - 1)]
        dt = time.perf_counter() - t
        out["direct_ok"] = direct == [got.get(0), got.get(a.clients - 1)]
        out["library_GHs_same_gpus"] = round(2 * (top + 1) / dt / 1e9, 3)
    gpath = os.path.join(ROOT, "tests", "golden", "c5_clients.json")
    if os.path.exists(gpath):  # full CPU scans of each client's range (AVX-512 oracle)
        gold = json.load(open(gpath))
        if gold["upper"] == top:
            out["golden_ok"] = all(tuple(gold["clients"][msgs[i]]) == got.get(i)
                                   for i in range(a.clients) if msgs[i] in gold["clients"])
            out["golden_checked"] = sum(1 for m in msgs if m in gold["clients"])
    for m in gminers:
        m.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
