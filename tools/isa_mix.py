#!/usr/bin/env python3
"""Per-nonce VALU mix of the search kernel's inner loop for given layouts, read
from the built assembly (after csrc/bm_prio.py) and classified as bm_prio.py
does: fast ops (co-issue with another wave's fast op) and slow ops (issue
alone).  Issue bound per 64 nonces = 4 SIMD-cycles x max(slow, (slow+fast)/2):
every slow op takes an issue slot of its own, fast ops fill the second slot
beside it.  Writes distributed_bitcoin_minter_amd/csrc/
isa_mix.json, which bench.py reads to report the issue bound.

    python tools/isa_mix.py 18:1 12:1 56:c 60:k1 ...  (P:NBV pairs, P:c = search_kernel_padc<P>,
                                                P:kK = search_kernel_padk<P, K>; default 18:1 12:1;
                                                "all": every layout)
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, CSRC)
import bm_prio  # noqa: E402
import isa_loops  # noqa: E402

CYC_SLOT = 4.0  # SIMD-cycles per issue slot (one slow op, or two fast ops of two waves)


def inner_ops(sfile, kernel_sub):
    """The per-nonce inner loop's instructions: among the blocks of the
    DEEPEST loop (the compiler's "Loop Header: Depth=N" / "in Loop: ...
    Depth=N" annotations, as isa_loops.py reads them), the one with the most
    VALU.  (Until round 6 this took the block with the most VALU anywhere, and
    for NBV = 2 layouts that was the per-task block -- the block before
    re-compressed once per 100-nonce task -- whose VALU count is about the
    loop's: <13, 2> and <14, 2> then showed that block's 21 and 17
    v_readlane as if they ran per nonce.  Their inner loops have none.)"""
    ks = isa_loops.kernels(sfile, kernel_sub)
    name, lines = next(iter(ks.items()))
    blocks, depth, cur, pending = {}, {}, None, None
    for l in lines:
        m = re.match(r"^(\.LBB\d+_\d+):\s*(;.*)?$", l) or re.match(r"^; (%bb\.\d+):\s*(;.*)?$", l)
        ann = None
        if m:
            cur = m.group(1)
            blocks[cur], depth[cur] = [], 0
            ann, pending = m.group(2) or "", cur
        elif pending and re.match(r"^\s+;", l):
            ann = l
        else:
            pending = None if (l.strip() and not l.strip().startswith(";")) else pending
        if ann is not None and pending:
            d = re.search(r"(?:Loop Header|in Loop: Header=\S+) ?:? ?Depth=(\d+)", ann)
            if d:
                depth[pending] = int(d.group(1))
            continue
        s = l.strip()
        if cur and s and not s.startswith((";", ".")):
            blocks[cur].append((s.split()[0], s))
    deepest = max(depth.values())
    best = None
    for b, ops in blocks.items():
        if depth[b] != deepest:
            continue
        n = sum(1 for o, _ in ops if o.startswith("v_"))
        if best is None or n > best[1]:
            best = (b, n, ops)
    return best[2]


def classify(ops):
    fast = slow = 0
    for op, text in ops:
        if not op.startswith("v_") or op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
            continue
        rest = text.split(None, 1)[1] if " " in text else ""
        if bm_prio.classify(op, rest) == "F":
            fast += 1
        else:
            slow += 1
    return fast, slow


def asm_file(p, nbv, padk=0):
    """The unit's assembly (csrc/Makefile INST1 / INST2 / INSTK) that holds the
    layout: padk = K >= 3 lives in the instk_* units (K ranges)."""
    if padk >= 3:
        for r in ["3_4", "5_6", "7_8", "9_10", "11_12", "13_14", "15_15"]:
            lo, hi = map(int, r.split("_"))
            if lo <= padk <= hi:
                return os.path.join(CSRC, "build", f"instk_{r}-hip-amdgcn-amd-amdhsa-gfx950.s")
        raise ValueError((p, padk))
    ranges = {1: ["0_7", "8_15", "16_23", "24_31", "32_39", "40_47", "48_55", "56_63"],
              2: ["0_4", "5_9", "10_14", "15_18"]}[nbv]
    for r in ranges:
        lo, hi = map(int, r.split("_"))
        if lo <= p <= hi:
            return os.path.join(CSRC, "build", f"inst{nbv}_{r}-hip-amdgcn-amd-amdhsa-gfx950.s")
    raise ValueError((p, nbv))


def main():
    pairs = sys.argv[1:] or ["18:1", "12:1"]
    if pairs == ["all"]:  # every layout the library instantiates (bm_inst.hip)
        pairs = ([f"{p}:1" for p in range(64)] + [f"{p}:2" for p in range(19)] + [f"{p}:c" for p in range(55, 64)]
                 + [f"{p}:k{k}" for k in range(1, 16) for p in range(55, 64)])
    out = {"cycles_per_slot": CYC_SLOT, "model": "slots per 64 nonces = max(slow, (slow + fast) / 2)",
           "source": "tools/isa_mix.py on the built assembly (hipcc -O3 gfx950 + csrc/bm_prio.py)", "layouts": {}}
    for pr in pairs:
        # "P:c" = search_kernel_padc<P> (padding-block layout of a one-block
        # message), "P:kK" = search_kernel_padk<P, K> (the same after K prefix blocks)
        p, kind = pr.split(":")
        p = int(p)
        k = 0
        if kind == "c":
            nbv, sym = 1, f"search_kernel_padcILi{p}ELi1E"
        elif kind.startswith("k"):
            k = int(kind[1:])
            nbv, sym = 1, f"search_kernel_padkILi{p}ELi{k}ELi1E"
        else:
            nbv = int(kind)
            sym = f"search_kernelILi{p}ELi{nbv}E"
        ops = inner_ops(asm_file(p, nbv, k), sym)
        fast, slow = classify(ops)
        slots = max(slow, (slow + fast) / 2)
        # v_readlane in the loop: SGPRs the compiler spilled to VGPR lanes and
        # reads back per nonce (the generic padding-block kernel's 64 kernarg
        # K+W words)
        readlanes = sum(1 for op, _ in ops if op.startswith("v_readlane"))
        out["layouts"][pr] = {"valu_fast": fast, "valu_slow": slow, "valu": fast + slow,
                              "issue_slots": slots, "simd_cycles_per_64_nonces": slots * CYC_SLOT,
                              "readlanes": readlanes}
        print(pr, out["layouts"][pr])
    json.dump(out, open(os.path.join(CSRC, "isa_mix.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
