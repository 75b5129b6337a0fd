#!/usr/bin/env python3
"""Check every search_kernel<P,NBV> in the build's ISA (build/*-gfx950.s,
kept by the Makefile via -save-temps) for spill or memory traffic inside
its innermost loop, and print the per-nonce VALU count of each layout.
Exit 1 if any inner loop holds scratch/global/readlane/writelane ops."""
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_loops  # noqa: E402
from isa_mix import classify  # noqa: E402

BAD = re.compile(r"^(scratch_|buffer_|global_|flat_|s_buffer)")      # memory traffic: never in a loop
LANE = re.compile(r"^(v_readlane|v_writelane)")                       # SGPR spill via VGPR lanes
args = [a for a in sys.argv[1:] if not a.startswith("-")]
build = args[0] if args else os.path.join(ROOT, "distributed_bitcoin_minter_amd/csrc/build")
bad = 0
rows = []
for sfile in sorted(glob.glob(os.path.join(build, "*gfx950.s"))):
    for name, lines in isa_loops.kernels(sfile, "search_kernel").items():
        m = re.search(r"search_kernelILi(\d+)ELi(\d)", name)
        if not m:
            continue
        blocks, cur = {}, None
        for l in lines:
            mm = re.match(r"^(\.LBB\d+_\d+):", l)
            if mm:
                cur = mm.group(1)
                blocks[cur] = []
                continue
            s = l.strip()
            if cur and s and not s.startswith((";", ".")):
                blocks[cur].append((s.split()[0], s))
        body = max(blocks.values(), key=lambda ops: sum(1 for o, _ in ops if o.startswith("v_")))
        nbad = sum(1 for o, _ in body if BAD.match(o))
        nlane = sum(1 for o, _ in body if LANE.match(o))
        fast, slow = classify(body)
        rows.append((int(m.group(2)), int(m.group(1)), fast + slow, slow, nbad, nlane))
        bad += nbad > 0
for nbv, p, valu, slow, nbad, nlane in sorted(rows):
    if nbad or "-v" in sys.argv:
        print(f"NBV={nbv} P={p:2d} inner VALU={valu} slow={slow} mem={nbad} lane-spill={nlane}")
print(f"{len(rows)} kernels checked, {bad} with scratch/memory ops in the inner loop")
sys.exit(1 if bad else 0)
