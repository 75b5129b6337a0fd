#!/usr/bin/env python3
"""Check every search kernel in the build's ISA (build/*-gfx950.s, kept by
the Makefile): search_kernel<P, NBV>, search_kernel_padc<P> and
search_kernel_padk<P, K>, for spill or memory traffic inside its innermost
loop, and print the per-nonce VALU count of each layout (-v).  Exit 1 if any
inner loop holds scratch/global/buffer ops; SGPR spills read back through
v_readlane (the generic padding-block kernel's) are counted and reported."""
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_loops  # noqa: E402
from isa_mix import classify, inner_ops  # noqa: E402

BAD = re.compile(r"^(scratch_|buffer_|global_|flat_|s_buffer)")      # memory traffic: never in a loop
LANE = re.compile(r"^(v_readlane|v_writelane)")                       # SGPR spill via VGPR lanes
args = [a for a in sys.argv[1:] if not a.startswith("-")]
build = args[0] if args else os.path.join(ROOT, "distributed_bitcoin_minter_amd/csrc/build")
bad = 0
rows = []
for sfile in sorted(glob.glob(os.path.join(build, "*gfx950.s"))):
    for name in isa_loops.kernels(sfile, "search_kernel"):
        m = re.search(r"search_kernel(_padc|_padk)?ILi(\d+)ELi(\d+)E(?:Li(\d+)E)?", name)
        if not m:
            continue
        kind, p, a = m.group(1), int(m.group(2)), int(m.group(3))
        tag = "c" if kind == "_padc" else f"k{a}" if kind == "_padk" else str(a)
        # the innermost loop (the deepest loop's biggest block: isa_mix.inner_ops)
        body = inner_ops(sfile, name)
        nbad = sum(1 for o, _ in body if BAD.match(o))
        nlane = sum(1 for o, _ in body if LANE.match(o))
        fast, slow = classify(body)
        rows.append((tag, p, fast + slow, slow, nbad, nlane))
        bad += nbad > 0
for tag, p, valu, slow, nbad, nlane in sorted(rows, key=lambda r: (len(r[0]), r[0], r[1])):
    if nbad or "-v" in sys.argv:
        print(f"{p:2d}:{tag:3s} inner VALU={valu} slow={slow} mem={nbad} lane-spill={nlane}")
print(f"{len(rows)} kernels checked, {bad} with scratch/memory ops in the inner loop, "
      f"{sum(1 for r in rows if r[5])} with v_readlane/v_writelane in it")
sys.exit(1 if bad else 0)
