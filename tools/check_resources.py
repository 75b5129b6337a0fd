#!/usr/bin/env python3
"""Summarise the search kernels' register use from the build remarks
(distributed_bitcoin_minter_amd/csrc/build/*.res) and flag anything that
would cost occupancy: VGPR spills, scratch, or sgpr_count > 80 / vgpr > 64
(8 waves/SIMD needs both; MI355X_MICROARCH.md §Residency)."""
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
bad = 0
rows = []
for f in sorted(glob.glob(os.path.join(ROOT, "distributed_bitcoin_minter_amd/csrc/build/*.res"))):
    cur = {}
    for line in open(f):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for key, pat in [("sgpr", r"TotalSGPRs: (\d+)"), ("vgpr", r"VGPRs: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)"),
                         ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                         ("sspill", r"SGPRs Spill: (\d+)")]:
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
for r in rows:
    m = re.search(r"search_kernelILi(\d+)ELi(\d)", r["name"])
    if not m:
        continue
    flag = r.get("vspill", 0) or r.get("scratch", 0) or r.get("sgpr", 0) > 80 or r.get("vgpr", 0) > 64
    bad += bool(flag)
    if flag or "-v" in sys.argv:
        print(f"P={m.group(1):>2} NBV={m.group(2)} sgpr={r.get('sgpr')} vgpr={r.get('vgpr')} "
              f"sspill={r.get('sspill')} vspill={r.get('vspill')} scratch={r.get('scratch')} occ={r.get('occ')}"
              + ("  <-- " if flag else ""))
n = sum(1 for r in rows if "search_kernel" in r["name"])
print(f"{n} search kernels, {bad} over budget")
sys.exit(1 if bad else 0)
