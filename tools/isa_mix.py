#!/usr/bin/env python3
"""Per-nonce VALU mix of the search kernel's inner loop for given layouts,
classified with the gfx950 issue costs measured in profiles/r01/ubench_*.log
(DESIGN.md §5).  Writes distributed_bitcoin_minter_amd/csrc/isa_mix.json,
which bench.py reads to report the instruction-mix ceiling.

    python tools/isa_mix.py 18:1 12:1 ...      (P:NBV pairs; default 18:1 12:1)
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_loops  # noqa: E402

FAST = re.compile(r"^v_(add_u32|sub_u32|subrev_u32|xor_b32|or_b32|and_b32|not_b32|lshrrev_b32|ashrrev_i32|"
                  r"bitop3_b32|mov_b32|add_f32|fma_f32|mul_f32)(_e32|_e64)?$")
CYC_SLOW, CYC_FAST = 4.0, 2.24


def inner_ops(sfile, kernel_sub):
    ks = isa_loops.kernels(sfile, kernel_sub)
    name, lines = next(iter(ks.items()))
    # innermost loop = the block with the most VALU among the deepest loop
    blocks, cur, best = {}, None, None
    for l in lines:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            continue
        s = l.strip()
        if cur and s and not s.startswith((";", ".")):
            blocks[cur].append((s.split()[0], s))
    for b, ops in blocks.items():
        n = sum(1 for o, _ in ops if o.startswith("v_"))
        if best is None or n > best[1]:
            best = (b, n, ops)
    return best[2]


def classify(ops):
    fast = slow = 0
    for op, text in ops:
        if not op.startswith("v_"):
            continue
        sgpr = re.search(r"\bs\[?\d", text.split(None, 1)[1] if " " in text else "")
        if FAST.match(op) and not sgpr:
            fast += 1
        else:
            slow += 1
    return fast, slow


def main():
    pairs = sys.argv[1:] or ["18:1", "12:1"]
    out = {"cycles": {"slow": CYC_SLOW, "fast": CYC_FAST},
           "source": "tools/isa_mix.py on hipcc -O3 gfx950 output", "layouts": {}}
    for pr in pairs:
        p, nbv = pr.split(":")
        subprocess.check_call(["make", "-s", "-C", CSRC, "isa", f"P={p}", f"NBV={nbv}"],
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        sfile = os.path.join(CSRC, "build", "bm_inst-hip-amdgcn-amd-amdhsa-gfx950.s")
        ops = inner_ops(sfile, f"search_kernelILi{p}ELi{nbv}E")
        fast, slow = classify(ops)
        out["layouts"][f"{p}:{nbv}"] = {"valu_fast": fast, "valu_slow": slow, "valu": fast + slow,
                                        "simd_cycles_per_64_nonces": slow * CYC_SLOW + fast * CYC_FAST}
        print(pr, out["layouts"][f"{p}:{nbv}"])
    json.dump(out, open(os.path.join(CSRC, "isa_mix.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
