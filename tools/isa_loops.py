#!/usr/bin/env python3
"""Summarise the loops of the kernels in a gfx950 .s file (hipcc -save-temps).

For every loop (from the compiler's "Loop Header: Depth=N" annotations) it
prints the instruction mix of each of its basic blocks, so the per-nonce
VALU count of the search kernel's inner loop can be read off directly.
Usage: isa_loops.py file.s [kernel-substring]
"""
import re
import sys
from collections import Counter, OrderedDict


def cls(op):
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "BR"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "WAIT"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "SMEM"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    return "OTHER"


def kernels(path, want):
    out = OrderedDict()
    cur = None
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1) if (want is None or want in m.group(1)) else None
            if cur:
                out[cur] = []
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        out[cur].append(line.rstrip("\n"))
    return out


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    for name, lines in kernels(path, want).items():
        blocks = OrderedDict()
        meta = {}
        cur = "entry"
        blocks[cur] = []
        meta[cur] = (None, 0)
        pending = None  # block whose annotation may follow on comment lines
        for l in lines:
            m = re.match(r"^(\.LBB\d+_\d+):\s*(;.*)?$", l) or re.match(r"^; (%bb\.\d+):\s*(;.*)?$", l)
            ann = None
            if m:
                cur = m.group(1)
                blocks[cur] = []
                meta[cur] = (None, 0)
                ann = m.group(2) or ""
                pending = cur
            elif pending and re.match(r"^\s+;", l):
                ann = l
            else:
                pending = None if (l.strip() and not l.strip().startswith(";")) else pending
            if ann is not None and pending:
                h = re.search(r"Loop Header: Depth=(\d+)", ann)
                i = re.search(r"in Loop: Header=(\S+) Depth=(\d+)", ann)
                if h:
                    meta[pending] = (pending, int(h.group(1)))
                elif i:
                    meta[pending] = (".L" + i.group(1), int(i.group(2)))
                continue
            s = l.strip()
            if not s or s.startswith((";", ".")):
                continue
            blocks[cur].append(s.split()[0])
        tot = Counter(cls(o) for b in blocks.values() for o in b)
        print(f"== {name}\n   whole kernel: {dict(tot)}")
        maxd = max(d for _, d in meta.values())
        for b, ops in blocks.items():
            hdr, d = meta[b]
            if d == 0:
                continue
            c = Counter(cls(o) for o in ops)
            tag = "  *innermost*" if d == maxd else ""
            print(f"   {b:10s} depth={d} loop={hdr}: {len(ops):5d} ops {dict(c)}{tag}")
            if d == maxd and c.get("VALU", 0) > 100:
                v = Counter(o for o in ops if o.startswith("v_"))
                print("      VALU mix:", ", ".join(f"{k}={n}" for k, n in v.most_common(16)))


if __name__ == "__main__":
    main()
