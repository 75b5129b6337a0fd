#!/usr/bin/env python3
"""Build step: wave-priority toggles around slow / fast VALU runs in the
search kernels' gfx950 assembly.

    bm_prio.py in.s out.s [--slow-prio 2] [--fast-prio 0] [--kernels search_kernel]
                          [--min-fast-run 1] [--fold-sgpr 1]

Why (tools/gen_ubench_pairs.py, profiles/r01/ubench_pairs4.log):
on gfx950 two waves of a SIMD can issue VALU in the same cycle when the ops
are of the "fast" class (v_add_u32, v_xor/or/and, v_lshrrev, v_bitop3, v_mov
... with no SGPR operand; PMC SQ_ACTIVE_INST_VALU2 counts them).  Slow ops
(v_alignbit, v_add3, shifts left, any SGPR operand) issue alone.  With the
default age-ordered arbitration a mixed stream like SHA-256's pairs poorly:
a slow op at the head of an old wave holds the issue while fast ops wait.
Raising the wave's priority for its slow runs (s_setprio 2) and dropping it
for its fast runs (s_setprio 0) lets the slow op go first and the other
waves' fast ops fill the second slot: a SHA-round-shaped microbenchmark goes
from 1.84 to 2.47 wave-instructions per CU-cycle.

Before that, fold_sgpr_constants turns slow ops into fast ones where an SGPR
operand provably holds a constant (its only definition in the kernel, or the
last one in the block, is s_mov_b32 sN, imm): the SGPR becomes the literal,
and v_add3_u32 x, y, K (slow) becomes two v_add_u32 (fast).  Fast ops cost
little once they pair, so trading one slow op for two fast ones shortens the
loop (C2 +1.8%, C3 +2.4%, profiles/r01/ab_fold_sgpr.log).

The pass inserts SOPP s_setprio instructions and makes those two
value-preserving rewrites; it changes no dependency, so results are
unaffected (tests/test_prio_pass.py interprets a sample both ways; the GPU
parity suite runs on the built library).  A toggle goes before the first
VALU of every run whose class differs from the current priority; the state is
reset at every label (any block may be entered from elsewhere).

The pass runs after LLVM's hazard recognizer and waitcnt insertion, so its
output goes through bm_asm_guard.check before it is written: no inserted or
moved instruction may touch a register an outstanding load targets, a
rewrite touches only the registers of the instruction it replaces, and no
pair of the compiler's instructions that needs wait states may end up closer
than the compiler placed it.  A refused rewrite fails the build (exit 3).
"""
import argparse
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bm_asm_guard import GuardError, Made, check as guard_check  # noqa: E402

FAST_OPS = {
    "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_xor_b32", "v_or_b32", "v_and_b32", "v_not_b32",
    "v_lshrrev_b32", "v_ashrrev_i32", "v_bitop3_b32", "v_mov_b32", "v_add_f32", "v_fma_f32",
}
SGPR_RE = re.compile(r"^-?(s\d+|s\[\d+:\d+\]|vcc(_lo|_hi)?|exec(_lo|_hi)?|m0|ttmp\d+|ttmp\[\d+:\d+\]|flat_scratch\S*)$")
INSN_RE = re.compile(r"^\s+(v_[a-z0-9_]+)\s*(.*)$")


def classify(mnemonic, operands):
    """'F' (can dual-issue), 'S' (issues alone)."""
    base = re.sub(r"_e(32|64)$|_sdwa$|_dpp$", "", mnemonic)
    if base not in FAST_OPS or mnemonic.endswith(("_sdwa", "_dpp")):
        return "S"
    ops = [o.strip() for o in operands.split(" bitop3:")[0].split(",")]
    for o in ops:
        tok = o.split()[0] if o.split() else ""
        if SGPR_RE.match(tok):
            return "S"
    return "F"

SREG_RE = re.compile(r"^s(\d+)$")
SRANGE_RE = re.compile(r"^s\[(\d+):(\d+)\]$")
VREG_RE = re.compile(r"^v\d+$")
IMM_RE = re.compile(r"^(0x[0-9a-fA-F]+|-?\d+)$")


def _operands(rest):
    return [o.strip() for o in rest.split(" bitop3:")[0].split(",") if o.strip()]


# VOP3B forms: vdst, sdst, src...  (the second operand is an SGPR the op writes)
VOP3B_RE = re.compile(r"^v_(add|sub|subrev|addc|subb|subbrev)_co_|^v_(mad|mul)_[ui]64_|^v_div_scale")


def _sreg_nums(tok):
    if SREG_RE.match(tok):
        return [int(SREG_RE.match(tok).group(1))]
    r = SRANGE_RE.match(tok)
    if r:
        return list(range(int(r.group(1)), int(r.group(2)) + 1))
    return []


def _sdefs(line):
    """SGPR numbers an instruction writes: its first operand, and the carry /
    scale SGPR destination of VOP3B forms (v_add_co_u32_e64 v, s[..], ...)."""
    m = re.match(r"^\s+([sv]_[a-z0-9_]+)\s*(.*)$", line)
    if not m or m.group(1).startswith(("s_cmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_setprio",
                                        "s_endpgm", "s_barrier", "s_sleep")):
        return []
    ops = _operands(m.group(2))
    if not ops:
        return []
    out = _sreg_nums(ops[0].split()[0])
    if VOP3B_RE.match(m.group(1)) and len(ops) > 1:
        out += _sreg_nums(ops[1].split()[0])
    return out


def fold_sgpr_constants(lines, kernels):
    """Replace SGPR operands holding a known constant by the literal, so the
    VALU op stays in the fast class, and split v_add3_u32 with such an
    operand into two v_add_u32 (two fast ops for one slow one).  A constant is
    known when the SGPR's only definition in the kernel is s_mov_b32 sN, imm,
    or, inside a block, since the last s_mov_b32 sN, imm."""
    out, i, n_fold, n_split = [], 0, 0, 0
    while i < len(lines):
        m_fn = re.match(r"^(_Z\S+):", lines[i])
        if not (m_fn and any(k in m_fn.group(1) for k in kernels)):
            out.append(lines[i])
            i += 1
            continue
        j = i
        while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
            j += 1
        body = lines[i:j]
        defs, single = {}, {}
        for ln in body:
            for r in _sdefs(ln):
                defs[r] = defs.get(r, 0) + 1
        for ln in body:
            m = re.match(r"^\s+s_mov_b32 s(\d+), (\S+)\s*$", ln)
            if m and defs.get(int(m.group(1))) == 1 and IMM_RE.match(m.group(2)):
                single[int(m.group(1))] = m.group(2)
        local = {}
        for ln in body:
            if re.match(r"^[.%$\w]+:", ln) or ln.startswith("; %bb"):
                local = {}
            m = re.match(r"^\s+(v_add3_u32|v_add_u32_e32|v_xor_b32_e32)\s+(.*)$", ln)
            if m:
                ops = _operands(m.group(2))
                known = lambda o: (local.get(int(SREG_RE.match(o).group(1))) or single.get(int(SREG_RE.match(o).group(1)))) \
                    if SREG_RE.match(o) else None
                if m.group(1) == "v_add3_u32" and len(ops) == 4:
                    ks = [k for k in range(1, 4) if known(ops[k])]
                    vs = [k for k in range(1, 4) if VREG_RE.match(ops[k])]
                    if len(ks) == 1 and len(vs) == 2:
                        lit = known(ops[ks[0]])
                        x, y = ops[vs[0]], ops[vs[1]]
                        out.append(Made(f"\tv_add_u32_e32 {ops[0]}, {x}, {y}\n", "rewrite", ln))
                        out.append(Made(f"\tv_add_u32_e32 {ops[0]}, {lit}, {ops[0]}\n", "rewrite", ln))
                        n_split += 1
                        continue
                elif len(ops) == 3 and known(ops[1]) and VREG_RE.match(ops[2]):
                    out.append(Made(f"\t{m.group(1)} {ops[0]}, {known(ops[1])}, {ops[2]}\n", "rewrite", ln))
                    n_fold += 1
                    continue
            for r in _sdefs(ln):
                local.pop(r, None)
            m = re.match(r"^\s+s_mov_b32 s(\d+), (\S+)\s*$", ln)
            if m and IMM_RE.match(m.group(2)):
                local[int(m.group(1))] = m.group(2)
            out.append(ln)
        i = j
    return out, n_fold, n_split


def drop_dead_smov(lines, kernels, replace=None):
    """Delete s_mov_b32 sN, imm that the literal fold left dead: inside one
    block, sN is written again by another s_mov_b32 before anything else
    names sN.  Any other appearance of sN (as a source, a destination of
    another op, inside a register range or in inline asm) counts as a use, so
    the rule only ever removes a write nothing can read."""
    out, n = list(lines), 0
    in_kernel = False
    pending = {}  # sN -> index in out of its last s_mov_b32 with no use since
    dead = set()
    mov_re = re.compile(r"^\s+s_mov_b32 s(\d+), (\S+)\s*$")
    for i, ln in enumerate(lines):
        m_fn = re.match(r"^(_Z\S+):", ln)
        if m_fn:
            in_kernel = any(k in m_fn.group(1) for k in kernels)
            pending = {}
            continue
        if ln.startswith(".Lfunc_end"):
            in_kernel = False
        if not in_kernel:
            continue
        if re.match(r"^[.%$\w]+:", ln) or ln.startswith("; %bb") or re.match(r"^\s+s_(cbranch|branch|setpc|swappc)", ln):
            pending = {}
            continue
        code = ln.split(";")[0]
        m = mov_re.match(code)
        if m and IMM_RE.match(m.group(2)):
            r = int(m.group(1))
            if r in pending:
                dead.add(pending[r])
            pending[r] = i
            continue
        for r in [int(x[1:]) for x in _regs(code) if x.startswith("s")]:
            pending.pop(r, None)
    for i in sorted(dead, reverse=True):
        if replace is None:
            del out[i]
        else:
            out[i] = Made(replace, "rewrite", lines[i])
        n += 1
    return out, n


def space_dependent_valu(lines, kernels, spacer="\ts_nop 0\n"):
    """Insert `spacer` (s_nop 0) between two adjacent VALU ops of the search
    kernels' big blocks when the second reads what the first wrote (an A/B
    probe of whether the dead SALU writes the fold leaves behind help by
    spacing a wave's dependent VALU)."""
    out, in_kernel, prev, n = [], False, None, 0
    for ln in lines:
        m_fn = re.match(r"^(_Z\S+):", ln)
        if m_fn:
            in_kernel = any(k in m_fn.group(1) for k in kernels)
            prev = None
        elif ln.startswith(".Lfunc_end"):
            in_kernel = False
        du = _defs_uses(ln) if in_kernel else None
        if du is None:
            if in_kernel and ln.strip() and not ln.strip().startswith(";"):
                prev = None
            out.append(ln)
            continue
        mn, defs, uses = du
        if mn.startswith("v_"):
            if prev is not None and prev & uses:
                out.append(Made(spacer, "insert"))
                n += 1
            prev = defs
        out.append(ln)
    return out, n


def split_add3(lines, kernels, every):
    """Split every `every`-th all-VGPR v_add3_u32 d, a, b, c of the search
    kernels into v_add_u32 d, x, y; v_add_u32 d, z, d.  The loop is slow-slot
    bound (S > (S+F)/2): each split moves one op from the slow
    class to two in the fast class, and the issue bound max(S, (S+F)/2) falls
    until the two terms meet (about 1 in 8 of the C2 loop's add3).  The pair
    whose first add overwrites d must read every source equal to d."""
    out, n, seen, in_kernel = [], 0, 0, False
    for ln in lines:
        m_fn = re.match(r"^(_Z\S+):", ln)
        if m_fn:
            in_kernel = any(k in m_fn.group(1) for k in kernels)
        elif ln.startswith(".Lfunc_end"):
            in_kernel = False
        m = re.match(r"^\s+v_add3_u32\s+(.*)$", ln) if in_kernel else None
        if m:
            ops = _operands(m.group(1))
            if len(ops) == 4 and all(VREG_RE.match(o) for o in ops):
                d, srcs = ops[0], ops[1:]
                hits = [s for s in srcs if s == d]
                rest = [s for s in srcs if s != d]
                if len(hits) < 3:
                    seen += 1
                    if seen % every == 0:
                        first = (hits + rest)[:2]   # every read of d happens in the first add
                        last = (hits + rest)[2]
                        if len(hits) <= 2 and last != d:
                            out.append(Made(f"\tv_add_u32_e32 {d}, {first[0]}, {first[1]}\n", "rewrite", ln))
                            out.append(Made(f"\tv_add_u32_e32 {d}, {last}, {d}\n", "rewrite", ln))
                            n += 1
                            continue
        out.append(ln)
    return out, n


# Ops cluster_runs may move: single-destination VALU (no carry, no VCC/EXEC
# side effects) and SALU arithmetic (which writes SCC).  Anything else fences.
CLUSTER_VALU = {"v_alignbit_b32", "v_bitop3_b32", "v_add_u32_e32", "v_add3_u32", "v_lshrrev_b32_e32",
                "v_xor_b32_e32", "v_xad_u32", "v_or_b32_e32", "v_and_b32_e32", "v_mov_b32_e32", "v_sub_u32_e32",
                "v_lshlrev_b32_e32", "v_perm_b32", "v_bfi_b32", "v_or3_b32", "v_xor3_b32", "v_lshl_or_b32",
                "v_lshl_add_u32", "v_add_lshl_u32", "v_and_or_b32", "v_not_b32_e32"}
CLUSTER_SALU_SCC = {"s_lshr_b32", "s_lshl_b32", "s_or_b32", "s_xor_b32", "s_and_b32", "s_add_i32", "s_add_u32",
                    "s_sub_i32", "s_sub_u32"}
CLUSTER_SALU = {"s_mov_b32", "s_movk_i32"} | CLUSTER_SALU_SCC
REG_TOK = re.compile(r"\b([vs])(\d+)\b|\b([vs])\[(\d+):(\d+)\]")


def _regs(text):
    out = set()
    for m in REG_TOK.finditer(text):
        if m.group(1):
            out.add(f"{m.group(1)}{m.group(2)}")
        else:
            out.update(f"{m.group(3)}{k}" for k in range(int(m.group(4)), int(m.group(5)) + 1))
    return out


def _defs_uses(line):
    """(mnemonic, defs, uses) of a movable instruction, or None (a fence)."""
    m = re.match(r"^\s+([sv]_[a-z0-9_]+)\s+(.*)$", line)
    if not m or m.group(1) not in CLUSTER_VALU | CLUSTER_SALU:
        return None
    ops = _operands(m.group(2))
    if len(ops) < 2:
        return None
    defs = _regs(ops[0])
    uses = set().union(*(_regs(o) for o in ops[1:]))
    if m.group(1) in CLUSTER_SALU_SCC:
        defs.add("scc")
    return m.group(1), defs, uses


def _schedule(seg, max_run):
    """Reorder one fence-free segment: a list schedule over its register
    dependences (RAW, WAR, WAW, SCC) that keeps issuing VALU of the current
    class (slow / fast) while any is ready, up to max_run in a row, then
    switches; SALU goes as soon as it is ready; ties go to program order."""
    n = len(seg)
    succ = [[] for _ in range(n)]
    indeg = [0] * n
    last_def, readers = {}, {}

    def edge(a, b):
        if a != b:
            succ[a].append(b)
            indeg[b] += 1

    info = []
    for i, ln in enumerate(seg):
        mn, defs, uses = _defs_uses(ln)
        rest = ln.split(None, 1)[1] if len(ln.split(None, 1)) > 1 else ""
        cls = "N" if mn.startswith("s_") else classify(mn, rest)
        info.append(cls)
        for r in uses:
            if r in last_def:
                edge(last_def[r], i)
        for r in defs:
            if r in last_def:
                edge(last_def[r], i)
            for u in readers.get(r, ()):
                edge(u, i)
        for r in uses:
            readers.setdefault(r, []).append(i)
        for r in defs:
            last_def[r] = i
            readers[r] = []
    import heapq
    ready = [i for i in range(n) if indeg[i] == 0]
    heapq.heapify(ready)
    order, cur, run = [], None, 0
    while ready:
        pool = sorted(ready)
        pick = next((i for i in pool if info[i] == "N"), None)
        if pick is None:
            same = [i for i in pool if info[i] == cur] if (cur and (max_run <= 0 or run < max_run)) else []
            pick = same[0] if same else pool[0]
            if info[pick] != cur:
                cur, run = info[pick], 0
            run += 1
        ready.remove(pick)
        heapq.heapify(ready)
        order.append(pick)
        for j in succ[pick]:
            indeg[j] -= 1
            if indeg[j] == 0:
                heapq.heappush(ready, j)
    assert len(order) == n, "dependence cycle"
    return [seg[i] if k == i else Made(seg[i], "move", seg[i].orig if isinstance(seg[i], Made) else seg[i])
            for k, i in enumerate(order)]


def cluster_runs(lines, kernels, max_run=0, min_valu=64):
    """Reorder the straight-line stretches of the search kernels' big blocks
    (>= min_valu VALU between fences) so slow and fast VALU come in longer
    runs: fewer s_setprio toggles, longer phases for the arbiter to pair."""
    out, in_kernel, seg = [], False, []

    def flush():
        nv = sum(1 for ln in seg if ln.lstrip().startswith("v_"))
        out.extend(_schedule(seg, max_run) if nv >= min_valu else seg)
        seg.clear()

    for ln in lines:
        m_fn = re.match(r"^(_Z\S+):", ln)
        if m_fn:
            in_kernel = any(k in m_fn.group(1) for k in kernels)
        elif ln.startswith(".Lfunc_end"):
            in_kernel = False
        if in_kernel and _defs_uses(ln) is not None:
            seg.append(ln)
            continue
        flush()
        out.append(ln)
    flush()
    return out


def run(lines, kernels, slow, fast, min_fast_run=1):
    """Insert the toggles.  A fast run shorter than min_fast_run VALU (counted
    up to the next label) keeps the slow priority."""
    cls = [None] * len(lines)  # VALU class per line (None: not a VALU / not in a search kernel)
    in_kernel = False
    for i, line in enumerate(lines):
        m_fn = re.match(r"^(_Z\S+):", line)
        if m_fn:
            in_kernel = any(k in m_fn.group(1) for k in kernels)
        elif line.startswith(".Lfunc_end"):
            in_kernel = False
        if in_kernel:
            if re.match(r"^[.%$\w]+:", line) or line.startswith("; %bb"):
                cls[i] = "L"  # label: block boundary
                continue
            m = INSN_RE.match(line)
            if m and not m.group(1).startswith(("v_readlane", "v_readfirstlane", "v_writelane", "v_nop")):
                cls[i] = classify(m.group(1), m.group(2))
    out, cur = [], None
    n_toggle = n_valu = 0
    for i, line in enumerate(lines):
        c = cls[i]
        if c == "L":
            cur = None
        elif c in ("S", "F"):
            n_valu += 1
            want = c
            if c == "F" and min_fast_run > 1:
                run_len, j = 0, i
                while j < len(lines) and cls[j] != "L" and cls[j] != "S" and run_len < min_fast_run:
                    run_len += cls[j] == "F"
                    j += 1
                if run_len < min_fast_run and cur == "S":
                    want = "S"
            if want != cur:
                out.append(Made(f"\ts_setprio {slow if want == 'S' else fast}\n", "insert"))
                n_toggle += 1
                cur = want
        out.append(line)
    return out, n_toggle, n_valu


def lead_toggles(lines, prio):
    """Move every `s_setprio <prio>` one VALU earlier: above the last op of
    the run it ends, when that run has at least two VALU (an A/B probe of the
    toggle's timing relative to the ops it reorders)."""
    out = list(lines)
    n = 0
    is_valu = lambda ln: ln.lstrip().startswith("v_")
    for i in range(2, len(out)):
        if out[i].strip() == f"s_setprio {prio}" and is_valu(out[i - 1]) and is_valu(out[i - 2]):
            out[i - 1], out[i] = out[i], out[i - 1]
            n += 1
    return out, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--slow-prio", type=int, default=2)
    ap.add_argument("--fast-prio", type=int, default=0)
    ap.add_argument("--kernels", default="search_kernel")
    ap.add_argument("--min-fast-run", type=int, default=1)
    ap.add_argument("--fold-sgpr", type=int, default=1, help="1: literal-fold known SGPR constants, split add3")
    ap.add_argument("--drop-dead-smov", type=int, default=0,
                    help="1: delete the s_mov_b32 sN, imm the fold left with no reader before the next one; "
                         "2: replace each by s_nop 0 (measured: 1 is C2 -0.7%%, profiles/r02/ab_dead_smov.log)")
    ap.add_argument("--lead-slow", type=int, default=0, help="1: each s_setprio <slow> one VALU earlier")
    ap.add_argument("--lead-fast", type=int, default=0, help="1: each s_setprio <fast> one VALU earlier")
    ap.add_argument("--space-dependent", type=int, default=0,
                    help="1: s_nop 0 between adjacent VALU where the second reads the first's result; "
                         "2: s_mov_b32 s0, s0 there instead (round 2's faulting variant, DESIGN.md §8)")
    ap.add_argument("--split-add3-every", type=int, default=0,
                    help="K > 0: split every K-th all-VGPR v_add3_u32 into two v_add_u32")
    ap.add_argument("--cluster", type=int, default=-1,
                    help=">= 0: reorder big blocks into longer slow / fast runs (0: unbounded runs, "
                         "K: at most K in a row); -1: off")
    a = ap.parse_args()
    orig = open(a.src).readlines()
    lines = list(orig)
    if a.fold_sgpr:
        lines, n_fold, n_split = fold_sgpr_constants(lines, a.kernels.split(","))
        print(f"bm_prio: {a.src}: {n_fold} SGPR constants folded, {n_split} v_add3 split", file=sys.stderr)
    if a.drop_dead_smov:
        lines, n_dead = drop_dead_smov(lines, a.kernels.split(","), "\ts_nop 0\n" if a.drop_dead_smov == 2 else None)
        print(f"bm_prio: {a.src}: {n_dead} dead s_mov_b32 {'removed' if a.drop_dead_smov == 1 else 'made s_nop 0'}",
              file=sys.stderr)
    if a.space_dependent:
        spacer = "\ts_mov_b32 s0, s0\n" if a.space_dependent == 2 else "\ts_nop 0\n"
        lines, n_sp = space_dependent_valu(lines, a.kernels.split(","), spacer)
        print(f"bm_prio: {a.src}: {n_sp} `{spacer.strip()}` between dependent VALU", file=sys.stderr)
    if a.split_add3_every:
        lines, n_split3 = split_add3(lines, a.kernels.split(","), a.split_add3_every)
        print(f"bm_prio: {a.src}: {n_split3} all-VGPR v_add3 split", file=sys.stderr)
    if a.cluster >= 0:
        lines = cluster_runs(lines, a.kernels.split(","), max_run=a.cluster)
    out, n_toggle, n_valu = run(lines, a.kernels.split(","), a.slow_prio, a.fast_prio, a.min_fast_run)
    for prio, on in ((a.slow_prio, a.lead_slow), (a.fast_prio, a.lead_fast)):
        if on:
            out, n_lead = lead_toggles(out, prio)
            print(f"bm_prio: {a.src}: {n_lead} s_setprio {prio} moved one VALU earlier", file=sys.stderr)
    # every rewrite checked against the compiler's own assembly (bm_asm_guard.py)
    try:
        g = guard_check(orig, out, a.kernels.split(","))
    except GuardError as e:
        print(f"bm_prio: {a.src}: REFUSED by the assembly guard: {e}", file=sys.stderr)
        sys.exit(3)
    open(a.dst, "w").writelines(out)
    print(f"bm_prio: {a.src}: {n_toggle} s_setprio over {n_valu} VALU; guard: {g['kernels']} kernels, "
          f"{g['inserted']} inserted, {g['rewritten']} rewritten, {g['moved']} moved, {g['deleted']} deleted, "
          f"{g['pairs']} padded pairs closer (all interlocked)", file=sys.stderr)


if __name__ == "__main__":
    main()
