"""Build-time guard for bm_prio.py's rewrites of the search kernels' gfx950
assembly.

bm_prio.py edits the compiler's output AFTER LLVM's hazard recognizer and
waitcnt insertion have run, so nothing downstream re-checks what it does.
Every rewrite it makes is checked here against the compiler's own assembly
of the same kernels, and the build fails on any violation:

1. Memory counters.  A line the pass inserts (or moves) may not read or
   write a register that an outstanding load still targets.  The model runs
   a dataflow over each kernel's control-flow graph: SMEM loads (s_load*,
   out of order: done only at lgkmcnt(0)), LDS ops (in order within the
   lgkm counter), and VMEM/scratch loads and returning atomics (in order
   within vmcnt).  An entry is done once `s_waitcnt <cnt>(N)` has seen at
   least N younger in-order ops of its counter.  At a join the pending sets
   merge by union, each with its smallest count of younger ops.
2. Rewrites.  A line that replaces an instruction (the literal fold, the
   v_add3 split, a dead write made s_nop) reads only registers the replaced
   instruction read or wrote and writes only registers it wrote, so it
   needs no wait the compiler did not already place.
3. Wait states.  For every pair of the compiler's instructions within 6
   issue slots where the second accesses a register the first wrote (or the
   second writes a register the first read), the distance in the rewritten
   code may not shrink unless the hardware interlocks that pair: a plain
   VALU reading a VGPR, or an SALU consumer.  Inserting instructions only
   lengthens distances, so the shipped toggle insertion and fold always
   pass; deleting or reordering instructions (--drop-dead-smov 1,
   --cluster) can shorten a pair the compiler padded (VALU writes VGPR ->
   DPP / v_readlane / v_readfirstlane, VALU writes SGPR -> VMEM / lane
   select, store data -> overwrite) and is refused there.
4. New pairs.  An inserted instruction that reads or writes registers may
   not form, with any instruction within 6 issue slots of it, a pair the
   hardware does not interlock (conservatively: an SALU write feeding a
   VMEM address counts as one).

bm_prio marks what it produced with `Made` lines: unchanged lines pass
through as the same Python objects, so the guard pairs each line of the
output with the compiler's line it came from.
"""
import re

WINDOW = 6  # issue slots: the longest gfx950 non-MFMA wait-state rule is 5


class Made(str):
    """An output line bm_prio produced.  kind: 'insert' (a new instruction:
    s_setprio, a spacer), 'rewrite' (replaces the compiler's line `orig`),
    'move' (the compiler's line `orig`, reordered)."""

    def __new__(cls, text, kind, orig=None):
        s = str.__new__(cls, text)
        s.kind = kind
        s.orig = orig
        return s


class GuardError(RuntimeError):
    pass


LABEL_RE = re.compile(r"^([.%$\w]+):")
INSN_RE = re.compile(r"^\s+([a-z][a-z0-9_]*)\b\s*(.*)$")
REG_RE = re.compile(r"\b([vs])(\d+)\b|\b([vs])\[(\d+):(\d+)\]|\b(vcc|exec|scc|m0)(?:_lo|_hi)?\b")
NO_REG_OPS = ("s_waitcnt", "s_nop", "s_setprio", "s_barrier", "s_endpgm", "s_sleep", "s_sethalt", "s_trap",
              "s_dcache", "s_icache", "s_branch", "s_cbranch", "s_setpc", "s_sendmsg", "s_ttrace")
# VALU ops that write their first two operands (VOP3B: vdst, sdst)
VOP3B_RE = re.compile(r"^v_(add|sub|subrev|addc|subb|subbrev)_co_\w*_e64$|^v_(mad|mul)_[ui]64_|^v_div_scale")
# VALU consumers the hardware does NOT interlock against a recent VALU write
UNLOCKED_VALU_RE = re.compile(r"_dpp$|_sdwa$|^v_readlane|^v_readfirstlane|^v_writelane|^v_permlane|^v_div_fmas|"
                              r"^v_mfma|^v_smfmac|^v_accvgpr|^v_movrel")


def regs_of(text):
    out = set()
    for m in REG_RE.finditer(text):
        if m.group(1):
            out.add(f"{m.group(1)}{m.group(2)}")
        elif m.group(3):
            out.update(f"{m.group(3)}{k}" for k in range(int(m.group(4)), int(m.group(5)) + 1))
        else:
            out.add(m.group(6))
    return out


def operands(rest):
    """Operand texts before modifiers (bitop3:, offset:, sc0 ...) and comments."""
    rest = rest.split(";")[0]
    return [o.strip() for o in rest.split(",") if o.strip()]


class Insn:
    """One instruction: mnemonic, registers read / written, memory class."""

    __slots__ = ("mn", "reads", "writes", "mem", "ooo", "slots", "line")

    def __init__(self, line):
        m = INSN_RE.match(line.split(";")[0])
        self.line = line
        self.mn = mn = m.group(1)
        ops = operands(m.group(2))
        first = regs_of(ops[0].split()[0]) if ops else set()
        rest = set().union(*(regs_of(o) for o in ops[1:])) if len(ops) > 1 else set()
        self.mem, self.ooo, self.slots = None, False, 1
        reads, writes = set(), set()
        if mn.startswith(NO_REG_OPS):
            if mn.startswith("s_cbranch"):
                reads = {"scc"} if "scc" in mn else {"vcc"} if "vcc" in mn else {"exec"} if "exec" in mn else set()
            elif mn == "s_nop":
                self.slots = int(ops[0], 0) + 1 if ops else 1
        elif mn.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_scratch_load")):
            writes, reads, self.mem, self.ooo = first, rest, "lgkm", True
        elif mn.startswith("s_"):
            if mn.startswith(("s_cmp", "s_bitcmp")):
                reads, writes = first | rest, {"scc"}
            else:
                writes, reads = set(first), set(rest)
                if not mn.startswith(("s_mov", "s_movk", "s_cmov", "s_cselect", "s_getpc", "s_setreg", "s_getreg")):
                    writes.add("scc")
                if mn.startswith(("s_cselect", "s_cmov", "s_addc", "s_subb", "s_cbranch_scc")):
                    reads.add("scc")
                if "saveexec" in mn:
                    writes.add("exec")
                    reads.add("exec")
        elif mn.startswith("ds_"):
            self.mem = "lgkm"
            if re.match(r"ds_(read|load|swizzle|permute|bpermute)|ds_\w*_rtn_", mn):
                writes, reads = first, rest
            else:
                reads = first | rest
        elif mn.startswith(("global_", "buffer_", "scratch_", "flat_")):
            self.mem = "vm"
            returning = "_atomic" in mn and re.search(r"\b(sc0|glc)\b", m.group(2))
            if "_load" in mn or returning:
                writes, reads = first, rest
            else:
                reads = first | rest
        elif mn.startswith("v_"):
            reads = set(rest) | {"exec"}
            if mn.startswith("v_cmpx"):
                writes = {"exec"} | (first if mn.endswith("_e64") else set())
                reads |= first if not mn.endswith("_e64") else set()
            elif mn.startswith("v_cmp") and mn.endswith("_e32"):
                writes, reads = {"vcc"}, reads | first
            elif VOP3B_RE.match(mn) and len(ops) > 1:
                writes = first | regs_of(ops[1].split()[0])
                reads = set().union(*(regs_of(o) for o in ops[2:])) | {"exec"}
            else:
                writes = set(first)
                if "_co_" in mn and mn.endswith("_e32"):
                    writes.add("vcc")
                if mn.startswith(("v_addc", "v_subb", "v_cndmask")) and mn.endswith("_e32"):
                    reads.add("vcc")
                if mn.startswith("v_writelane"):
                    reads |= first
        else:
            reads = first | rest  # unknown: read everything it names
        self.reads, self.writes = reads, writes


def is_insn(line):
    return bool(INSN_RE.match(line.split(";")[0])) and not line.lstrip().startswith((".", ";"))


def kernel_ranges(lines, kernels):
    """(start, end) line ranges of the named kernels' bodies."""
    out, i = [], 0
    while i < len(lines):
        m = re.match(r"^(_Z\S+):", lines[i])
        if m and any(k in m.group(1) for k in kernels):
            j = i + 1
            while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
                j += 1
            out.append((m.group(1), i + 1, j))
            i = j
        else:
            i += 1
    return out


# ---------------------------------------------------------------- counters --

def _issue(state, ins):
    """Pending loads after `ins` issues.  state: {(reg, cnt): (younger, ooo)}."""
    if ins.mn == "s_waitcnt":
        return _wait(state, ins.line)
    if ins.mem is None:
        # a non-memory write of a pending register: the compiler waited first
        return state
    new = {}
    for (r, c), (age, ooo) in state.items():
        bump = c == ins.mem and not ins.ooo and not ooo
        new[(r, c)] = (min(age + 1, 64) if bump else age, ooo)
    for r in ins.writes:
        for c in ("vm", "lgkm") if ins.mn.startswith("flat_") else (ins.mem,):
            new[(r, c)] = (0, ins.ooo)
    return new


def _wait(state, line):
    text = line.split(";")[0]
    lim = {}
    for c in ("vmcnt", "lgkmcnt"):
        m = re.search(c + r"\((\d+)\)", text)
        if m:
            lim[c[:-3]] = int(m.group(1))
    if re.match(r"^\s+s_waitcnt\s+0\s*$", text):
        lim = {"vm": 0, "lgkm": 0}
    out = {}
    for (r, c), (age, ooo) in state.items():
        n = lim.get(c)
        done = n is not None and (n == 0 if ooo else age >= n)
        if not done:
            out[(r, c)] = (age, ooo)
    return out


def _merge(a, b):
    out = dict(a)
    for k, (age, ooo) in b.items():
        if k in out:
            out[k] = (min(out[k][0], age), out[k][1] or ooo)
        else:
            out[k] = (age, ooo)
    return out


def pending_states(lines, lo, hi):
    """{line index: pending loads just before it} for the instructions of one
    kernel body lines[lo:hi], by a fixpoint over its basic blocks."""
    blocks, labels, cur = [], {}, None
    for i in range(lo, hi):
        ln = lines[i]
        lab = LABEL_RE.match(ln)
        if lab:
            cur = None
            labels[lab.group(1)] = len(blocks)
            blocks.append([])
            cur = blocks[-1]
            continue
        if not is_insn(ln):
            continue
        if cur is None:
            blocks.append([])
            cur = blocks[-1]
        cur.append(i)
        if Insn(ln).mn.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            cur = None
    succ = []
    for b, idx in enumerate(blocks):
        last = Insn(lines[idx[-1]]).mn if idx else ""
        target = None
        if idx and last.startswith(("s_branch", "s_cbranch")):
            t = operands(INSN_RE.match(lines[idx[-1]]).group(2))[0].split()[0]
            if t not in labels:
                raise GuardError(f"branch to unknown label {t}")
            target = labels[t]
        s = []
        if target is not None:
            s.append(target)
        if not (last.startswith(("s_branch", "s_endpgm", "s_setpc"))) and b + 1 < len(blocks):
            s.append(b + 1)
        succ.append(s)
    insns = {i: Insn(lines[i]) for idx in blocks for i in idx}
    ins_state = [None] * len(blocks)
    ins_state[0] = {}
    work = [0]
    while work:
        b = work.pop()
        st = ins_state[b]
        for i in blocks[b]:
            st = _issue(st, insns[i])
        for s in succ[b]:
            merged = st if ins_state[s] is None else _merge(ins_state[s], st)
            if merged != ins_state[s]:
                ins_state[s] = merged
                work.append(s)
    before = {}
    for b, idx in enumerate(blocks):
        st = ins_state[b] if ins_state[b] is not None else {}
        for i in idx:
            before[i] = st
            st = _issue(st, insns[i])
    return before, insns


# ------------------------------------------------------------------ checks --

def _interlocked(p, c, reg):
    """Does the hardware hold consumer c until producer p's write of reg lands
    (so no wait states are needed between them)?"""
    if p.mem is not None and reg in p.writes:
        return True  # a load's destination: the memory counters cover it
    if c.mn.startswith("s_") and c.mem is None and not c.mn.startswith(("s_cbranch", "s_setreg", "s_getreg",
                                                                        "s_sendmsg", "s_movrel")):
        return True
    if c.mn.startswith("v_") and not UNLOCKED_VALU_RE.search(c.mn):
        return reg.startswith("v") or p.mn.startswith("s_")
    return False


def _positions(lines, lo, hi):
    """{key: [slot, ...]} of the instructions in lines[lo:hi]; key = id() of
    the compiler's line each came from; slot counts issue slots."""
    pos, slot = {}, 0
    for i in range(lo, hi):
        ln = lines[i]
        if not is_insn(ln):
            continue
        key = id(ln.orig) if isinstance(ln, Made) and ln.orig is not None else (None if isinstance(ln, Made) else id(ln))
        if key is not None:
            pos.setdefault(key, []).append(slot)
        slot += Insn(ln).slots
    return pos


def check(orig, final, kernels):
    """Raise GuardError listing every violation in `final` (bm_prio's output)
    against `orig` (the compiler's assembly).  Returns a summary dict."""
    problems = []
    o_k = {name: (lo, hi) for name, lo, hi in kernel_ranges(orig, kernels)}
    f_k = {name: (lo, hi) for name, lo, hi in kernel_ranges(final, kernels)}
    if set(o_k) != set(f_k):
        raise GuardError(f"kernel set changed: {sorted(set(o_k) ^ set(f_k))}")
    stats = {"kernels": len(f_k), "inserted": 0, "rewritten": 0, "moved": 0, "deleted": 0, "pairs": 0}
    for name, (flo, fhi) in f_k.items():
        short = name[:60]
        before, insns = pending_states(final, flo, fhi)
        # 1-2: what the pass produced
        for i in range(flo, fhi):
            ln = final[i]
            if not isinstance(ln, Made) or not is_insn(ln):
                continue
            ins = insns[i]
            busy = {r for (r, _c) in before[i]}
            if ln.kind == "rewrite":
                stats["rewritten"] += 1
                o = Insn(ln.orig)
                if not ins.writes <= o.writes or not ins.reads <= (o.reads | o.writes):
                    problems.append(f"{short}: rewrite `{ln.strip()}` of `{ln.orig.strip()}` touches other registers")
            else:
                stats["inserted" if ln.kind == "insert" else "moved"] += 1
            hit = (ins.reads | ins.writes) & busy
            if ln.kind != "rewrite" and hit:
                problems.append(f"{short}: `{ln.strip()}` (line {i - flo}) touches {sorted(hit)} while a load "
                                f"into it is outstanding")
        # 4: an inserted instruction against its neighbours: as a new producer
        # or consumer of a register it must not form a pair the hardware does
        # not interlock within the window (e.g. an SGPR written just before a
        # VMEM reads it, or a VGPR written just after a store issued with it)
        seq, slot = [], 0
        for i in range(flo, fhi):
            if is_insn(final[i]):
                seq.append((i, insns[i], slot))
                slot += insns[i].slots
        for k, (i, x, sx) in enumerate(seq):
            if not (isinstance(final[i], Made) and final[i].kind == "insert") or not (x.reads | x.writes):
                continue
            for j in range(k - 1, -1, -1):
                _i, y, sy = seq[j]
                if sx - sy >= WINDOW:
                    break
                bad = [r for r in y.writes & (x.reads | x.writes) if not _interlocked(y, x, r)]
                if y.reads & x.writes and (y.mem == "vm" or y.mn.startswith(("ds_", "v_readlane", "v_readfirstlane"))):
                    bad += sorted(y.reads & x.writes)
                if bad:
                    problems.append(f"{short}: inserted `{final[i].strip()}` after `{y.line.strip()}` on {sorted(set(bad))}")
            for j in range(k + 1, len(seq)):
                _i, z, sz = seq[j]
                if sz - sx >= WINDOW:
                    break
                bad = [r for r in x.writes & (z.reads | z.writes) if not _interlocked(x, z, r)]
                if bad:
                    problems.append(f"{short}: inserted `{final[i].strip()}` before `{z.line.strip()}` on {sorted(set(bad))}")
        # 3: wait states between the compiler's instructions
        olo, ohi = o_k[name]
        oins = [(id(orig[i]), Insn(orig[i])) for i in range(olo, ohi) if is_insn(orig[i])]
        opos, slot = [], 0
        for _k, ins in oins:
            opos.append(slot)
            slot += ins.slots
        fpos = _positions(final, flo, fhi)
        stats["deleted"] += sum(1 for k, _ in oins if k not in fpos)
        for a, (ka, pa) in enumerate(oins):
            if ka not in fpos:
                continue
            for b in range(a + 1, len(oins)):
                d0 = opos[b] - opos[a]
                if d0 >= WINDOW:
                    break
                kb, pb = oins[b]
                if kb not in fpos:
                    continue
                raw = pa.writes & (pb.reads | pb.writes)
                war = pa.reads & pb.writes
                if not raw and not war:
                    continue
                d1 = min(fpos[kb]) - max(fpos[ka])
                if d1 >= min(d0, WINDOW):
                    continue
                stats["pairs"] += 1
                bad = [r for r in raw if not _interlocked(pa, pb, r)]
                if war and (pa.mem == "vm" or pa.mn.startswith(("ds_", "v_readlane", "v_readfirstlane"))):
                    bad += sorted(war)  # a memory op or lane read may read its operands after issue
                if bad:
                    problems.append(f"{short}: `{pa.line.strip()}` -> `{pb.line.strip()}` on {sorted(set(bad))}: "
                                    f"{d0} slots apart in the compiler's code, {d1} after the pass")
    if problems:
        raise GuardError(f"{len(problems)} unsafe rewrite(s):\n  " + "\n  ".join(problems[:40]))
    return stats
