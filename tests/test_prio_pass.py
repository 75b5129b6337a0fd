"""csrc/bm_prio.py, the build step that adds wave-priority toggles to the
search kernels' assembly and folds known SGPR constants (CPU only).

The pass must not change what the kernel computes: it only inserts
s_setprio, replaces an SGPR operand by the literal the SGPR provably holds,
and splits v_add3_u32 x, y, K into two v_add_u32.  A small interpreter for
the ops involved checks that on random register values."""
import os
import random

import pytest
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc"))

import bm_prio  # noqa: E402

M32 = 0xFFFFFFFF

KERNEL = """\
_ZN2bm13search_kernelILi18ELi1EEEvNS_10SearchArgsEPNS_7PartialEPy:
\ts_mov_b32 s16, 0x923f82a4
.LBB5_1:
\tv_add_u32_e32 v20, s55, v26
\tv_alignbit_b32 v10, v7, v7, 25
\tv_bitop3_b32 v10, v21, v11, v10 bitop3:0x96
\ts_mov_b32 s10, 0x1e376c08
\tv_add3_u32 v2, v2, v3, s10
\tv_add3_u32 v3, s16, v9, v3
\tv_add_u32_e32 v46, s16, v46
\tv_lshrrev_b32_e32 v47, 10, v44
\tv_add3_u32 v11, v3, v10, v2
\ts_cbranch_scc1 .LBB5_1
.Lfunc_end5:
"""


def run_block(lines, regs):
    """Interpret the straight-line ops of the test kernel."""
    r = dict(regs)

    def val(o):
        o = o.strip()
        if o.startswith(("v", "s")) and o[1:].isdigit():
            return r[o]
        return int(o, 0) & M32

    for ln in lines:
        t = ln.strip()
        if not t or t.endswith(":") or t.startswith(("s_setprio", "s_cbranch", ".", "_Z")):
            continue
        op, rest = t.split(None, 1)
        ops = [o.strip() for o in rest.split(" bitop3:")[0].split(",")]
        d = ops[0]
        if op == "s_mov_b32":
            r[d] = val(ops[1])
        elif op == "v_add_u32_e32":
            r[d] = (val(ops[1]) + val(ops[2])) & M32
        elif op == "v_add3_u32":
            r[d] = (val(ops[1]) + val(ops[2]) + val(ops[3])) & M32
        elif op == "v_lshrrev_b32_e32":
            r[d] = val(ops[2]) >> val(ops[1])
        elif op == "v_alignbit_b32":
            r[d] = (((val(ops[1]) << 32) | val(ops[2])) >> (val(ops[3]) & 31)) & M32
        elif op == "v_bitop3_b32":
            assert "bitop3:0x96" in t
            r[d] = val(ops[1]) ^ val(ops[2]) ^ val(ops[3])
        else:
            raise AssertionError(op)
    return r


def test_classify():
    assert bm_prio.classify("v_add_u32_e32", "v1, v2, v3") == "F"
    assert bm_prio.classify("v_add_u32_e32", "v1, 0x1234, v3") == "F"
    assert bm_prio.classify("v_add_u32_e32", "v1, s5, v3") == "S"        # SGPR operand
    assert bm_prio.classify("v_bitop3_b32", "v1, v2, v3, v4 bitop3:0x96") == "F"
    assert bm_prio.classify("v_bitop3_b32", "v1, v2, s3, v4 bitop3:0x96") == "S"
    assert bm_prio.classify("v_alignbit_b32", "v1, v2, v2, 7") == "S"
    assert bm_prio.classify("v_add3_u32", "v1, v2, v3, v4") == "S"
    assert bm_prio.classify("v_lshlrev_b32_e32", "v1, 3, v2") == "S"
    assert bm_prio.classify("v_lshrrev_b32_e32", "v1, 3, v2") == "F"
    assert bm_prio.classify("v_xor_b32_sdwa", "v1, v2, v3") == "S"


def test_toggles_at_run_starts_and_labels():
    lines = KERNEL.splitlines(keepends=True)
    out, n_toggle, n_valu = bm_prio.run(lines, ["search_kernel"], 2, 0)
    body = [l.strip() for l in out]
    assert n_valu == 8
    # every VALU is preceded (within its run) by the toggle of its class
    cur = None
    for t in body:
        if t.endswith(":"):
            cur = None
        elif t.startswith("s_setprio"):
            cur = int(t.split()[1])
        elif t.startswith("v_"):
            cls = bm_prio.classify(t.split()[0], t.split(None, 1)[1])
            assert cur == (2 if cls == "S" else 0), t
    # a label resets the state: the first VALU after .LBB5_1 has its own toggle
    i = body.index(".LBB5_1:")
    assert body[i + 1].startswith("s_setprio")


def test_fold_and_split_keep_results():
    lines = KERNEL.splitlines(keepends=True)
    out, n_fold, n_split = bm_prio.fold_sgpr_constants(lines, ["search_kernel"])
    text = "".join(out)
    assert n_split == 2 and n_fold == 1, (n_fold, n_split)
    assert "v_add3_u32 v2, v2, v3, s10" not in text          # split with the block-local constant
    assert "v_add_u32_e32 v46, 0x923f82a4, v46" in text       # single-definition constant folded
    assert "v_add3_u32 v11, v3, v10, v2" in text              # all-VGPR add3 untouched
    final, _, _ = bm_prio.run(out, ["search_kernel"], 2, 0)
    rng = random.Random(7)
    for _ in range(200):
        regs = {f"v{i}": rng.getrandbits(32) for i in range(64)}
        regs.update({f"s{i}": rng.getrandbits(32) for i in range(64)})
        assert run_block(lines, regs) == run_block(final, regs)


def test_multi_def_sgpr_not_folded_across_blocks():
    src = """\
_ZN2bm13search_kernelILi5ELi1EEEvNS_10SearchArgsEPNS_7PartialEPy:
\ts_mov_b32 s10, 7
.LBB1_1:
\tv_add_u32_e32 v1, s10, v1
\ts_mov_b32 s10, 9
\ts_cbranch_scc1 .LBB1_1
.Lfunc_end1:
"""
    out, n_fold, n_split = bm_prio.fold_sgpr_constants(src.splitlines(keepends=True), ["search_kernel"])
    assert n_fold == 0 and n_split == 0   # s10 has two definitions; at the loop head it is not known


def test_split_all_vgpr_add3_keeps_results_with_aliased_dest():
    """--split-add3-every (measured, not on by default: profiles/r01/ab_split_add3.log)."""
    src = """\
_ZN2bm13search_kernelILi18ELi1EEEvNS_10SearchArgsEPNS_7PartialEPy:
.LBB5_1:
\tv_add3_u32 v1, v2, v3, v4
\tv_add3_u32 v2, v3, v4, v2
\tv_add3_u32 v3, v3, v5, v3
\tv_add3_u32 v4, v4, v4, v4
\tv_add3_u32 v5, v1, s3, v2
\ts_cbranch_scc1 .LBB5_1
.Lfunc_end5:
"""
    lines = src.splitlines(keepends=True)
    out, n = bm_prio.split_add3(lines, ["search_kernel"], 1)
    assert n == 3                                  # d == every source, and SGPR operands, stay add3
    assert "v_add3_u32 v4, v4, v4, v4" in "".join(out)
    rng = random.Random(11)
    for _ in range(200):
        regs = {f"v{i}": rng.getrandbits(32) for i in range(8)}
        regs.update({f"s{i}": rng.getrandbits(32) for i in range(8)})
        assert run_block(lines, regs) == run_block(out, regs)
    out2, n2 = bm_prio.split_add3(lines, ["search_kernel"], 2)
    assert n2 == 1


def test_vop3b_carry_destination_counts_as_a_definition():
    """An SGPR set by s_mov_b32 and ALSO written as the carry-out of a VOP3B op
    (v_add_co_u32_e64 v, s[..], ...) holds that constant only until the carry
    write: the pass must not fold it after that point, neither through the
    whole-kernel 'single definition' rule nor the in-block rule."""
    k = """\
_ZN2bm13search_kernelILi18ELi1EEEvNS_10SearchArgsEPNS_7PartialEPy:
\ts_mov_b32 s20, 0x923f82a4
\ts_mov_b32 s21, 0x11111111
.LBB5_1:
\tv_add_u32_e32 v1, s20, v2
\tv_add_co_u32_e64 v3, s[20:21], v4, v5
\tv_add_u32_e32 v6, s20, v7
\tv_add3_u32 v8, s21, v9, v10
\tv_mad_u64_u32 v[12:13], s[22:23], v14, v15, 0
\ts_cbranch_scc1 .LBB5_1
.Lfunc_end5:
"""
    assert bm_prio._sdefs("\tv_add_co_u32_e64 v3, s[20:21], v4, v5") == [20, 21]
    assert bm_prio._sdefs("\tv_mad_u64_u32 v[12:13], s[22:23], v14, v15, 0") == [22, 23]
    assert bm_prio._sdefs("\tv_add_u32_e32 v1, s20, v2") == []
    out, n_fold, n_split = bm_prio.fold_sgpr_constants(k.splitlines(keepends=True), ["search_kernel"])
    out = "".join(out)
    assert n_fold == 0 and n_split == 0
    # s20 / s21 have two definitions: no literal may replace them anywhere
    assert "0x923f82a4, v2" not in out and "0x923f82a4, v7" not in out
    assert "v_add_u32_e32 v6, s20, v7" in out and "v_add3_u32 v8, s21, v9, v10" in out


def _interp(lines, regs):
    """Straight-line interpreter for the ops of a search-kernel inner loop
    (VALU as one lane, SALU, s_setprio ignored)."""
    r = dict(regs)

    def val(o):
        o = o.strip()
        if o in r:
            return r[o]
        return int(o, 0) & M32

    def bitop3(a, b, c, imm):
        out = 0
        for k in range(32):
            idx = (((a >> k) & 1) << 2) | (((b >> k) & 1) << 1) | ((c >> k) & 1)
            out |= ((imm >> idx) & 1) << k
        return out

    for ln in lines:
        t = ln.strip()
        if not t or t.startswith(("s_setprio", ";")):
            continue
        op, rest = t.split(None, 1)
        imm = int(rest.split("bitop3:")[1], 0) if "bitop3:" in rest else None
        ops = [o.strip() for o in rest.split(" bitop3:")[0].split(",")]
        d, a = ops[0], [val(o) for o in ops[1:]]
        if op in ("s_mov_b32", "v_mov_b32_e32"):
            v = a[0]
        elif op in ("v_add_u32_e32", "s_add_i32", "s_add_u32"):
            v = a[0] + a[1]
        elif op == "v_add3_u32":
            v = a[0] + a[1] + a[2]
        elif op == "v_xad_u32":
            v = (a[0] ^ a[1]) + a[2]
        elif op == "v_lshrrev_b32_e32":
            v = a[1] >> (a[0] & 31)
        elif op == "s_lshr_b32":
            v = a[0] >> (a[1] & 31)
        elif op == "s_lshl_b32":
            v = a[0] << (a[1] & 31)
        elif op in ("v_xor_b32_e32", "s_xor_b32"):
            v = a[0] ^ a[1]
        elif op in ("v_or_b32_e32", "s_or_b32"):
            v = a[0] | a[1]
        elif op in ("v_and_b32_e32", "s_and_b32"):
            v = a[0] & a[1]
        elif op == "v_alignbit_b32":
            v = ((a[0] << 32) | a[1]) >> (a[2] & 31)
        elif op == "v_bitop3_b32":
            v = bitop3(a[0], a[1], a[2], imm)
        else:
            raise AssertionError(op)
        r[d] = v & M32
    return r


def _inner_block(sfile, kernel):
    """The straight-line body of the kernel's biggest basic block."""
    import re
    text = open(sfile).read()
    i = text.index(kernel)
    j = text.index(".Lfunc_end", i)
    blocks, cur = {}, None
    for ln in text[i:j].splitlines(keepends=True):
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m:
            cur = m.group(1)
            blocks[cur] = []
        elif cur:
            blocks[cur].append(ln)
    body = max(blocks.values(), key=lambda b: sum(1 for ln in b if ln.lstrip().startswith("v_")))
    return [ln for ln in body if bm_prio._defs_uses(ln) is not None or ln.strip().startswith("s_setprio")]


def test_cluster_runs_preserves_the_inner_loop():
    """--cluster (measured: C2 +0.2%, C3 -0.1%, off by default,
    profiles/r02/ab_pin_cluster.log) reorders only along register dependences:
    the real C2 inner loop (from the build's device assembly) computes the
    same registers before and after, on random inputs."""
    import glob
    srcs = glob.glob(os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc", "build", "inst1_16_23.dev.s"))
    if not srcs:
        pytest.skip("device assembly not built (make -C distributed_bitcoin_minter_amd/csrc)")
    lines = open(srcs[0]).readlines()
    lines, _, _ = bm_prio.fold_sgpr_constants(lines, ["search_kernel"])
    kern = "_ZN2bm13search_kernelILi18ELi1EEEvNS_10SearchArgsEPNS_7PartialEPy:"
    before = _inner_block_from(lines, kern)
    after = _inner_block_from(bm_prio.cluster_runs(lines, ["search_kernel"], max_run=0), kern)
    assert sorted(before) == sorted(after) and before != after
    rng = random.Random(5)
    for _ in range(20):
        regs = {f"v{i}": rng.getrandbits(32) for i in range(256)}
        regs.update({f"s{i}": rng.getrandbits(32) for i in range(106)})
        assert _interp(before, regs) == _interp(after, regs)


def _inner_block_from(lines, kernel):
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".s", delete=False) as f:
        f.writelines(lines)
    try:
        return _inner_block(f.name, kernel)
    finally:
        os.unlink(f.name)


def test_cluster_schedule_respects_war_and_scc():
    """Synthetic block: a write-after-read on v1 and SALU ops chained through
    SCC-writing instructions keep their order."""
    blk = ["\tv_add_u32_e32 v2, v1, v3\n", "\tv_alignbit_b32 v1, v4, v4, 7\n", "\ts_lshr_b32 s5, s6, 3\n",
           "\tv_xor_b32_e32 v7, s5, v2\n", "\tv_alignbit_b32 v8, v1, v1, 2\n", "\ts_lshl_b32 s6, s9, 1\n"]
    out = bm_prio._schedule(blk, 0)
    assert out.index(blk[0]) < out.index(blk[1])      # v1 read before it is overwritten
    assert out.index(blk[2]) < out.index(blk[5])      # s6 read, then written (and SCC)
    rng = random.Random(1)
    for _ in range(50):
        regs = {f"v{i}": rng.getrandbits(32) for i in range(10)}
        regs.update({f"s{i}": rng.getrandbits(32) for i in range(10)})
        assert _interp(blk, regs) == _interp(out, regs)


def test_drop_dead_smov_keeps_the_inner_loop():
    """--drop-dead-smov removes only s_mov_b32 writes that a later s_mov_b32
    of the same SGPR in the block overwrites with no read between: the real C2
    inner loop leaves every register (the removed SGPRs included, whose last
    write stays) as before, on random inputs; a read between two writes, and
    a block boundary, keep the first write."""
    import glob
    srcs = glob.glob(os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc", "build", "inst1_16_23.dev.s"))
    if not srcs:
        pytest.skip("device assembly not built (make -C distributed_bitcoin_minter_amd/csrc)")
    lines, _, _ = bm_prio.fold_sgpr_constants(open(srcs[0]).readlines(), ["search_kernel"])
    kern = "_ZN2bm13search_kernelILi18ELi1EEEvNS_10SearchArgsEPNS_7PartialEPy:"
    dropped, n = bm_prio.drop_dead_smov(lines, ["search_kernel"])
    before, after = _inner_block_from(lines, kern), _inner_block_from(dropped, kern)
    assert n > 0 and len(after) < len(before)
    assert all(ln.strip().startswith("s_mov_b32") for ln in set(before) - set(after))
    rng = random.Random(9)
    for _ in range(10):
        regs = {f"v{i}": rng.getrandbits(32) for i in range(256)}
        regs.update({f"s{i}": rng.getrandbits(32) for i in range(106)})
        assert _interp(before, regs) == _interp(after, regs)
    blk = ["_Z3foo:\n", "\ts_mov_b32 s4, 1\n", "\tv_add_u32_e32 v1, s4, v1\n", "\ts_mov_b32 s4, 2\n",
           "\ts_mov_b32 s5, 3\n", ".LBB0_1:\n", "\ts_mov_b32 s5, 4\n", "\ts_mov_b32 s6, 5\n",
           "\ts_mov_b32 s6, 6\n", ".Lfunc_end0:\n"]
    out, n = bm_prio.drop_dead_smov(blk, ["foo"])
    assert n == 1 and "\ts_mov_b32 s6, 5\n" not in out and len(out) == len(blk) - 1


def test_no_inner_loop_spills_in_the_build():
    """Every search kernel of the built library -- 83 search_kernel<P, NBV>,
    9 search_kernel_padc<P>, 135 search_kernel_padk<P, K> (K = 1..15) --
    keeps its inner loop free of scratch / memory ops (tools/check_inner.py
    on the device assembly, innermost loop): the occupancy requests (7
    waves/SIMD for the 1-block and most NBV = 2 layouts) must not push the hot
    loop into spills.  The only inner loops that read spilled SGPRs back
    (v_readlane) are the generic padding-block kernel's (its 64 kernarg K+W
    words), which since round 6 serve only messages over 15 prefix blocks."""
    import glob
    import subprocess
    import sys
    build = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc", "build")
    if not glob.glob(os.path.join(build, "inst*-hip-amdgcn-amd-amdhsa-gfx950.s")):
        pytest.skip("device assembly not built (make -C distributed_bitcoin_minter_amd/csrc)")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_inner.py"), build], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "227 kernels checked, 0 with scratch" in r.stdout, r.stdout[-500:]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_inner.py"), build, "-v"],
                       capture_output=True, text=True, timeout=300)
    lanes = [ln.split()[0] for ln in r.stdout.splitlines() if "lane-spill=" in ln and "lane-spill=0" not in ln]
    assert lanes and all(x.endswith(":1") and int(x.split(":")[0]) >= 55 for x in lanes), lanes


# ---- the assembly guard (csrc/bm_asm_guard.py) -------------------------------

import bm_asm_guard as guard  # noqa: E402

BUILD = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc", "build")


def _passes(lines, spacer=None, drop=0, cluster=-1):
    """bm_prio's pipeline as main() runs it (fold, options, toggles)."""
    ks = ["search_kernel"]
    out, _, _ = bm_prio.fold_sgpr_constants(list(lines), ks)
    if drop:
        out, _ = bm_prio.drop_dead_smov(out, ks, "\ts_nop 0\n" if drop == 2 else None)
    if spacer:
        out, _ = bm_prio.space_dependent_valu(out, ks, spacer)
    if cluster >= 0:
        out = bm_prio.cluster_runs(out, ks, max_run=cluster)
    out, _, _ = bm_prio.run(out, ks, 2, 0)
    return out


SMEM_KERNEL = """\
_ZN2bm13search_kernelILi16ELi1EEEvNS_10SearchArgsEPNS_7PartialEPy:
\ts_load_dwordx4 s[0:3], s[12:13], 0x1e0
\tv_mov_b32_e32 v2, s25
\tv_bitop3_b32 v2, s24, v2, v3 bitop3:0xca
\tv_alignbit_b32 v3, s20, s20, 2
\ts_waitcnt lgkmcnt(0)
\tv_mov_b32_e32 v4, s0
\tv_add_u32_e32 v5, v4, v2
\tv_xor_b32_e32 v6, v5, v4
\tv_xor_b32_e32 v7, v6, v4
\tv_xor_b32_e32 v8, v7, v4
\tv_xor_b32_e32 v9, v8, v4
\tv_xor_b32_e32 v10, v9, v4
\tv_xor_b32_e32 v11, v10, v4
\tglobal_store_dwordx4 v12, v[0:3], s[0:1]
\ts_endpgm
.Lfunc_end5:
"""


def test_guard_refuses_a_write_racing_an_outstanding_smem_load():
    """Round 2's faulting variant: `s_mov_b32 s0, s0` between
    dependent VALU landed while `s_load_dwordx4 s[0:3]` (the partials and
    counter pointers) was still outstanding in search_kernel<16, 1> of the
    8-wave build.  The self-move reads the stale s0 and writes it back, so a
    load landing in between loses its low half.  The guard refuses it; the
    same spacer after the wait, and the s_nop spacer, pass."""
    orig = SMEM_KERNEL.splitlines(keepends=True)
    bad = _passes(orig, spacer="\ts_mov_b32 s0, s0\n")
    assert "\ts_mov_b32 s0, s0\n" in bad
    with pytest.raises(guard.GuardError, match=r"s_mov_b32 s0, s0.*\['s0'\].*outstanding"):
        guard.check(orig, bad, ["search_kernel"])
    guard.check(orig, _passes(orig, spacer="\ts_nop 0\n"), ["search_kernel"])
    # the same instruction inserted after the wait, away from any memory op, is fine ...
    late = list(orig)
    late.insert(6, guard.Made("\ts_mov_b32 s0, s0\n", "insert"))
    guard.check(orig, late, ["search_kernel"])
    # ... but not right before the store that reads s[0:1] as its address
    # (rule 4, conservative: an SALU write feeding a VMEM address)
    near = list(orig)
    near.insert(14, guard.Made("\ts_mov_b32 s0, s0\n", "insert"))
    with pytest.raises(guard.GuardError, match="before `global_store_dwordx4"):
        guard.check(orig, near, ["search_kernel"])


def test_guard_counter_model():
    """LDS returns in order within lgkmcnt, SMEM out of order (only
    lgkmcnt(0) retires it), VMEM in order within vmcnt; a join keeps what
    either path left pending."""
    k = """\
_ZN2bm13search_kernelILi3ELi1EEEvNS_10SearchArgsEPNS_7PartialEPy:
\ts_load_dword s4, s[0:1], 0x0
\tds_read_b32 v1, v0
\tds_read_b32 v2, v0 offset:4
\ts_waitcnt lgkmcnt(1)
\tv_add_u32_e32 v9, v9, v9
\tscratch_load_dword v3, off, off
\tscratch_load_dword v4, off, off offset:4
\ts_waitcnt vmcnt(1)
\ts_cbranch_scc1 .LBB0_2
\tds_read_b32 v5, v0
.LBB0_2:
\tv_add_u32_e32 v8, v8, v8
\ts_endpgm
.Lfunc_end0:
"""
    lines = k.splitlines(keepends=True)
    _, lo, hi = guard.kernel_ranges(lines, ["search_kernel"])[0]
    before, _ = guard.pending_states(lines, lo, hi)
    at = lambda text: {r for r, _c in before[next(i for i in range(lo, hi) if lines[i].strip() == text)]}
    p = at("v_add_u32_e32 v9, v9, v9")
    assert "v1" not in p and "v2" in p and "s4" in p      # lgkmcnt(1): the older LDS read is done, SMEM is not
    p = at("v_add_u32_e32 v8, v8, v8")
    assert "v3" not in p and "v4" in p and "v5" in p      # vmcnt(1) retires v3; v5 pending on the fall-through path


def test_guard_refuses_shrinking_a_padded_pair_and_foreign_rewrites():
    """Deleting an instruction between a VALU write of v1 and a DPP read of it
    (which the hardware does not interlock) shortens what the compiler padded;
    a rewrite that reads a register its original did not is refused too."""
    k = """\
_ZN2bm13search_kernelILi3ELi1EEEvNS_10SearchArgsEPNS_7PartialEPy:
\tv_add_u32_e32 v1, v2, v3
\ts_mov_b32 s4, 1
\ts_mov_b32 s4, 2
\tv_mov_b32_dpp v2, v1 row_shr:1 row_mask:0xf bank_mask:0xf
\tv_add_u32_e32 v6, s4, v6
\ts_endpgm
.Lfunc_end0:
"""
    orig = k.splitlines(keepends=True)
    dropped, n = bm_prio.drop_dead_smov(list(orig), ["search_kernel"])
    assert n == 1
    with pytest.raises(guard.GuardError, match="v_mov_b32_dpp"):
        guard.check(orig, dropped, ["search_kernel"])
    noped, _ = bm_prio.drop_dead_smov(list(orig), ["search_kernel"], "\ts_nop 0\n")
    guard.check(orig, noped, ["search_kernel"])          # same slot count: accepted
    foreign = list(orig)
    foreign[5] = guard.Made("\tv_add_u32_e32 v6, v7, v6\n", "rewrite", orig[5])
    with pytest.raises(guard.GuardError, match="touches other registers"):
        guard.check(orig, foreign, ["search_kernel"])


@pytest.mark.parametrize("name", ["inst1_16_23", "inst1_56_63"])
def test_guard_on_the_built_assembly(name):
    """The shipped pipeline passes the guard on the real device assembly
    (the build runs the same check and fails on a violation); the s0 spacer
    variant is refused on the padding-block layouts, whose compiler code
    keeps `s_load_dwordx4 s[0:3]` outstanding across VALU rounds."""
    src = os.path.join(BUILD, f"{name}.dev.s")
    if not os.path.exists(src):
        pytest.skip("device assembly not built (make -C distributed_bitcoin_minter_amd/csrc)")
    orig = open(src).readlines()
    st = guard.check(orig, _passes(orig), ["search_kernel"])
    # 8 search_kernel<P, 1> per range, + search_kernel_padc<P> and
    # search_kernel_padk<P, 1>, <P, 2> for P = 56..63
    assert st["kernels"] == {"inst1_16_23": 8, "inst1_56_63": 32}[name]
    assert st["inserted"] > 1000 and st["rewritten"] > 0 and st["deleted"] == 0
    guard.check(orig, _passes(orig, drop=2), ["search_kernel"])
    if name == "inst1_56_63":
        with pytest.raises(guard.GuardError, match="outstanding"):
            guard.check(orig, _passes(orig, spacer="\ts_mov_b32 s0, s0\n"), ["search_kernel"])
