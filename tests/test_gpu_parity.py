"""GPU parity: the gfx950 search (bm_search_gpu) and hash (bm_hash_gpu)
through the C ABI, bit-exact against the golden fixtures and the CPU oracle.

Reference semantics checked: bitcoin.Hash (hash.go:11-15) and the miner's
strict-'<' ascending min-scan (miner.go:45-46, 59-65) on inclusive bounds
(README:329).  Every kernel layout the planner can emit is exercised.
"""
import random

import pytest

from conftest import U64, load_golden
from distributed_bitcoin_minter_amd import plan_segments

pytestmark = pytest.mark.gpu

M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]


def test_readme_known_answers(gpu_ctx):
    ka = load_golden("known_answers.json")
    for e in ka["hash"]:
        assert gpu_ctx.hash_many(e["msg"].encode(), [e["nonce"]]) == [e["hash"]]
    for e in ka["search"]:
        assert gpu_ctx.search(e["msg"].encode(), e["lower"], e["upper"]) == (e["hash"], e["nonce"])


def test_hash_vectors(gpu_ctx):
    by_msg = {}
    for v in load_golden("hash_vectors.json")["vectors"]:
        by_msg.setdefault(v["msg_hex"], []).append(v)
    for mh, vs in by_msg.items():
        got = gpu_ctx.hash_many(bytes.fromhex(mh), [v["nonce"] for v in vs])
        assert got == [v["hash"] for v in vs]


def test_search_vectors(gpu_ctx):
    for c in load_golden("search_vectors.json")["cases"]:
        got = gpu_ctx.search(bytes.fromhex(c["msg_hex"]), c["lower"], c["upper"])
        assert got == (c["hash"], c["nonce"]), c


@pytest.mark.parametrize("cfg", ["C1", "C2", "C3"])
def test_full_range_configs(gpu_ctx, cfg):
    """BASELINE configs C1/C2/C3 over their whole ranges vs the oracle's
    whole-range answers (tests/golden/full_range.json)."""
    c = next(c for c in load_golden("full_range.json")["cases"] if c["config"] == cfg)
    got = gpu_ctx.search(bytes.fromhex(c["msg_hex"]), c["lower"], c["upper"])
    assert got == (c["hash"], c["nonce"])


def _layout_cases():
    """One (msg, lower, upper, max_windows) per kernel layout (nbv, p),
    found with the CPU planner: windows of ~3,000 nonces.  nbv = 2 layouts
    need more than 64 high-digit windows; max_windows = 0 forces them on a
    small range (the planner knob exists for exactly this)."""
    want = {(1, p) for p in range(64)} | {(2, p) for p in range(17)}
    found = {}
    for mw in (64, 0):
        for L in range(0, 128):
            msg = bytes((97 + (i * 7) % 26) for i in range(L))
            for D in range(1, 21):
                lo = 0 if D == 1 else 10 ** (D - 1)
                top = U64 if D == 20 else 10 ** D - 1
                for start in (lo, lo + 123_457 if D > 7 else lo, max(lo, top - 3000)):
                    hi = min(start + 3000, top)
                    for s in plan_segments(msg, start, hi, max_windows=mw):
                        key = (s.nbv, s.p)
                        if key in want and key not in found:
                            found[key] = (msg, s.nonce_base + s.vlo, s.nonce_base + s.vhi, mw)
            if len(found) == len(want):
                return found
    return found


_LAYOUTS = _layout_cases()


def test_layout_table_complete():
    assert len(_LAYOUTS) == 64 + 17


@pytest.mark.parametrize("key", sorted(_LAYOUTS))
def test_every_kernel_layout(gpu_ctx, oracle, key):
    """Each layout with both task shapes: 10-nonce tasks (what a small launch
    gets by default) and 100-nonce tasks (forced; large launches' default)."""
    msg, lo, hi, mw = _LAYOUTS[key]
    want = oracle.search(msg, lo, hi, threads=8)
    gpu_ctx.set_max_windows(mw)
    try:
        for td in (0, 2):
            gpu_ctx.set_task_digits(td)
            assert gpu_ctx.search(msg, lo, hi) == want, td
            st = gpu_ctx.last_stats()
            assert any((st.launch[i].nbv, st.launch[i].p) == key for i in range(st.recorded))
    finally:
        gpu_ctx.set_max_windows(64)
        gpu_ctx.set_task_digits(0)


def test_random_windows(gpu_ctx, oracle):
    rng = random.Random(0x5EED)
    for k in range(40):
        gpu_ctx.set_task_digits(2 if k % 2 else 0)
        L = rng.choice([0, 3, 8, 20, 45, 54, 55, 60, 63, 64, 100, 120, 128, 250, 600])
        msg = bytes(rng.randrange(32, 127) for _ in range(L))
        D = rng.randint(1, 20)
        dlo = 0 if D == 1 else 10 ** (D - 1)
        dhi = U64 if D == 20 else 10 ** D - 1
        lo = rng.randint(dlo, dhi)
        hi = min(U64, lo + rng.randint(0, 1 << rng.randint(4, 18)))
        assert gpu_ctx.search(msg, lo, hi) == oracle.search(msg, lo, hi, threads=8), (L, lo, hi)
    gpu_ctx.set_task_digits(0)


def test_edges(gpu_ctx, oracle):
    msg = b"bradfitz"
    assert gpu_ctx.search(msg, 10, 9) == (U64, U64)          # empty range
    assert gpu_ctx.search(msg, 7, 7) == (oracle.hash(msg, 7), 7)
    assert gpu_ctx.search(msg, U64, U64) == (oracle.hash(msg, U64), U64)
    assert gpu_ctx.search(b"", 0, 5000) == oracle.search(b"", 0, 5000)
    raw = bytes(range(256)) * 2                                 # arbitrary bytes, 512 B
    assert gpu_ctx.search(raw, 10 ** 12, 10 ** 12 + 3000) == oracle.search(raw, 10 ** 12, 10 ** 12 + 3000)
    # digit-count boundaries inside one call: 9->10 ... 19->20 digits
    for d in range(1, 20):
        lo = 10 ** d - 700
        assert gpu_ctx.search(msg, lo, lo + 1400) == oracle.search(msg, lo, lo + 1400), d


@pytest.fixture(scope="module")
def generic_pad_ctx():
    """A context that never uses search_kernel_padc / _padk (BTCMINER_PADC=0,
    read at creation): the generic padding-block kernel for every such layout."""
    import os
    from distributed_bitcoin_minter_amd import Context
    old = os.environ.get("BTCMINER_PADC")
    os.environ["BTCMINER_PADC"] = "0"
    try:
        ctx = Context(num_gpus=1)
    finally:
        if old is None:
            del os.environ["BTCMINER_PADC"]
        else:
            os.environ["BTCMINER_PADC"] = old
    yield ctx
    ctx.close()


@pytest.mark.parametrize("P", range(55, 64))
def test_padding_block_layouts_folded_and_generic(gpu_ctx, generic_pad_ctx, oracle, P):
    """The padding-block layouts (last digit at byte P >= 55 of its block, so
    SHA-256's length words spill into a block of their own), 10-digit
    nonces, both task shapes: a message of K whole prefix blocks plus the
    varying one runs the kernel with the padding block's constants folded --
    K = 0: search_kernel_padc (IV folded too; stats pad_block = 2), K = 1..15:
    search_kernel_padk<P, K> (midstate from kernargs; pad_block = 2 + K;
    K = 1, 2 since round 5, 3..15 since round 6: every message an LSP packet
    carries) -- and K = 16, or any K under BTCMINER_PADC=0, the generic
    kernel (pad_block = 1); every answer equals the oracle's."""
    lo = 10 ** 9 + 7_777_777
    hi = lo + 20_000
    msgs = [bytes(97 + (i + k) % 26 for i in range(P - 10 + 64 * k)) for k in range(17)]  # ends at byte P of block k
    runs = [(gpu_ctx, msgs[k], 2 + k) for k in range(16)] + [(gpu_ctx, msgs[16], 1)]
    runs += [(generic_pad_ctx, msgs[k], 1) for k in (0, 1, 2, 3, 15)]
    for ctx, msg, pad in runs:
        want = oracle.search(msg, lo, hi, threads=8)
        for td in (0, 2):
            ctx.set_task_digits(td)
            try:
                assert ctx.search(msg, lo, hi) == want, (len(msg), pad, td)
            finally:
                ctx.set_task_digits(0)
            st = ctx.last_stats()
            assert [(st.launch[i].p, st.launch[i].pad_block) for i in range(st.recorded)] == [(P, pad)]


def _layout_ranges():
    import json
    import os
    from conftest import ROOT
    return json.load(open(os.path.join(ROOT, "tests", "golden", "layout_ranges.json")))["cases"]


@pytest.mark.parametrize("case", _layout_ranges(), ids=lambda c: f"L{c['len']}")
def test_layout_full_range_goldens(gpu_ctx, case):
    """Round 4's kernels at full size: a whole 2^32-nonce 10-digit range for
    a padc message (L = 50, and L = 46 with the two-word inner loop), a
    padding-block one after a prefix block (L = 114: search_kernel_padk<P, 1>
    since round 5, the generic kernel before), and an NBV = 2
    one (L = 59), against the AVX-512 oracle's full scans
    (tests/golden/make_layout_golden.py); the launch stats name the kernel."""
    msg = bytes.fromhex(case["msg_hex"])
    assert gpu_ctx.search(msg, case["lower"], case["upper"]) == (case["hash"], case["nonce"])
    st = gpu_ctx.last_stats()
    dom = max((st.launch[i] for i in range(st.recorded)), key=lambda x: x.nonces)
    # 114, 178, 242, 1010: padk<60, K> with K = 1, 2, 3, 15 (pad_block 2 + K)
    want = {50: (1, 2), 46: (1, 2), 114: (1, 3), 59: (2, 0), 178: (1, 4), 242: (1, 5), 1010: (1, 17)}[case["len"]]
    assert (dom.nbv, dom.pad_block) == want, (dom.nbv, dom.pad_block)


def test_split_and_merge_equals_whole(gpu_ctx):
    """Size-independent property at full C2 size: scanning two halves and
    taking the lexicographic min equals one scan of the whole range."""
    msg, lo, hi = b"bradfitz", 0, 2 ** 32 - 1
    whole = gpu_ctx.search(msg, lo, hi)
    mid = 1_626_825_724  # split right at C2's argmin
    a = gpu_ctx.search(msg, lo, mid)
    b = gpu_ctx.search(msg, mid + 1, hi)
    assert min(a, b) == whole
    assert gpu_ctx.hash_many(msg, [whole[1]]) == [whole[0]]


def test_idempotent(gpu_ctx):
    r = [gpu_ctx.search(M120, U64 - (1 << 28), U64) for _ in range(3)]
    assert r[0] == r[1] == r[2]


def test_hash_batch_random(gpu_ctx, oracle):
    rng = random.Random(11)
    for L in [0, 1, 54, 55, 63, 64, 119, 200]:
        msg = bytes(rng.randrange(256) for _ in range(L))
        ns = [rng.randrange(1 << rng.randint(1, 64)) for _ in range(3000)]
        assert gpu_ctx.hash_many(msg, ns) == [oracle.hash(msg, n) for n in ns]


def test_bitcoin_mirror_and_miner(oracle):
    from distributed_bitcoin_minter_amd import Miner, bitcoin
    assert bitcoin.Hash("msg", 1) == 4754799531757243342
    with Miner() as m:
        out = bitcoin.Message.unmarshal(m.handle_payload(bitcoin.NewRequest("msg", 0, 2).marshal()))
        assert out == bitcoin.NewResult(4754799531757243342, 1)
    with Miner(exclusive_upper=True) as m:  # miner.go:59's literal i < Upper
        assert m.search("bradfitz", 0, 10000) == oracle.search_excl(b"bradfitz", 0, 10000)


def test_device_list_context(oracle):
    from distributed_bitcoin_minter_amd import Context
    with Context(devices=[0]) as c:
        assert c.num_devices() == 1
        assert c.search(b"bradfitz", 0, 9999) == (1419516646206828, 9898)


@pytest.mark.parametrize("mode", [1, 2])
def test_combine_modes(mode):
    """The multi-device combine paths on one GPU: RCCL allgather (ncclCommInitAll
    over the context's devices + ncclAllGather of the 16-B partial) and plain
    host copies must both return the C2-window answer."""
    from distributed_bitcoin_minter_amd import Context
    with Context(devices=[0]) as c:
        c.set_combine(mode)
        for _ in range(2):
            assert c.search(b"bradfitz", 0, 9999) == (1419516646206828, 9898)
        assert c.search(b"msg", 0, 2) == (4754799531757243342, 1)


def test_c4_shape_single_process(gpu_ctx, oracle):
    """C4's path (one process, every visible GPU, one ctx) at 2^34 nonces:
    the answer re-hashes to itself, equals the min over two halves, and its
    neighbourhood re-scanned by the oracle agrees."""
    from distributed_bitcoin_minter_amd import Context, device_count
    msg, lo, hi = b"bradfitz", 0, (1 << 34) - 1
    with Context(num_gpus=device_count()) as c:
        h, n = c.search(msg, lo, hi)
    assert gpu_ctx.hash_many(msg, [n]) == [h]
    mid = (1 << 33) - 1
    assert min(gpu_ctx.search(msg, lo, mid), gpu_ctx.search(msg, mid + 1, hi)) == (h, n)
    a, b = max(lo, n - 20000), min(hi, n + 20000)
    assert oracle.search(msg, a, b, threads=8) == (h, n)


@pytest.mark.parametrize("streams", [1, 2, 4])
def test_launch_streams(oracle, monkeypatch, streams):
    """Launches of one call spread over 1, 2 or 4 streams (BTCMINER_STREAMS,
    read at context creation; default 2): the multi-launch ranges (every digit
    length from 1, a 19/20-digit boundary, the C2 range) give the same answers,
    and the small windows equal the oracle."""
    from distributed_bitcoin_minter_amd import Context
    monkeypatch.setenv("BTCMINER_STREAMS", str(streams))
    c2 = next(c for c in load_golden("full_range.json")["cases"] if c["config"] == "C2")
    with Context(devices=[0]) as c:
        assert c.search(b"bradfitz", 0, 9999) == (1419516646206828, 9898)
        for msg, lo, hi in ((b"bradfitz", 0, 3_000_000), (M120, 10**19 - 1_500_000, 10**19 + 1_500_000)):
            assert c.search(msg, lo, hi) == oracle.search(msg, lo, hi, threads=8)
        assert c.search(bytes.fromhex(c2["msg_hex"]), c2["lower"], c2["upper"]) == (c2["hash"], c2["nonce"])


@pytest.mark.parametrize("tail", [0, 1, 99_991, 1 << 24])
def test_tail_launch_split(oracle, monkeypatch, tail):
    """The biggest launch's last BTCMINER_TAIL nonces run as a launch of their
    own (10-nonce tasks) when there are streams to overlap on: the split at
    any size, including 1 nonce and a prime, leaves every answer unchanged."""
    from distributed_bitcoin_minter_amd import Context
    monkeypatch.setenv("BTCMINER_TAIL", str(tail))
    c2 = next(c for c in load_golden("full_range.json")["cases"] if c["config"] == "C2")
    with Context(devices=[0]) as c:
        for msg, lo, hi in ((b"bradfitz", 0, 3_000_000), (M120, 2**64 - 2_000_000, 2**64 - 1)):
            assert c.search(msg, lo, hi) == oracle.search(msg, lo, hi, threads=8)
        assert c.search(bytes.fromhex(c2["msg_hex"]), c2["lower"], c2["upper"]) == (c2["hash"], c2["nonce"])


def test_maximum_message_sizes(gpu_ctx, oracle):
    """Messages up to the ABI's maximum (BM_MAX_MSG_LEN = 1 MiB: README:61's
    LSP payloads are ~1 KB, so this is far past anything a Request carries):
    the host folds every whole block into the midstate and the kernel sees
    only the tail, whatever the length; one byte more is refused."""
    from distributed_bitcoin_minter_amd import BtcMinerError
    from distributed_bitcoin_minter_amd._lib import BM_EINVAL
    rng = random.Random(0x1EE7)
    big = bytes(rng.randrange(256) for _ in range(1 << 20))
    for L in (65_535, 65_536 + 55, (1 << 20) - 9, 1 << 20):
        msg = big[:L]
        lo = rng.randrange(10 ** 11, 10 ** 12)
        assert gpu_ctx.search(msg, lo, lo + 99) == oracle.search(msg, lo, lo + 99, threads=8), L
        ns = [rng.randrange(1 << 64) for _ in range(8)]
        assert gpu_ctx.hash_many(msg, ns) == [oracle.hash(msg, n) for n in ns], L
    with pytest.raises(BtcMinerError) as ei:
        gpu_ctx.search(big + b"x", 0, 9)
    assert ei.value.status == BM_EINVAL


def test_failed_calls_leave_outputs_untouched(gpu_ctx):
    """include/btcminer.h: "On failure the output arguments are left
    untouched" -- a Go caller that ignores the status must not read a half
    result.  Refused arguments (BM_EINVAL) and a search that fails part-way
    (bm_ctx_set_test_fault: BM_EINTERNAL after some launches) leave a
    sentinel result and hash array as they were; the context then answers
    correctly again."""
    import ctypes
    from distributed_bitcoin_minter_amd import _lib
    lib, h = _lib.load(), gpu_ctx.handle
    sentinel = (0x0123456789ABCDEF, 0xFEDCBA9876543210)
    r = _lib.Result(*sentinel)
    big = b"\0" * ((1 << 20) + 1)
    assert lib.bm_search_gpu(h, big, len(big), 0, 9, ctypes.byref(r)) == _lib.BM_EINVAL
    assert lib.bm_search_gpu(h, None, 3, 0, 9, ctypes.byref(r)) == _lib.BM_EINVAL
    assert (r.hash, r.nonce) == sentinel
    try:
        for k in (0, 1, 3):
            gpu_ctx.set_test_fault(k)
            assert lib.bm_search_gpu(h, b"bradfitz", 8, 0, (1 << 32) - 1, ctypes.byref(r)) == _lib.BM_EINTERNAL
            assert (r.hash, r.nonce) == sentinel, k
    finally:
        gpu_ctx.set_test_fault(-1)  # the session's shared context
    outs = (ctypes.c_uint64 * 4)(*([0xA5A5A5A5A5A5A5A5] * 4))
    nonces = (ctypes.c_uint64 * 4)(0, 1, 2, 3)
    assert lib.bm_hash_gpu(h, big, len(big), nonces, 4, outs) == _lib.BM_EINVAL
    assert lib.bm_hash_gpu(h, b"msg", 3, None, 4, outs) == _lib.BM_EINVAL
    assert list(outs) == [0xA5A5A5A5A5A5A5A5] * 4
    assert lib.bm_search_gpu(h, b"msg", 3, 0, 2, ctypes.byref(r)) == _lib.BM_OK
    assert (r.hash, r.nonce) == (4754799531757243342, 1)  # README:331
