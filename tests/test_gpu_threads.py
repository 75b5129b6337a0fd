"""The C ABI's threading contract (include/btcminer.h).

* A context may be used from any OS thread, one call at a time: cgo moves a
  goroutine between OS threads, and the HIP current device is per thread, so
  every entry point selects its devices itself.  Here each call comes from a
  thread that never touched HIP before.
* Separate contexts are independent: threads with a context each search at
  the same time on the same GPU (ctypes releases the GIL around the calls)
  and every answer stays bit-exact.

Reference semantics: bitcoin.Hash (hash.go:11-15) and the strict-'<' scan
(miner.go:45-46, 59-65); answers come from the committed goldens."""
import threading

import pytest

from conftest import load_golden
from distributed_bitcoin_minter_amd import Context

pytestmark = pytest.mark.gpu


def _cases():
    out = [(bytes.fromhex(c["msg_hex"]), c["lower"], c["upper"], (c["hash"], c["nonce"]))
           for c in load_golden("search_vectors.json")["cases"]]
    for e in load_golden("known_answers.json")["search"]:
        out.append((e["msg"].encode(), e["lower"], e["upper"], (e["hash"], e["nonce"])))
    return out


def _on_thread(fn):
    box = {}

    def run():
        try:
            box["v"] = fn()
        except BaseException as e:  # re-raised on the caller's thread
            box["e"] = e
    t = threading.Thread(target=run)
    t.start()
    t.join(timeout=300)
    assert not t.is_alive(), "call did not return"
    if "e" in box:
        raise box["e"]
    return box["v"]


def test_one_context_from_fresh_threads(gpu_ctx):
    """Every call from a new OS thread (goroutine migration under cgo)."""
    cases = _cases()[::7]
    for msg, lo, hi, want in cases:
        assert _on_thread(lambda: gpu_ctx.search(msg, lo, hi)) == want, (msg, lo, hi)
    c2 = next(c for c in load_golden("full_range.json")["cases"] if c["config"] == "C2")
    got = _on_thread(lambda: gpu_ctx.search(bytes.fromhex(c2["msg_hex"]), c2["lower"], c2["upper"]))
    assert got == (c2["hash"], c2["nonce"])
    ka = load_golden("known_answers.json")["hash"]
    for e in ka:
        assert _on_thread(lambda: gpu_ctx.hash_many(e["msg"].encode(), [e["nonce"]])) == [e["hash"]]


def test_contexts_on_concurrent_threads():
    """Four threads, a context each, searching at once: the golden cases
    dealt round-robin, and one thread also runs C2's whole range (2^32
    nonces) so the others' launches share the GPU with a long one."""
    cases = _cases()
    c2 = next(c for c in load_golden("full_range.json")["cases"] if c["config"] == "C2")
    nthreads = 4
    work = [cases[i::nthreads] for i in range(nthreads)]
    work[0] = [(bytes.fromhex(c2["msg_hex"]), c2["lower"], c2["upper"], (c2["hash"], c2["nonce"]))] + work[0]
    bad, errs = [], []
    start = threading.Barrier(nthreads)

    def worker(mine):
        try:
            with Context(num_gpus=1) as ctx:
                start.wait(timeout=120)
                for _ in range(2):
                    for msg, lo, hi, want in mine:
                        got = ctx.search(msg, lo, hi)
                        if got != want:
                            bad.append((msg, lo, hi, got, want))
        except BaseException as e:
            errs.append(repr(e))
    ts = [threading.Thread(target=worker, args=(w,)) for w in work]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    assert not errs, errs
    assert not bad, bad[:5]


def test_multi_slot_context_from_fresh_threads_keeps_its_submission_pool():
    """Round 6: a multi-device context keeps one submission thread
    per device but the first across searches (its SubmitPool), whatever OS
    thread calls it -- cgo moves goroutines between threads.  Twelve searches
    of a 4-slot context, each from a new thread, then a close: every answer
    equals the oracle's, every call reports 4 submitting threads, and the
    close returns (the pool's threads end with the context)."""
    import threading
    from distributed_bitcoin_minter_amd import Context
    cases = [(b"bradfitz", 0, 9999, (1419516646206828, 9898)), (b"msg", 0, 2, (4754799531757243342, 1))]
    got, threads = [], []
    with Context(devices=[0, 0, 0, 0]) as c:
        for i in range(12):
            msg, lo, hi, want = cases[i % 2]

            def go():
                got.append((c.search(msg, lo, hi), want, c.last_stats().start_threads))
            t = threading.Thread(target=go)
            t.start()
            t.join(timeout=60)
            threads.append(t)
    assert len(got) == 12 and all(g == w and n == 4 for g, w, n in got), got
