"""The distributed system around the hot path, on CPU over localhost UDP:
server scheduler (server.py), miner process (miner.run), request client
(client.py), on the LSP transport with lspnet drop injection.

Reference behaviour: project2/README.md:341-417 (Part B spec: Join /
Request / Result, "Result <hash> <nonce>" / "Disconnected", failover and
load balancing), bitcoin/server/server.go:73-197, bitcoin/miner/miner.go:20-74,
bitcoin/client/client.go:14-83.  The Part B graders (ctest/mtest/stest) are
absent from the reference (.MISSING_LARGE_BLOBS:1-10), so results are
checked against the CPU oracle's sequential scan of the whole range.

The miners here search with the CPU oracle (test infrastructure) instead of
the GPU: these tests pin the control plane; tests/test_system_gpu.py runs
the same system with GPU miners.
"""
import collections
import io
import threading
import time

import pytest

from conftest import U64
from distributed_bitcoin_minter_amd import client, lsp, lspnet, miner
from distributed_bitcoin_minter_amd.bitcoin import Message, MsgType, NewJoin, NewRequest, NewResult
from distributed_bitcoin_minter_amd.server import BitcoinServer


@pytest.fixture(autouse=True)
def _reset_drops():
    lspnet.ResetDropPercent()
    lspnet.seed(0x5EED)
    yield
    lspnet.ResetDropPercent()


def params(ms=20, k=50, w=1):
    return lsp.Params(EpochLimit=k, EpochMillis=ms, WindowSize=w)


class OracleSearcher:
    """Stands in for the GPU search (test infrastructure only)."""

    def __init__(self, oracle, delay=0.0, fail_first=False):
        self.oracle = oracle
        self.delay = delay
        self.fail_first = fail_first
        self.jobs = []

    def search(self, data, lo, hi):
        self.jobs.append((lo, hi))
        if self.fail_first and len(self.jobs) == 1:
            raise RuntimeError("miner crashed")
        if self.delay:
            time.sleep(self.delay)
        return self.oracle.search(data.encode(), lo, hi)


class System:
    def __init__(self, chunk, p, target_ms=0):
        """target_ms = 0: fixed chunks (these tests pin the tiling); the
        rate-sized chunks of the product default are tested below."""
        self.p = p
        self.srv = lsp.NewServer(0, p)
        self.bs = BitcoinServer(self.srv, chunk=chunk, target_ms=target_ms)
        self.hostport = f"127.0.0.1:{self.srv.port}"
        self.threads = [threading.Thread(target=self.bs.serve, daemon=True)]
        self.threads[0].start()

    def add_miner(self, searcher):
        def go():
            try:
                miner.run(self.hostport, self.p, searcher=searcher)
            except RuntimeError:
                pass  # a crashing searcher: the miner process dies
        t = threading.Thread(target=go, daemon=True)
        t.start()
        self.threads.append(t)
        return t

    def wait(self, pred, timeout=30):
        t0 = time.monotonic()
        while not pred():
            assert time.monotonic() - t0 < timeout, "timed out"
            time.sleep(0.01)

    def close(self):
        lspnet.ResetDropPercent()
        self.bs.close()
        for t in self.threads:
            t.join(timeout=10)


def test_c1_end_to_end(oracle):
    """BASELINE config C1: server + 1 miner + client, "bradfitz", 0..9999."""
    s = System(chunk=1000, p=params())
    s.add_miner(OracleSearcher(oracle))
    out = io.StringIO()
    assert client.main([s.hostport, "bradfitz", "9999", "--epoch-millis", "20", "--epoch-limit", "50"], out=out) == 0
    assert out.getvalue() == "Result 1419516646206828 9898\n"
    assert s.bs.stats["chunks_done"] == 10
    s.close()


def test_readme_example(oracle):
    s = System(chunk=2, p=params())
    s.add_miner(OracleSearcher(oracle))
    assert client.request(s.hostport, "msg", 2, params()) == (4754799531757243342, 1)  # README:331
    s.close()


def test_c5_shape_16_clients_4_miners_10pct_drop(oracle):
    """BASELINE config C5 at CPU scale: 4 miners, 16 concurrent clients,
    10% read and write drop on every endpoint; every client gets the exact
    sequential-scan answer and the load is spread over all miners."""
    p = params(ms=20, k=200)
    s = System(chunk=600, p=p, target_ms=300)  # the product's rate-sized chunks
    searchers = [OracleSearcher(oracle) for _ in range(4)]
    for m in searchers:
        s.add_miner(m)
    s.wait(lambda: s.bs.stats["joins"] == 4)
    lspnet.SetReadDropPercent(10)
    lspnet.SetWriteDropPercent(10)
    msgs = [f"client-{i:02d}" for i in range(16)]
    max_nonce = 3000 + 137 * 16
    got = {}

    def ask(i):
        got[i] = client.request(s.hostport, msgs[i], max_nonce - 137 * i, p)

    th = [threading.Thread(target=ask, args=(i,)) for i in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    lspnet.ResetDropPercent()
    for i in range(16):
        assert got.get(i) == oracle.search(msgs[i].encode(), 0, max_nonce - 137 * i), i
    assert all(m.jobs for m in searchers)  # every miner took work
    s.close()


def test_lost_miner_job_is_reassigned_to_a_later_miner(oracle):
    """README:413: the job of a miner that dies goes to another miner; with
    none left, it waits for a new one to join."""
    p = params(ms=20, k=5)
    s = System(chunk=500, p=p)
    crashing = OracleSearcher(oracle, fail_first=True)
    s.add_miner(crashing)
    s.wait(lambda: s.bs.stats["joins"] == 1)
    res = {}
    t = threading.Thread(target=lambda: res.setdefault("r", client.request(s.hostport, "bradfitz", 1999, p)))
    t.start()
    s.wait(lambda: s.bs.stats["miners_lost"] == 1)
    assert s.bs.stats["chunks_reassigned"] == 2  # both queued jobs (depth 2)
    healthy = OracleSearcher(oracle)
    s.add_miner(healthy)
    t.join(timeout=60)
    assert res["r"] == oracle.search(b"bradfitz", 0, 1999)
    assert crashing.jobs[0] in healthy.jobs  # the crashed chunk was redone
    s.close()


def test_lost_client_request_is_dropped(oracle):
    """README:414: a request whose client disappears stops being scheduled;
    other clients are still served."""
    p = params(ms=20, k=5)
    s = System(chunk=100, p=p)
    slow = OracleSearcher(oracle, delay=0.02)
    s.add_miner(slow)
    s.wait(lambda: s.bs.stats["joins"] == 1)
    doomed = lsp.NewClient(s.hostport, p)
    doomed.Write(NewRequest("doomed", 0, 10 ** 6).marshal())  # 10,000 chunks
    s.wait(lambda: s.bs.stats["chunks_sent"] >= 2)
    doomed._stop = True  # the client process dies: no Close, no more epochs
    for th in doomed._threads:
        th.join()
    doomed._conn.close()
    s.wait(lambda: s.bs.stats["clients_lost"] == 1)
    sent = s.bs.stats["chunks_sent"]
    assert client.request(s.hostport, "bradfitz", 999, p) == oracle.search(b"bradfitz", 0, 999)
    assert s.bs.stats["chunks_sent"] - sent <= 10 + 2  # only the new request's chunks (+ the doomed queue)
    s.close()


def test_client_prints_disconnected_without_server():
    probe = lspnet.listen(0)
    port = probe.local_port()
    probe.close()
    out = io.StringIO()
    client.main([f"127.0.0.1:{port}", "msg", "2", "--epoch-millis", "20", "--epoch-limit", "3"], out=out)
    assert out.getvalue() == "Disconnected\n"


def test_client_prints_disconnected_when_server_dies(oracle):
    p = params(ms=20, k=5)
    srv = lsp.NewServer(0, p)  # a server that accepts but never answers, then dies
    out = io.StringIO()
    t = threading.Thread(target=client.main, args=([f"127.0.0.1:{srv.port}", "msg", "2", "--epoch-millis", "20",
                                                    "--epoch-limit", "5"],), kwargs={"out": out})
    t.start()
    assert srv.Read()[1] == NewRequest("msg", 0, 2).marshal()
    srv._stop = True
    for th in srv._threads:
        th.join()
    srv._conn.close()
    t.join(timeout=10)
    assert out.getvalue() == "Disconnected\n"


def test_client_rejects_bad_max_nonce():
    assert client.main(["127.0.0.1:1", "m", "-1"]) == 2
    assert client.main(["127.0.0.1:1", "m", str(U64 + 1)]) == 2


def test_miner_shuts_down_when_server_is_lost(oracle):
    p = params(ms=20, k=4)
    srv = lsp.NewServer(0, p)
    done = []
    t = threading.Thread(target=lambda: done.append(miner.run(f"127.0.0.1:{srv.port}", p,
                                                              searcher=OracleSearcher(oracle))))
    t.start()
    cid, raw = srv.Read()
    assert Message.unmarshal(raw) == NewJoin()  # miner.go:34-38
    srv.Write(cid, NewRequest("msg", 0, 2).marshal())
    assert Message.unmarshal(srv.Read()[1]) == NewResult(4754799531757243342, 1)
    srv._stop = True
    for th in srv._threads:
        th.join()
    srv._conn.close()
    t.join(timeout=10)
    assert done == [1]


# ---- scheduler unit tests (no network) -----------------------------------

class FakeLSP:
    """Records writes; connections in `dead` refuse them."""

    def __init__(self):
        self.sent = []
        self.dead = set()

    def Write(self, cid, payload):
        if cid in self.dead:
            raise lsp.LSPError("gone", cid)
        self.sent.append((cid, Message.unmarshal(payload)))

    def jobs_for(self, cid):
        return [(m.Lower, m.Upper) for c, m in self.sent if c == cid and m.Type == MsgType.Request]

    def results_for(self, cid):
        return [(m.Hash, m.Nonce) for c, m in self.sent if c == cid and m.Type == MsgType.Result]


def make(chunk, depth=1, **kw):
    f = FakeLSP()
    kw.setdefault("target_ms", 0)  # fixed chunks unless a test asks for rate-sized ones
    return f, BitcoinServer(f, chunk=chunk, depth=depth, **kw)


def test_chunks_tile_the_range_exactly():
    for lo, hi, chunk in [(0, 9999, 1000), (5, 5, 3), (0, 10, 3), (U64 - 10, U64, 4), (0, U64, 1 << 62), (7, 6, 5)]:
        f, s = make(chunk)
        s._on_message(1, NewJoin())
        s._on_message(100, NewRequest("x", lo, hi))
        seen = []
        while f.jobs_for(1)[len(seen):]:
            a, b = f.jobs_for(1)[len(seen)]
            seen.append((a, b))
            s._on_message(1, NewResult(a, a))
        if lo > hi:
            assert seen == [] and f.results_for(100) == [(U64, U64)]  # miner.go:45-46, zero iterations
            continue
        assert seen[0][0] == lo and seen[-1][1] == hi
        assert all(b + 1 == c for (_, b), (c, _) in zip(seen, seen[1:]))
        assert all(b - a + 1 <= chunk for a, b in seen)
        assert f.results_for(100) == [(lo, lo)]


def test_merge_is_lexicographic_whatever_the_arrival_order():
    """server.go:113 keeps the first strict-< result in arrival order; the
    build's merge equals the sequential scan: on a hash tie the smaller nonce."""
    f, s = make(10)
    for m in (1, 2, 3):
        s._on_message(m, NewJoin())
    s._on_message(100, NewRequest("x", 0, 29))
    s._on_message(3, NewResult(7, 25))  # chunk [20,29] reports first
    s._on_message(2, NewResult(7, 12))
    s._on_message(1, NewResult(9, 3))
    assert f.results_for(100) == [(7, 12)]


def test_fair_share_between_requests():
    f, s = make(10)
    miners = [1, 2, 3, 4]
    for m in miners:
        s._on_message(m, NewJoin())
    s._on_message(100, NewRequest("a", 0, 10 ** 6))
    assert all(len(f.jobs_for(m)) == 1 for m in miners)  # request a alone: all 4 miners
    s._on_message(200, NewRequest("b", 0, 10 ** 6))
    s._on_message(1, NewResult(1, 1))  # freed miners go to b until shares are equal
    s._on_message(2, NewResult(1, 1))
    inflight = {r.client: r.inflight for r in s.requests.values()}
    assert inflight == {100: 2, 200: 2}
    s._on_message(300, NewRequest("c", 0, 10 ** 6))
    for m in (3, 4, 1, 2):
        s._on_message(m, NewResult(1, 1))
    inflight = sorted(r.inflight for r in s.requests.values())
    assert inflight[-1] - inflight[0] <= 1 and sum(inflight) == 4


def test_miner_lost_while_busy_or_idle():
    f, s = make(10)
    s._on_message(1, NewJoin())
    s._on_message(2, NewJoin())
    s._on_message(100, NewRequest("x", 0, 9))  # one chunk -> miner 1
    assert f.jobs_for(1) == [(0, 9)]
    s._on_lost(2)  # idle miner lost: nothing to reassign
    s._on_lost(1)  # busy miner lost: chunk waits for a new miner
    assert s.stats["chunks_reassigned"] == 1 and f.results_for(100) == []
    s._on_message(3, NewJoin())
    assert f.jobs_for(3) == [(0, 9)]
    s._on_message(1, NewResult(0, 0))  # a stray result from the dead miner is ignored
    s._on_message(3, NewResult(5, 5))
    assert f.results_for(100) == [(5, 5)]


def test_write_to_vanished_miner_keeps_the_chunk():
    f, s = make(10)
    f.dead.add(1)
    s._on_message(1, NewJoin())
    s._on_message(2, NewJoin())
    s._on_message(100, NewRequest("x", 0, 9))
    assert f.jobs_for(2) == [(0, 9)]


def test_results_answered_in_request_order_per_client():
    f, s = make(10)
    s._on_message(1, NewJoin())
    s._on_message(2, NewJoin())
    s._on_message(100, NewRequest("a", 0, 9))   # -> miner 1
    s._on_message(100, NewRequest("b", 0, 9))   # -> miner 2
    s._on_message(2, NewResult(2, 2))           # b finishes first: held back
    assert f.results_for(100) == []
    s._on_message(1, NewResult(1, 1))
    assert f.results_for(100) == [(1, 1), (2, 2)]


def test_lost_client_results_ignored():
    f, s = make(10)
    s._on_message(1, NewJoin())
    s._on_message(100, NewRequest("a", 0, 99))
    s._on_lost(100)
    s._on_message(1, NewResult(1, 1))  # result for a dead client: miner goes idle
    assert f.results_for(100) == [] and s.idle_miners() == [1]
    assert len(f.jobs_for(1)) == 1


@pytest.mark.parametrize("target_ms", [0, 300])
@pytest.mark.parametrize("seed", range(12))
def test_scheduler_random_event_sequences(seed, target_ms):
    """Random joins, losses, requests, client deaths and out-of-order
    results against the scheduler (no network).  Invariants: every request
    whose client survives is answered exactly once, in its client's order,
    with the lexicographic min over its whole inclusive range; a miner never
    holds two chunks; no chunk of a live request is lost.  The toy hash has
    many ties, so the nonce tie-break is exercised."""
    import random

    rng = random.Random(seed)

    def toy_hash(data, n):
        return (n * 7 + len(data)) % 13

    def brute(data, lo, hi):
        return min(((toy_hash(data, n), n) for n in range(lo, hi + 1)), default=(U64, U64))

    now = [0.0]  # a fake clock: rate-sized chunks (target_ms > 0) see random job times

    def clock():
        now[0] += rng.random() * 0.2
        return now[0]
    f, s = make(rng.choice([1, 3, 7, 50]), depth=rng.choice([1, 2, 3]), target_ms=target_ms, clock=clock,
                max_mult=8)
    next_id = [1]
    miners, clients = set(), {}
    expected = {}  # client -> [answers in order]

    def new_id():
        next_id[0] += 1
        return next_id[0]

    def deliver(mid):
        jobs = s.miners.get(mid)
        if jobs:
            rid, lo, hi = jobs[0][:3]
            data = next((r.data for r in s.requests.values() if r.rid == rid), "gone")
            s._on_message(mid, NewResult(*brute(data, lo, hi)))

    for _ in range(300):
        ev = rng.random()
        if ev < 0.15 or not miners:
            m = new_id()
            miners.add(m)
            s._on_message(m, NewJoin())
        elif ev < 0.35:
            c = rng.choice(list(clients)) if clients and rng.random() < 0.3 else new_id()
            lo = rng.randint(0, 200)
            hi = lo + rng.randint(-2, 150)
            data = f"d{c}-{lo}"
            clients.setdefault(c, True)
            s._on_message(c, NewRequest(data, lo, hi))
            expected.setdefault(c, []).append(brute(data, lo, hi) if lo <= hi else (U64, U64))
        elif ev < 0.45 and len(miners) > 1:
            m = rng.choice(sorted(miners))
            miners.discard(m)
            s._on_lost(m)
        elif ev < 0.5 and clients:
            c = rng.choice(sorted(clients))
            del clients[c]
            expected.pop(c, None)
            s._on_lost(c)
        else:
            busy = [m for m in miners if s.miners.get(m)]
            if busy:
                deliver(rng.choice(busy))
        assert all(len(j) <= s.depth for j in s.miners.values())
    # drain: answer every outstanding chunk (a miner must exist)
    if not miners:
        m = new_id()
        miners.add(m)
        s._on_message(m, NewJoin())
    for _ in range(100000):
        busy = [m for m in miners if s.miners.get(m)]
        if not busy:
            break
        deliver(busy[0])
    assert not s.requests, "requests left unanswered"
    for c, answers in expected.items():
        assert f.results_for(c) == answers, c


def test_depth_two_queues_the_next_job():
    """With depth 2 every miner holds its next chunk before finishing the
    current one; slots fill level by level and a lost miner's whole queue
    is reassigned in ascending order."""
    f, s = make(10, depth=2)
    s._on_message(1, NewJoin())
    s._on_message(2, NewJoin())
    s._on_message(100, NewRequest("x", 0, 59))
    assert f.jobs_for(1) == [(0, 9), (20, 29)] and f.jobs_for(2) == [(10, 19), (30, 39)]
    s._on_message(1, NewResult(5, 5))      # answers its oldest job first
    assert f.jobs_for(1)[-1] == (40, 49)
    s._on_lost(2)                          # (10,19) and (30,39) go back, lowest first
    assert list(s.requests.values())[0].retry == collections.deque([(10, 19), (30, 39)])
    s._on_message(3, NewJoin())
    assert f.jobs_for(3) == [(10, 19), (30, 39)]
    for m, jobs in ((1, [(20, 29), (40, 49)]), (3, [(10, 19), (30, 39)])):
        for lo, hi in jobs:
            s._on_message(m, NewResult(lo + 1, lo))
    s._on_message(1, NewResult(99, 50))    # (50, 59) went to miner 1 when it freed up
    assert f.results_for(100) == [(5, 5)]


def test_server_survives_malformed_client_payloads(oracle):
    """A client whose LSP payloads are not valid bitcoin Messages (null, an
    array, Data not a string, a float nonce ...) is logged and ignored; the
    server keeps serving, including that client's later valid Request
    (these used to crash the server loop)."""
    s = System(chunk=1000, p=params())
    s.add_miner(OracleSearcher(oracle))
    c = lsp.NewClient(s.hostport, params())
    for raw in [b"null", b"[]", b"7", b'{"Type":1,"Data":5,"Upper":10}', b'{"Type":1,"Data":"x","Upper":1.5}',
                b'{"Type":1,"Data":["x"],"Upper":10}', b'{"Type":"1"}', b"\xff"]:
        c.Write(raw)
    c.Write(NewRequest("bradfitz", 0, 9999).marshal())
    got = Message.unmarshal(c.Read())
    assert (got.Type, got.Hash, got.Nonce) == (MsgType.Result, 1419516646206828, 9898)
    c.Close()
    s.close()


# ---- rate-sized chunks (round 6) --------------------------

def test_chunk_for_policy():
    """server.chunk_for: about target_s of the miner's work, rounded to whole
    base chunks, in [1, max_mult], at most twice the previous multiple, at
    most the miner's rate share of what the request has left."""
    from distributed_bitcoin_minter_amd.server import chunk_for
    B = 1 << 32
    assert chunk_for(B, 0.3, 64, None, 0, 1 << 40, 0.5) == 1              # no rate yet: one base
    assert chunk_for(B, 0.0, 64, 1e12, 8, 1 << 40, 0.5) == 1              # sizing off
    assert chunk_for(B, 0.3, 64, 55e9, 4, 1 << 40, 0.5) == 4              # 16.5 G = 3.8 bases
    assert chunk_for(B, 0.3, 64, 440e9, 4, 1 << 50, 0.9) == 8             # 31 bases, ramp: 2 x 4
    assert chunk_for(B, 0.3, 64, 440e9, 32, 1 << 50, 0.9) == 31
    assert chunk_for(B, 0.3, 16, 440e9, 32, 1 << 50, 0.9) == 16           # cap
    assert chunk_for(B, 0.3, 64, 440e9, 32, 10 * B, 0.5) == 5             # its share of the tail
    assert chunk_for(B, 0.3, 64, 1e3, 1, 1 << 40, 0.01) == 1              # never below one base


def _simulate(rates, base, target_ms, nonces, depth=2, max_mult=64):
    """The scheduler against miners of given rates (nonces/s) on a simulated
    clock: each miner works through its jobs in order and answers each one
    when its nonces are done.  Returns (per miner: the sizes of its jobs,
    the simulated seconds)."""
    import heapq
    now = [0.0]
    f, s = make(base, depth=depth, target_ms=target_ms, max_mult=max_mult, clock=lambda: now[0])
    mids = list(range(1, len(rates) + 1))
    for m in mids:
        s._on_message(m, NewJoin())
    s._on_message(100, NewRequest("x", 0, nonces - 1))
    busy_until = {m: 0.0 for m in mids}
    done = {m: 0 for m in mids}
    events = []

    def plan(m):  # queue the completion of m's next unplanned job
        jobs = f.jobs_for(m)
        while done[m] < len(jobs) and len([e for e in events if e[1] == m]) < 1:
            lo, hi = jobs[done[m]]
            t = max(now[0], busy_until[m]) + (hi - lo + 1) / rates[m - 1]
            busy_until[m] = t
            heapq.heappush(events, (t, m, lo, hi))
            break
    for m in mids:
        plan(m)
    while events:
        t, m, lo, hi = heapq.heappop(events)
        now[0] = t
        done[m] += 1
        s._on_message(m, NewResult(lo, lo))
        for x in mids:
            plan(x)
    assert f.results_for(100) == [(0, 0)]
    return {m: [b - a + 1 for a, b in f.jobs_for(m)] for m in mids}, now[0]


def test_fast_miner_gets_proportionally_larger_chunks():
    """Two miners, one 8x faster: once the rates are measured, the fast one's
    jobs are about 8x the slow one's (each about target_ms of its own work),
    and the request's tail is split by rate so both finish close together.
    With fixed chunks the same run takes far more jobs."""
    base = 1000
    rates = [160_000.0, 20_000.0]           # nonces/s: 8x apart
    sizes, secs = _simulate(rates, base, 200, 4_000_000)
    fast, slow = sizes[1], sizes[2]
    # steady state: the middle of the run (ramp-up before, the tail after)
    f_mid = sorted(fast)[len(fast) // 2]
    s_mid = sorted(slow)[len(slow) // 2]
    assert f_mid == 32 * base and s_mid == 4 * base, (fast, slow)   # 0.2 s of each miner's work
    assert 7.0 <= f_mid / s_mid <= 9.0
    ideal = 4_000_000 / sum(rates)
    assert secs < ideal * 1.15, (secs, ideal)
    fixed, secs_fixed = _simulate(rates, base, 0, 4_000_000)
    assert len(fixed[1]) + len(fixed[2]) == 4000 and len(fast) + len(slow) < 300
    # the wire format is unchanged: every job is an inclusive [Lower, Upper]
    # tile of the request, in base multiples except the request's end


def test_rate_sized_chunks_end_to_end(oracle):
    """The same over the network: two CPU miners whose searches take time in
    proportion to their nonces, one 8x faster; the answer is the sequential
    scan's and the fast miner's median job is about 8x the slow one's."""
    class Paced(OracleSearcher):
        def __init__(self, oracle, rate):
            super().__init__(oracle)
            self.rate = rate

        def search(self, data, lo, hi):
            self.jobs.append((lo, hi))
            time.sleep((hi - lo + 1) / self.rate)
            return self.oracle.search(data.encode(), lo, hi)

    p = params(ms=20, k=100)
    s = System(chunk=2000, p=p, target_ms=200)
    fast, slow = Paced(oracle, 400_000), Paced(oracle, 50_000)
    s.add_miner(fast)
    s.add_miner(slow)
    s.wait(lambda: s.bs.stats["joins"] == 2)
    n = 1_200_000
    assert client.request(s.hostport, "paced", n - 1, p) == oracle.search(b"paced", 0, n - 1)
    med = lambda js: sorted(b - a + 1 for a, b in js)[len(js) // 2]  # noqa: E731
    ratio = med(fast.jobs) / med(slow.jobs)
    assert 4.0 <= ratio <= 12.0, (fast.jobs, slow.jobs)
    s.close()


def test_lost_fast_miners_chunk_is_cut_for_the_slow_one():
    """A fast miner holding rate-sized jobs dies: its chunks go back to the
    front of the request and are re-issued cut to the size of the miner that
    takes them (here a new miner: one base), in ascending order, the rest
    staying queued; the request still tiles exactly."""
    now = [0.0]
    f, s = make(1000, depth=2, target_ms=200, clock=lambda: now[0])
    s._on_message(1, NewJoin())
    s._on_message(100, NewRequest("x", 0, 10 ** 7 - 1))
    for _ in range(6):  # miner 1 runs at 160k nonces/s: its jobs ramp up to 32 bases
        rid, lo, hi, sent = s.miners[1][0]
        now[0] = max(now[0], sent) + (hi - lo + 1) / 160_000
        s._on_message(1, NewResult(lo, lo))
    big = [b - a + 1 for a, b in f.jobs_for(1)]
    assert big[-1] >= 8000, big
    held = [(lo, hi) for _, lo, hi, _ in s.miners[1]]
    s._on_lost(1)
    s._on_message(2, NewJoin())  # a new miner: no rate yet, one base per job
    got = f.jobs_for(2)
    assert got[0] == (held[0][0], held[0][0] + 999) and got[1] == (held[0][0] + 1000, held[0][0] + 1999), (got, held)
    r = list(s.requests.values())[0]
    assert r.retry[0] == (held[0][0] + 2000, held[0][1]) and r.retry[1] == held[1]
