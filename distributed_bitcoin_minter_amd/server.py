"""Bitcoin server: the range scheduler between request clients and miners.

Reference: project2/bitcoin/server/server.go (``acceptMessage`` :73-142,
``scheduleJobs`` :145-197, ``minerLoad = 24`` :18) and the Part B spec,
project2/README.md:341-417.  The reference does not compile;
this module implements the behaviour the spec asks for, over the same wire
format (JSON ``bitcoin.Message`` inside LSP payloads):

* A miner connects and sends ``Join`` (README:376); it is then idle.
* A client sends ``Request(Data, Lower, Upper)`` (README:382-385).  The server
  cuts ``[Lower, Upper]`` (inclusive, README:329) into chunks of ``chunk``
  nonces and hands them to idle miners as ``Request`` messages.
* Each miner answers ``Result(Hash, Nonce)``; when every chunk of a request
  is back, the client gets ``Result`` with the minimum (README:392-393).

Differences from server.go, each deliberate:

* Chunk size.  ``minerLoad = 24`` (:18) makes a GPU miner spend all its time
  in the protocol; the default here is 2^32 nonces (about 0.13 s on one
  MI355X), the retune SURVEY.md §8f(f1) asks for.  (:157-169 also lose the
  intended ``upper = lower + 24`` to ``:=`` shadowing; chunks here tile the
  range exactly.)
* Merge.  server.go:113 keeps the first strict-``<`` result in ARRIVAL order,
  so a hash tie between two chunks resolves differently run to run.  Here
  the merge is the lexicographic (hash, nonce) minimum, which equals the
  sequential strict-``<`` scan of the whole range whatever
  order the chunks come back in.
* Failures (README:408-417, absent from server.go but for :177-179).  A lost
  miner's chunk goes back to the front of its request's queue and is handed
  to the next idle miner (or waits for one to join).  A lost client's request
  is dropped; chunks already on miners finish and their results are ignored.

Scheduler (README:417 asks for it to be documented): fair share by
assignment count.  Whenever a miner has a free job slot, it gets the next
chunk of the active request that currently has the FEWEST chunks in flight,
ties going to the oldest request.  With m miners and r requests each request
therefore holds floor(m/r) or ceil(m/r) of the miners' slots at any moment,
and a new request gets slots as soon as the next ones free up instead of
waiting for earlier requests to drain.  Chunks of one request are issued in
ascending order.

Chunk size per miner (round 6).  A fixed chunk does not fit every miner: a
miner driving 8 GPUs (the Go shim's default, bm_ctx_create(0)) finishes a
2^32-nonce job in about 10 ms, most of it per-call cost.  So ``chunk`` is the
BASE size, and each miner's jobs are a multiple of it sized from the miner's
own measured rate (``chunk_for``): about ``target_ms`` of its work per job
(default 300 ms), at most ``max_mult`` bases (default 64), at most twice the
miner's previous multiple (a ramp, so one odd sample cannot jump the size),
and at most the miner's rate-proportional share of what the request has left
(so a fast miner does not take a short request's whole tail while slower
miners idle).  The rate is the median of the miner's last 5 jobs, each its
nonces over the time from when the miner could start it (its send, or the
previous result if that came later) to its result.  A new miner gets one
base, and a lost miner's chunk is re-issued cut to the size of whoever takes
it.  ``target_ms = 0`` keeps the fixed chunk.  The wire format is
unchanged: a Request's [Lower, Upper] is just wider.

Job queue depth.  Each miner holds up to ``depth`` jobs (default 2; the
reference's one-job-per-miner is depth 1).  A miner works through its jobs in
order (LSP delivers in order), so when a GPU finishes a chunk the next one is
already in its window: it does not idle for the Result -> Request round
trip, which under packet loss includes a whole LSP epoch (2 s by default)
per dropped message.  Free slots are filled level by level: every miner gets
its first job before any gets a second.

The server is one event loop on one thread (the LSP endpoint has its own
reader/epoch threads): every decision happens in ``_on_message`` /
``_on_lost``, so there are no locks in the scheduler itself.
"""
import argparse
import collections
import itertools
import sys
import time

from . import lsp
from .bitcoin import Message, MsgType, NewRequest, NewResult, U64_MAX

DEFAULT_CHUNK = 1 << 32
DEFAULT_DEPTH = 2
DEFAULT_TARGET_MS = 300   # per-miner job time the chunk sizing aims at
DEFAULT_MAX_MULT = 64     # largest job, in base chunks
RATE_SAMPLES = 5          # a miner's rate: the median of its last jobs


def chunk_for(base, target_s, max_mult, rate, prev_mult, remaining, share):
    """Multiple of `base` nonces for a miner's next job (module docstring):
    rate (nonces/s, None before the miner's first result) x target_s, rounded,
    in [1, max_mult], at most 2 x prev_mult, and at most the miner's `share`
    (its fraction of all miners' rates) of the request's `remaining` nonces,
    rounded up to a base.  Returns the multiple k >= 1."""
    if target_s <= 0 or not rate:
        return 1
    k = int(rate * target_s / base + 0.5)
    k = max(1, min(k, max_mult, 2 * max(1, prev_mult)))
    if 0 < share < 1:
        k = min(k, max(1, -(-int(remaining * share) // base)))
    return k


class _Request:
    """One client request being mined."""
    __slots__ = ("rid", "client", "data", "lower", "upper", "next_lower", "done", "retry",
                 "inflight", "best", "answered")

    def __init__(self, rid, client, msg):
        self.rid = rid
        self.client = client
        self.data = msg.Data
        self.lower = msg.Lower
        self.upper = msg.Upper
        self.next_lower = msg.Lower        # first nonce not yet handed out
        self.done = msg.Lower > msg.Upper  # every chunk issued
        self.retry = collections.deque()   # chunks of lost miners, issued first
        self.inflight = 0
        self.best = (U64_MAX, U64_MAX)     # miner.go:45-46 initial state
        self.answered = False

    def has_work(self):
        return bool(self.retry) or not self.done

    def finished(self):
        return not self.has_work() and self.inflight == 0

    def take(self, chunk):
        """Next chunk [lo, hi] (inclusive), at most `chunk` nonces.  A lost
        miner's chunk is re-issued first, cut to the taker's size (a fast
        miner's big job does not land whole on a slow one); its rest stays at
        the front of the queue."""
        if self.retry:
            lo, hi = self.retry.popleft()
            if hi - lo >= chunk:  # more than `chunk` nonces: the rest goes back first
                self.retry.appendleft((lo + chunk, hi))
                hi = lo + chunk - 1
            return lo, hi
        lo = self.next_lower
        hi = lo + chunk - 1 if self.upper - lo >= chunk else self.upper
        if hi == self.upper:
            self.done = True
        else:
            self.next_lower = hi + 1
        return lo, hi

    def merge(self, h, n):
        if (h, n) < self.best:
            self.best = (h, n)


class BitcoinServer:
    """Owns an ``lsp.Server``; ``serve()`` runs the event loop until the LSP
    server is closed (``close()`` from another thread ends it)."""

    def __init__(self, lsp_server, chunk=DEFAULT_CHUNK, depth=DEFAULT_DEPTH, log=None, target_ms=DEFAULT_TARGET_MS,
                 max_mult=DEFAULT_MAX_MULT, clock=time.monotonic):
        if chunk < 1 or depth < 1 or target_ms < 0 or max_mult < 1:
            raise ValueError("chunk, depth and max_mult must be >= 1, target_ms >= 0")
        self.srv = lsp_server
        self.chunk = int(chunk)
        self.depth = int(depth)
        self.target_s = target_ms / 1e3
        self.max_mult = int(max_mult)
        self.clock = clock
        self.log = log or (lambda *a: None)
        self.miners = {}                    # conn id -> deque of (request id, lo, hi, sent at) sent, oldest first
        self.rates = {}                     # conn id -> deque of its last jobs' rates (nonces/s)
        self._mult = {}                     # conn id -> multiple of its last fresh chunk
        self._last_done = {}                # conn id -> time of its last result
        self._free_since = {}               # conn id -> tick at which its job count last dropped
        self._tick = itertools.count()
        self.requests = collections.OrderedDict()  # rid -> _Request, oldest first
        self.client_reqs = collections.defaultdict(collections.deque)  # client -> rids, in arrival order
        self._rids = itertools.count(1)
        self.stats = collections.Counter()

    def idle_miners(self):
        """Miners with no job at all."""
        return [m for m, jobs in self.miners.items() if not jobs]

    # ---- event handling -------------------------------------------------
    def serve(self):
        while True:
            try:
                cid, payload = self.srv.Read()
            except lsp.LSPError as e:
                if e.conn_id == 0:
                    return  # server closed
                self._on_lost(e.conn_id)
                continue
            try:
                msg = Message.unmarshal(payload)
            except (ValueError, KeyError, TypeError):
                self.log(f"conn {cid}: bad message {payload!r}")
                continue
            self._on_message(cid, msg)

    def _on_message(self, cid, msg):
        if msg.Type == MsgType.Join:
            if cid not in self.miners:
                self.miners[cid] = collections.deque()
                self.rates[cid] = collections.deque(maxlen=RATE_SAMPLES)
                self._mult[cid] = 0
                self._last_done[cid] = None
                self._free_since[cid] = next(self._tick)
                self.stats["joins"] += 1
        elif msg.Type == MsgType.Request:
            if cid in self.miners:
                return  # a miner does not make requests
            r = _Request(next(self._rids), cid, msg)
            self.requests[r.rid] = r
            self.client_reqs[cid].append(r.rid)
            self.stats["requests"] += 1
            self._maybe_finish(r)
        elif msg.Type == MsgType.Result:
            jobs = self.miners.get(cid)
            if not jobs:
                return  # not a miner, or a miner with no job: stray
            # a miner answers its jobs in the order it got them (LSP delivers in order)
            rid, lo, hi, sent = jobs.popleft()
            self._free_since[cid] = next(self._tick)
            # its rate on this job: from when it could start it (sent, or
            # its previous result if that came later) to this result
            now = self.clock()
            prev = self._last_done.get(cid)
            start = sent if prev is None else max(sent, prev)
            self._last_done[cid] = now
            if now > start:
                self.rates[cid].append((hi - lo + 1) / (now - start))
            r = self.requests.get(rid)
            if r is not None:  # None: its client is gone, ignore (README:414)
                r.inflight -= 1
                r.merge(msg.Hash, msg.Nonce)
                self.stats["chunks_done"] += 1
                self._maybe_finish(r)
        self._schedule()

    def _on_lost(self, cid):
        if cid in self.miners:
            jobs = self.miners.pop(cid)
            self._free_since.pop(cid, None)
            for d in (self.rates, self._mult, self._last_done):
                d.pop(cid, None)
            self.stats["miners_lost"] += 1
            for rid, lo, hi, _sent in reversed(jobs):  # README:413: reassign, lowest chunk first
                r = self.requests.get(rid)
                if r is not None:
                    r.inflight -= 1
                    r.retry.appendleft((lo, hi))
                    self.stats["chunks_reassigned"] += 1
        elif cid in self.client_reqs:
            for rid in self.client_reqs.pop(cid):
                self.requests.pop(rid, None)  # README:414: stop working for it
            self.stats["clients_lost"] += 1
        self._schedule()

    # ---- scheduling -----------------------------------------------------
    def _pick(self):
        """Active request with the fewest chunks in flight (oldest on ties)."""
        best = None
        for r in self.requests.values():
            if r.has_work() and (best is None or r.inflight < best.inflight):
                best = r
        return best

    def _free_miner(self):
        """Miner with a free job slot: fewest queued jobs first, then the one
        whose count dropped longest ago."""
        best, key = None, None
        for m, jobs in self.miners.items():
            if len(jobs) < self.depth:
                k = (len(jobs), self._free_since[m])
                if key is None or k < key:
                    best, key = m, k
        return best

    def rate(self, mid):
        """The miner's measured rate (nonces/s): median of its last jobs, or None."""
        xs = sorted(self.rates.get(mid) or ())
        if not xs:
            return None
        m = len(xs) // 2
        return xs[m] if len(xs) % 2 else (xs[m - 1] + xs[m]) / 2

    def chunk_size(self, mid, r):
        """Nonces of miner mid's next fresh chunk of request r (chunk_for)."""
        rate = self.rate(mid)
        if self.target_s <= 0 or rate is None:
            k = 1
        else:
            known = [x for x in (self.rate(m) for m in self.miners) if x]
            total = sum(self.rate(m) or (sum(known) / len(known)) for m in self.miners)
            remaining = r.upper - r.next_lower + 1 if not r.done else 0
            k = chunk_for(self.chunk, self.target_s, self.max_mult, rate, self._mult.get(mid, 0), remaining,
                          rate / total if total > 0 else 1.0)
        self._mult[mid] = k
        return k * self.chunk

    def _schedule(self):
        while True:
            mid = self._free_miner()
            if mid is None:
                return
            r = self._pick()
            if r is None:
                return
            lo, hi = r.take(self.chunk_size(mid, r))
            try:
                self.srv.Write(mid, NewRequest(r.data, lo, hi).marshal())
            except lsp.LSPError:
                # miner already gone (server.go:177-179): put the chunk back,
                # and its queued jobs with it
                r.retry.appendleft((lo, hi))
                self._on_lost(mid)
                return
            self.miners[mid].append((r.rid, lo, hi, self.clock()))
            r.inflight += 1
            self.stats["chunks_sent"] += 1
            self.stats["nonces_sent"] += hi - lo + 1

    def _maybe_finish(self, r):
        if not r.finished():
            return
        r.answered = True
        q = self.client_reqs.get(r.client)
        # answer a client's requests in the order it sent them
        while q and self.requests[q[0]].answered:
            done = self.requests.pop(q.popleft())
            try:
                self.srv.Write(done.client, NewResult(*done.best).marshal())
                self.stats["results"] += 1
            except lsp.LSPError:
                pass  # client gone; its loss is reported by Read
        if q is not None and not q:
            self.client_reqs.pop(r.client, None)

    def close(self):
        try:
            self.srv.Close()
        except lsp.LSPError:
            pass


def main(argv=None):
    """``server <port>`` (README:365-368)."""
    ap = argparse.ArgumentParser(prog="server", description="bitcoin mining server (LSP)")
    ap.add_argument("port", type=int)
    ap.add_argument("--chunk", type=int, default=DEFAULT_CHUNK,
                    help="base nonces per miner job (default 2^32); jobs are multiples of it sized by each miner's rate")
    ap.add_argument("--target-ms", type=int, default=DEFAULT_TARGET_MS,
                    help="per-miner job time the sizing aims at (default 300 ms; 0: every job is one base chunk)")
    ap.add_argument("--max-mult", type=int, default=DEFAULT_MAX_MULT, help="largest job in base chunks (default 64)")
    ap.add_argument("--depth", type=int, default=DEFAULT_DEPTH,
                    help="jobs queued per miner (default 2: the next job is already there when one ends)")
    ap.add_argument("--epoch-limit", type=int, default=lsp.DefaultEpochLimit)
    ap.add_argument("--epoch-millis", type=int, default=lsp.DefaultEpochMillis)
    ap.add_argument("--window-size", type=int, default=lsp.DefaultWindowSize)
    ap.add_argument("-v", action="store_true", help="log to stderr")
    a = ap.parse_args(argv)
    params = lsp.Params(a.epoch_limit, a.epoch_millis, a.window_size)
    try:
        srv = lsp.NewServer(a.port, params)
    except lsp.LSPError as e:
        print(f"Failed to start server: {e}", file=sys.stderr)
        return 1
    log = (lambda *x: print(*x, file=sys.stderr, flush=True)) if a.v else None
    s = BitcoinServer(srv, chunk=a.chunk, depth=a.depth, log=log, target_ms=a.target_ms, max_mult=a.max_mult)
    try:
        s.serve()
    except KeyboardInterrupt:
        s.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
