"""GPU miner: the drop-in for the reference miner's job loop body.

Reference: project2/bitcoin/miner/miner.go:43-74 (``workWorkWorkWorkWork``):
read a JSON Request {Data, Lower, Upper}, scan the nonces keeping the
strict-'<' minimum of bitcoin.Hash starting from (2^64-1, 2^64-1)
(:45-46, :59-65), answer with JSON Result {Hash, Nonce} (:68-72).

Here the scan is one bm_search_gpu call.  The range is INCLUSIVE
[Lower, Upper] as the spec says (project2/README.md:329, "0 <= n <= N");
``exclusive_upper=True`` reproduces miner.go:59's literal ``i < Upper``.

``run(hostport)`` is the miner process (miner.go:20-41 + the job loop):
connect over LSP, send ``Join``, then answer every ``Request`` with a
``Result`` until the server is lost, at which point the miner shuts itself
down (README:412).  ``python -m distributed_bitcoin_minter_amd.miner
host:port`` is ``./miner host:port`` (README:370-374).
"""
import argparse
import sys

from . import _lib, lsp
from .bitcoin import Message, MsgType, NewJoin, NewResult, U64_MAX, _as_bytes


class Miner:
    """Owns a GPU context (one or more devices) and answers jobs."""

    def __init__(self, devices=None, num_gpus=1, exclusive_upper=False):
        self.ctx = _lib.Context(devices=devices, num_gpus=num_gpus)
        if self.ctx.num_devices() > 1:
            self.ctx.set_balance(True)  # pieces follow each GPU's measured rate (bm_ctx_set_balance)
        self.exclusive_upper = exclusive_upper

    def close(self):
        self.ctx.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def search(self, data, lower: int, upper: int):
        """min over nonces of (Hash(data, n), n); ties -> smallest nonce."""
        if not (0 <= lower <= U64_MAX and 0 <= upper <= U64_MAX):
            raise ValueError("bounds must be uint64")
        if self.exclusive_upper:
            if upper <= lower:
                return U64_MAX, U64_MAX
            upper -= 1
        return self.ctx.search(_as_bytes(data), lower, upper)

    def handle(self, job: Message) -> Message:
        """Request -> Result (miner.go:54-72)."""
        if job.Type != MsgType.Request:
            raise ValueError(f"miner expects a Request, got {job.Type!r}")
        h, n = self.search(job.Data, job.Lower, job.Upper)
        return NewResult(h, n)

    def handle_payload(self, payload: bytes) -> bytes:
        """JSON bytes in (an LSP payload), JSON bytes out."""
        return self.handle(Message.unmarshal(payload)).marshal()


def run(hostport, params=None, searcher=None, log=None):
    """The miner process body (miner.go:20-74).  ``searcher`` is anything
    with ``search(data, lower, upper) -> (hash, nonce)``; by default a GPU
    ``Miner`` over one device (created BEFORE connecting, so a host with no
    GPU fails loudly instead of joining and then failing every job).
    Returns the number of jobs answered once the server is gone."""
    log = log or (lambda *a: None)
    own = searcher is None
    if own:
        searcher = Miner()
    jobs = 0
    try:
        client = lsp.NewClient(hostport, params)  # miner.go:29-31
    except lsp.LSPError:
        if own:
            searcher.close()
        raise
    try:
        client.Write(NewJoin().marshal())         # miner.go:34-38
        while True:
            try:
                payload = client.Read()           # miner.go:49
            except lsp.LSPError:
                log("lost contact with the server: shutting down")  # README:412
                break
            try:
                job = Message.unmarshal(payload)
            except (ValueError, KeyError, TypeError):
                log(f"bad job {payload!r}")
                continue
            if job.Type != MsgType.Request:
                continue
            h, n = searcher.search(job.Data, job.Lower, job.Upper)
            try:
                client.Write(NewResult(h, n).marshal())  # miner.go:68-72
            except lsp.LSPError:
                break
            jobs += 1
    finally:
        try:
            client.Close()
        except lsp.LSPError:
            pass
        if own:
            searcher.close()
    return jobs


def main(argv=None):
    """``miner <host:port>`` (README:370-374)."""
    ap = argparse.ArgumentParser(prog="miner", description="GPU bitcoin miner (LSP client)")
    ap.add_argument("hostport")
    ap.add_argument("--device", type=int, default=None, help="GPU to use (default: 0)")
    ap.add_argument("--gpus", type=int, default=1, help="GPUs driven by this one miner (0 = all)")
    ap.add_argument("--epoch-limit", type=int, default=lsp.DefaultEpochLimit)
    ap.add_argument("--epoch-millis", type=int, default=lsp.DefaultEpochMillis)
    ap.add_argument("--window-size", type=int, default=lsp.DefaultWindowSize)
    ap.add_argument("-v", action="store_true", help="log to stderr")
    a = ap.parse_args(argv)
    params = lsp.Params(a.epoch_limit, a.epoch_millis, a.window_size)
    devices = [a.device] if a.device is not None else None
    log = (lambda *x: print(*x, file=sys.stderr, flush=True)) if a.v else None
    m = Miner(devices=devices, num_gpus=a.gpus)
    try:
        run(a.hostport, params, searcher=m, log=log)
    except lsp.LSPError as e:
        print(f"Failed to connect to {a.hostport}: {e}", file=sys.stderr)
        return 1
    finally:
        m.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
