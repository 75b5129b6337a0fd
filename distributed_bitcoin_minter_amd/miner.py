"""GPU miner: the drop-in for the reference miner's job loop body.

Reference: project2/bitcoin/miner/miner.go:43-74 (``workWorkWorkWorkWork``):
read a JSON Request {Data, Lower, Upper}, scan the nonces keeping the
strict-'<' minimum of bitcoin.Hash starting from (2^64-1, 2^64-1)
(:45-46, :59-65), answer with JSON Result {Hash, Nonce} (:68-72).

Here the scan is one bm_search_gpu call.  The range is INCLUSIVE
[Lower, Upper] as the spec says (project2/README.md:329, "0 <= n <= N");
``exclusive_upper=True`` reproduces miner.go:59's literal ``i < Upper``.
"""
from . import _lib
from .bitcoin import Message, MsgType, NewResult, U64_MAX, _as_bytes


class Miner:
    """Owns a GPU context (one or more devices) and answers jobs."""

    def __init__(self, devices=None, num_gpus=1, exclusive_upper=False):
        self.ctx = _lib.Context(devices=devices, num_gpus=num_gpus)
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
