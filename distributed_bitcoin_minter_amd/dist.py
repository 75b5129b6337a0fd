"""Multi-process (one process per GPU) sharding of a nonce search.

The nonce range shards with no data exchange: rank r scans its contiguous
piece of [lower, upper] on its own GPU, and the only collective is one
all_gather of the 16-byte partial {hash, nonce} per rank, followed by a
lexicographic (hash, nonce) min, which equals the reference's sequential
strict-'<' scan (miner.go:59-65).  Inside one process the
same split is done by a multi-device bm_ctx with an RCCL allgather
(csrc/bm_api.hip).  With torch.distributed's "nccl" backend (RCCL on ROCm)
the gather runs over xGMI.  bench.py's torchrun ranks use the library's own
RCCL group instead (bm_ctx_create_rank, rendezvous.py), with no torch.
"""
import math

U64_MAX = (1 << 64) - 1


def split_range(lower: int, upper: int, n: int):
    """Contiguous near-equal inclusive pieces; mirrors bm::split_range
    (csrc/bm_plan.cpp).  Returns at most n pieces (fewer for short ranges)."""
    if lower > upper or n < 1:
        return []
    span = upper - lower
    n = min(n, span + 1)
    q, r = divmod(span, n)
    out, cur = [], lower
    for i in range(n):
        size_m1 = q if i <= r else q - 1
        out.append((cur, cur + size_m1))
        cur = cur + size_m1 + 1
    out[-1] = (out[-1][0], upper)
    return out


SHARE_SCALE = 65536  # the fastest slot's share (bm_api.hip kShareScale)


def slot_pieces(lower: int, upper: int, n: int, shares=None):
    """Exactly n inclusive pieces, None for an empty one; mirrors
    bm::slot_pieces (csrc/bm_plan.cpp), the library's partitioner.  shares
    None (or not n of them): split_range's near-equal pieces.  Else piece i
    holds [lower + B_i, lower + B_{i+1} - 1], B_i = count * (s_0 + ... +
    s_{i-1}) // sum(shares)."""
    if shares is None or len(shares) != n or lower > upper:
        p = split_range(lower, upper, n)
        return p + [None] * (n - len(p))
    count, total = upper - lower + 1, sum(shares)
    out, prefix, b0 = [], 0, 0
    for i, sh in enumerate(shares):
        prefix += sh
        b1 = count if i == n - 1 else count * prefix // total
        out.append((lower + b0, lower + b1 - 1) if b1 > b0 else None)
        b0 = b1
    return out


def shares_from_rates(rates):
    """Integer shares in proportion to measured rates (nonces per ms), the
    fastest slot getting SHARE_SCALE; the formula bm_ctx_set_balance uses, so
    every rank that gathered the same rates derives the same shares."""
    top = max(rates)
    return [max(1, math.floor(r / top * SHARE_SCALE + 0.5)) for r in rates]


def _median(xs):
    ys = sorted(xs)
    m = len(ys) // 2
    return ys[m] if len(ys) % 2 else (ys[m - 1] + ys[m]) / 2


def calibrated_rates(per_rank, bound=0.85, agree=0.02):
    """One rate per rank from the rates of its warmup steps (nonces per ms,
    each step after a process's first, which loads the code objects), robust
    to one transient step (a clock ramp or a late code-object load
    in the one step used before fixed a skewed split for every timed step):
      * each rank's rate is the median of its steps;
      * a rank below `bound` of the fastest rank is held at `bound` of it,
        unless two of its steps agree within `agree` that it really is that
        slow (a persistently slower GPU keeps its measured rate).
    Returns (rates, info): info["clamped"] lists the ranks held at the bound,
    info["spread"] each rank's (max - min) / max over its steps."""
    med = [_median(r) for r in per_rank]
    top = max(med)
    rates, clamped = [], []
    for i, (r, m) in enumerate(zip(per_rank, med)):
        if m < bound * top:
            low = sorted(x for x in r if x < bound * top)
            if not any(b - a <= agree * b for a, b in zip(low, low[1:])):
                m = bound * top
                clamped.append(i)
        rates.append(m)
    spread = [round((max(r) - min(r)) / max(r), 4) if max(r) > 0 else 0.0 for r in per_rank]
    return rates, {"clamped": clamped, "spread": spread}


def lex_min(pairs):
    """Lexicographic (hash, nonce) min; (2^64-1, 2^64-1) for no pairs."""
    best = (U64_MAX, U64_MAX)
    for p in pairs:
        if tuple(p) < best:
            best = tuple(p)
    return best


def rank_piece(lower: int, upper: int, rank: int, world: int, shares=None):
    """This rank's inclusive piece, or None if it is empty (a range shorter
    than world, or a tiny share)."""
    return slot_pieces(lower, upper, world, shares)[rank]


def combine(partial, device=None):
    """All-gather every rank's (hash, nonce) and return the global min.

    One collective of 2 x uint64 per rank: dist.all_gather_into_tensor on a
    uint64 tensor (RCCL when the process group is "nccl")."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    h, n = partial
    # two's-complement view: uint64 -> int64 bits survive the exchange
    def s64(x):
        return x - (1 << 64) if x >= 1 << 63 else x

    src = torch.tensor([s64(h), s64(n)], dtype=torch.int64, device=device)
    dst = torch.empty(2 * world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(dst, src)
    vals = [v & U64_MAX for v in dst.cpu().tolist()]
    return lex_min((vals[2 * i], vals[2 * i + 1]) for i in range(world))
