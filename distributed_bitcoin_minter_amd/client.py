"""Request client: ``client <host:port> <message> <maxNonce>``.

Reference: project2/bitcoin/client/client.go:14-83 and the spec,
project2/README.md:378-406.  It sends ``Request(message, 0, maxNonce)``
(client.go:33-36), waits for the server's ``Result`` (:42-50) and prints

    Result <minHash> <nonce>        (printResult, client.go:76-78)

or, if the connection to the server is lost (or cannot be made),

    Disconnected                    (printDisconnected, client.go:81-83)

and exits.  maxNonce is parsed as Go's strconv.ParseUint(s, 10, 64) would
(client.go:25 uses ParseInt; the spec's nonces are uint64).
"""
import argparse
import re
import sys

from . import lsp
from .bitcoin import Message, MsgType, NewRequest, U64_MAX


def request(hostport, message, max_nonce, params=None, lower=0):
    """Send one request and wait for its answer.  Returns (hash, nonce), or
    None when the connection is lost ("Disconnected")."""
    try:
        c = lsp.NewClient(hostport, params)
    except lsp.LSPError:
        return None
    try:
        c.Write(NewRequest(message, lower, max_nonce).marshal())
        while True:
            raw = c.Read()
            try:
                m = Message.unmarshal(raw)
            except (ValueError, KeyError, TypeError):
                continue
            if m.Type == MsgType.Result:
                return m.Hash, m.Nonce
    except lsp.LSPError:
        return None
    finally:
        try:
            c.Close()
        except lsp.LSPError:
            pass


def main(argv=None, out=None):
    out = out or sys.stdout
    ap = argparse.ArgumentParser(prog="client", description="bitcoin mining request client (LSP)")
    ap.add_argument("hostport")
    ap.add_argument("message")
    ap.add_argument("maxNonce")
    ap.add_argument("--epoch-limit", type=int, default=lsp.DefaultEpochLimit)
    ap.add_argument("--epoch-millis", type=int, default=lsp.DefaultEpochMillis)
    ap.add_argument("--window-size", type=int, default=lsp.DefaultWindowSize)
    a = ap.parse_args(argv)
    # strconv.ParseUint(s, 10, 64): ASCII digits only (no sign, spaces or
    # underscores, which Python's int() would take), at most 2^64-1 (leading
    # zeros allowed); more than 20 significant digits is out of range before
    # int() sees it (Python refuses > 4300-digit strings with ValueError)
    max_nonce = -1
    if re.fullmatch(r"[0-9]+", a.maxNonce, flags=re.ASCII):
        digits = a.maxNonce.lstrip("0") or "0"
        max_nonce = int(digits) if len(digits) <= 20 else -1
    if not 0 <= max_nonce <= U64_MAX:
        print(f"maxNonce must be an unsigned 64-bit integer, got {a.maxNonce!r}", file=sys.stderr)
        return 2
    params = lsp.Params(a.epoch_limit, a.epoch_millis, a.window_size)
    res = request(a.hostport, a.message, max_nonce, params)
    if res is None:
        print("Disconnected", file=out, flush=True)
    else:
        print("Result", res[0], res[1], file=out, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
