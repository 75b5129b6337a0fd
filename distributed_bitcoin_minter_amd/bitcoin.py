"""Mirror of the reference's `bitcoin` package (project2/bitcoin/).

* ``Hash(msg, nonce)``  -- bitcoin/hash.go:11-15, computed on the GPU
  (bm_hash_gpu).  "Only miners should ever need to call this method"
  (hash.go:9-10): the miner's search itself goes through
  ``miner.Miner.search`` / bm_search_gpu, never through per-nonce Hash calls.
* ``MsgType``, ``Message``, ``NewRequest``, ``NewResult``, ``NewJoin`` and
  ``Message.String`` -- bitcoin/message.go:5-60.  Messages marshal to the
  same JSON as Go's encoding/json does for the Go struct (field names
  Type/Data/Lower/Upper/Hash/Nonce, integers as JSON numbers), so they can
  ride in LSP payloads next to Go components.
"""
import enum
import json
import re
from dataclasses import dataclass

from . import _lib

U64_MAX = (1 << 64) - 1

_default_ctx = None


def _ctx():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = _lib.Context(num_gpus=1)
    return _default_ctx


def _as_bytes(msg) -> bytes:
    # Go's "%s" prints a string's raw bytes; a Python str is taken as UTF-8,
    # with the raw bytes of a surrogateescape-decoded str (argv) restored.
    return msg.encode("utf-8", "surrogateescape") if isinstance(msg, str) else bytes(msg)


_SURROGATE = re.compile("[\ud800-\udfff]")


def _go_decoded(s: str) -> str:
    """What Go's json.Unmarshal leaves in a string: "invalid UTF-8 or invalid
    UTF-16 surrogate pairs are not treated as an error. Instead, they are
    replaced by the Unicode replacement character U+FFFD."  Here an invalid
    raw byte arrives as a surrogateescape surrogate (one per byte, as Go's
    utf8.DecodeRune yields one RuneError per byte) and a lone \\uD8xx escape
    as a lone surrogate: both become U+FFFD."""
    return _SURROGATE.sub("\ufffd", s)


def Hash(msg, nonce: int) -> int:
    """bitcoin.Hash (hash.go:11-15): big-endian first 8 bytes of
    SHA-256(fmt.Sprintf("%s %d", msg, nonce)).  Runs on the GPU."""
    if not 0 <= nonce <= U64_MAX:
        raise ValueError("nonce must be a uint64")
    return _ctx().hash_many(_as_bytes(msg), [nonce])[0]


def go_json_string(s: str) -> str:
    """encoding/json's string encoder with HTML escaping (json.Marshal's
    default): <, >, & and control characters as \\u00XX (\\n, \\r, \\t short
    forms), U+2028/U+2029 escaped, everything else raw UTF-8.  A lone
    surrogate (what an invalid UTF-8 byte decodes to here, surrogateescape)
    becomes the six characters \ufffd, which is what Go writes for each
    invalid byte (encode.go: utf8.RuneError of width 1); a valid U+FFFD in
    the string stays raw, as in Go."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"' or ch == "\\":
            out.append("\\" + ch)
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        elif 0xD800 <= o <= 0xDFFF:
            out.append("\\ufffd")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


class MsgType(enum.IntEnum):
    """message.go:5-11 (iota order)."""
    Join = 0
    Request = 1
    Result = 2


@dataclass
class Message:
    """message.go:16-21."""
    Type: MsgType
    Data: str = ""
    Lower: int = 0
    Upper: int = 0
    Hash: int = 0
    Nonce: int = 0

    def marshal(self) -> bytes:
        """json.Marshal of the Go struct (field order as declared)."""
        return ('{"Type":%d,"Data":%s,"Lower":%d,"Upper":%d,"Hash":%d,"Nonce":%d}' % (
            int(self.Type), go_json_string(self.Data), self.Lower, self.Upper, self.Hash, self.Nonce)).encode()

    @classmethod
    def unmarshal(cls, raw) -> "Message":
        """json.Unmarshal into a Message: absent (or null) fields keep zero
        values; a field of the wrong JSON type is an error, as in Go (Data a
        string; Type an int; Lower/Upper/Hash/Nonce integers in uint64 range,
        no floats, no booleans).  Anything else raises ValueError."""
        if isinstance(raw, (bytes, bytearray, memoryview)):
            # Go decodes the payload as UTF-8 without rejecting invalid bytes
            # inside strings (they become U+FFFD, _go_decoded); outside a
            # string they are a syntax error either way
            raw = bytes(raw).decode("utf-8", "surrogateescape")
        try:
            d = json.loads(raw)
        except RecursionError as e:
            raise ValueError(f"not a JSON message: {e!r}") from None
        if not isinstance(d, dict):
            raise ValueError("bitcoin message is not a JSON object")

        def num(f, lo, hi):
            v = d.get(f)
            if v is None:
                return 0
            if isinstance(v, bool) or not isinstance(v, int):
                raise ValueError(f"{f} is not an integer")
            if not lo <= v <= hi:
                raise ValueError(f"{f} out of range")
            return v

        data = d.get("Data")
        if data is None:
            data = ""
        if not isinstance(data, str):
            raise ValueError("Data is not a string")
        data = _go_decoded(data)
        return cls(Type=MsgType(num("Type", -(1 << 63), (1 << 63) - 1)), Data=data,
                   Lower=num("Lower", 0, U64_MAX), Upper=num("Upper", 0, U64_MAX),
                   Hash=num("Hash", 0, U64_MAX), Nonce=num("Nonce", 0, U64_MAX))

    def String(self) -> str:
        """message.go:49-60."""
        if self.Type == MsgType.Request:
            return f"[Request {self.Data} {self.Lower} {self.Upper}]"
        if self.Type == MsgType.Result:
            return f"[Result {self.Hash} {self.Nonce}]"
        if self.Type == MsgType.Join:
            return "[Join]"
        return ""

    __str__ = String


def NewRequest(data: str, lower: int, upper: int) -> Message:
    """message.go:25-32."""
    return Message(Type=MsgType.Request, Data=data, Lower=lower, Upper=upper)


def NewResult(hash_: int, nonce: int) -> Message:
    """message.go:36-42."""
    return Message(Type=MsgType.Result, Hash=hash_, Nonce=nonce)


def NewJoin() -> Message:
    """message.go:45-47."""
    return Message(Type=MsgType.Join)
