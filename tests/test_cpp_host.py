"""The C++ host side (include/btcminer.hpp, examples/bm_miner.cpp): the
reference's bitcoin messages (message.go:5-60) and the miner's job loop
(miner.go:20-74) over the C ABI.

CPU: Message::Marshal / Unmarshal agree with the Python mirror
(distributed_bitcoin_minter_amd/bitcoin.py, itself pinned to Go's
encoding/json form in tests/test_messages.py) on random messages and on the
malformed payloads both must reject; without a GPU the miner fails loudly.
GPU: Request lines in, Result lines out, equal to the oracle's scan."""
import json
import os
import random
import subprocess

import pytest

from conftest import ROOT, U64
from distributed_bitcoin_minter_amd.bitcoin import Message, MsgType, NewJoin, NewRequest, NewResult

EXE = os.path.join(ROOT, "examples", "bm_miner")
CLIENT = os.path.join(ROOT, "examples", "bm_client")
SERVER = os.path.join(ROOT, "examples", "bm_server")
_HDRS = [os.path.join(ROOT, "include", h) for h in ("btcminer.hpp", "btcminer.h", "bm_json.hpp", "lsp.hpp")]


def _build(exe, src, gpu_lib):
    """(Re)build an example when it is older than its sources (the same
    command line as __graft_entry__.build)."""
    if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(p) for p in [src] + _HDRS):
        cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-pthread", "-I", os.path.join(ROOT, "include"), src]
        if gpu_lib:
            cmd += ["-L", os.path.join(ROOT, "distributed_bitcoin_minter_amd"), "-lbtcminer",
                    "-Wl,-rpath,$ORIGIN/../distributed_bitcoin_minter_amd"]
        subprocess.check_call(cmd + ["-o", exe])
    return exe


def _exe():
    return _build(EXE, os.path.join(ROOT, "examples", "bm_miner.cpp"), True)


def _client():
    return _build(CLIENT, os.path.join(ROOT, "examples", "bm_client.cpp"), False)


def _server():
    return _build(SERVER, os.path.join(ROOT, "examples", "bm_server.cpp"), False)


def _selftest(lines):
    r = subprocess.run([_exe(), "--json-selftest"], input=b"".join(l + b"\n" for l in lines),
                       capture_output=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout.split(b"\n")[:len(lines)]


def _random_data(rng):
    alphabet = ["a", "Z", "0", " ", "<", ">", "&", '"', "\\", "/", "\n", "\r", "\t", "\x00", "\x1f", "\x7f",
                "é", "中", " ", " ", "�", "😀", "'"]
    return "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 24)))


def test_marshal_matches_python_mirror():
    rng = random.Random(0x5EED)
    msgs = [NewJoin(), NewRequest("msg", 0, 2), NewResult(4754799531757243342, 1), NewRequest("", U64, U64)]
    for _ in range(300):
        t = rng.choice(list(MsgType))
        msgs.append(Message(Type=t, Data=_random_data(rng), Lower=rng.randrange(1 << 64),
                            Upper=rng.randrange(1 << rng.randint(1, 64)), Hash=rng.randrange(1 << 64),
                            Nonce=rng.choice([0, U64, rng.randrange(1 << 64)])))
    wires = [m.marshal() for m in msgs]
    assert _selftest(wires) == wires


def test_unmarshal_accepts_what_python_accepts():
    """Other spellings of the same message (whitespace, field order, escapes,
    nulls, unknown fields) decode to what the Python mirror decodes, and
    re-marshal to the same Go-form bytes."""
    cases = [b' { "Upper" : 9 , "Type" : 1 , "Data" : "x\\u003cy" } ',
             b'{"Type":2,"Hash":5,"Extra":[1,{"x":null},"s",true,-1.5e3]}',
             b'{"Type":1,"Data":null,"Lower":null,"Upper":7}',
             b'{"Type":1,"Data":"\\ud83d\\ude00 \\/ \\b\\f","Upper":-0}',
             b'{"Type":1,"Data":"dup","Data":"last"}', b'{}', b'{"Type":0}',
             # invalid UTF-8 inside strings and lone surrogate escapes: U+FFFD, as Go's json.Unmarshal
             b'{"Type":1,"Data":"a\xffb\xed\xa0\x80c\\ud800d\\udc00","Upper":5}',
             b'{"Type":2,"X":"\xfe\xc0\xaf","Hash":3}', b'{"Type":1,"Data":"\xf4\x90\x80\x80\xe2\x82"}']
    got = _selftest(cases)
    for raw, out in zip(cases, got):
        assert out == Message.unmarshal(raw).marshal(), raw


def test_unmarshal_rejects_what_python_rejects():
    from test_messages import BAD_PAYLOADS
    extra = [b'{"Type":1,"Data":"a\tb"}', b'{"Type":1} x', b'{"Type":01}', b'{"Type":1,"Upper":18446744073709551616}',
             b'{"Type":1,"Data":"\\x"}', b'{"Type":1,}', b'{"Type":1,"Data":"x"}\xff', b'\xef\xbb\xbf{"Type":1}']
    bad = BAD_PAYLOADS + extra  # one message per line: none holds a newline
    for b in bad:
        with pytest.raises(ValueError):
            Message.unmarshal(b)
    assert all(out.startswith(b"error ") for out in _selftest(bad)), list(zip(bad, _selftest(bad)))


def test_miner_without_gpu_fails_loudly():
    from distributed_bitcoin_minter_amd import device_count
    if device_count() > 0:
        pytest.skip("a GPU is present")
    r = subprocess.run([_exe(), "--stdin"], input=NewRequest("bradfitz", 0, 9999).marshal() + b"\n", capture_output=True,
                       timeout=60)
    assert r.returncode == 2 and r.stdout.startswith(b"error -2 ")


@pytest.mark.gpu
def test_miner_job_loop_on_gpu(oracle):
    """Join first; each Request answered with the oracle's (hash, nonce);
    Join/Result lines and undecodable lines produce no output."""
    reqs = [("bradfitz", 0, 9999), ("msg", 0, 2), ("The quick brown fox jumps over the lazy dog. " * 2, 999_990_000,
            1_000_020_000), ("bradfitz", U64 - 3000, U64), ("x", 10, 9)]
    lines = [NewRequest(*q).marshal() for q in reqs[:2]] + [NewJoin().marshal(), b"garbage", NewResult(1, 2).marshal()]
    lines += [NewRequest(*q).marshal() for q in reqs[2:]]
    r = subprocess.run([_exe(), "--stdin"], input=b"".join(l + b"\n" for l in lines), capture_output=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout.split(b"\n")
    assert out[0] == NewJoin().marshal()
    want = [oracle.search(m.encode(), lo, hi, threads=8) if lo <= hi else (U64, U64) for m, lo, hi in reqs]
    assert [Message.unmarshal(o) for o in out[1:1 + len(reqs)]] == [NewResult(h, n) for h, n in want]
    assert b"bad job" in r.stderr
    # miner.go:59's exclusive upper
    r = subprocess.run([_exe(), "--stdin", "--exclusive-upper"], input=NewRequest("bradfitz", 0, 10000).marshal() + b"\n",
                       capture_output=True, timeout=60)
    assert Message.unmarshal(r.stdout.split(b"\n")[1]) == NewResult(*oracle.search_excl(b"bradfitz", 0, 10000))
