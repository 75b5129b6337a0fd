"""The C++ LSP client (include/lsp.hpp) and the C++ miner / request client
programs built on it (examples/bm_miner.cpp, examples/bm_client.cpp).

CPU:
* wire bytes: against a raw UDP peer, the C++ client's Connect, Data and Ack
  datagrams are byte-identical to the Python mirror's (lsp.py, pinned to Go's
  encoding/json form of lsp.Message, message.go:16-22), and garbage datagrams
  are ignored;
* epochs (README:111-138): unacknowledged data is resent every epoch, and
  EpochLimit silent epochs end in "Disconnected" (client.go:81-83); a server
  that never answers the Connect gives the same;
* system: the C++ request client against the Python LSP server, the
  BitcoinServer scheduler and a miner whose searcher is the CPU oracle, with
  10% drops on every endpoint, prints the README:331-335 answers.
GPU: the C++ miner process (bm_miner host:port) joins the Python server and
answers clients' requests bit-exact with the oracle under 10% drops, then
shuts down once the server is gone (README:412)."""
import json
import os
import socket
import subprocess
import sys
import threading
import time

import pytest

from distributed_bitcoin_minter_amd import lsp, lspnet, miner
from distributed_bitcoin_minter_amd.bitcoin import Message, MsgType, NewJoin, NewRequest, NewResult, _as_bytes
from distributed_bitcoin_minter_amd.server import BitcoinServer
from conftest import ROOT
from test_cpp_host import _build, _client, _exe

KNOWN = [("bradfitz", 9999, "Result 1419516646206828 9898"), ("msg", 2, "Result 4754799531757243342 1")]


@pytest.fixture(autouse=True)
def _reset_drops():
    lspnet.ResetDropPercent()
    lspnet.seed(0x5EED)
    yield
    lspnet.ResetDropPercent()


class Peer:
    """A raw UDP endpoint standing in for the server."""

    def __init__(self):
        self.s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.s.bind(("127.0.0.1", 0))
        self.s.settimeout(10)
        self.port = self.s.getsockname()[1]
        self.addr = None

    def recv(self, want=None):
        """Next datagram (skipping those whose Type is not `want`)."""
        while True:
            data, self.addr = self.s.recvfrom(4096)
            if want is None or json.loads(data)["Type"] == want:
                return data

    def send(self, raw):
        self.s.sendto(raw, self.addr)

    def close(self):
        self.s.close()


def _run_client(port, msg, max_nonce, *extra):
    return subprocess.Popen([_client(), f"127.0.0.1:{port}", msg, str(max_nonce), *extra], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE)


def test_client_wire_bytes_match_python():
    peer = Peer()
    p = _run_client(peer.port, "bradfitz", 9999, "--epoch-millis", "100", "--epoch-limit", "50")
    try:
        assert peer.recv() == lsp.NewConnect().marshal()
        for junk in (b"garbage", b"null", b'{"Type":2,"ConnID":7,"SeqNum":0,"Payload":5}', b"\xff" * 3000):
            peer.send(junk)
        peer.send(lsp.NewAck(7, 0).marshal())
        req = NewRequest("bradfitz", 0, 9999).marshal()
        assert peer.recv(lsp.MsgData) == lsp.NewData(7, 1, req).marshal()
        peer.send(lsp.NewAck(7, 1).marshal())
        peer.send(lsp.NewData(7, 1, NewResult(1419516646206828, 9898).marshal()).marshal())
        while True:
            ack = peer.recv(lsp.MsgAck)
            if json.loads(ack)["SeqNum"] == 1:
                break
        assert ack == lsp.NewAck(7, 1).marshal()
        out, err = p.communicate(timeout=30)
        assert p.returncode == 0 and out == b"Result 1419516646206828 9898\n", err
    finally:
        if p.poll() is None:
            p.kill()
        peer.close()


@pytest.mark.parametrize("raw", [b"caf\xe9", b"a\xe2\x82b", b"\xed\xa0\x80x", b"\xc0\xaf", b"\xf4\x90\x80\x80",
                                 "\u00e9\u4e2d\U0001F600".encode()])
def test_client_request_bytes_for_non_utf8_messages(raw):
    """A message given as bytes that are not valid UTF-8 (a Go string can
    hold any bytes): the C++ client's Request is byte-identical to the Python
    mirror's, i.e. Go's encoding/json output (each invalid byte as \\ufffd,
    valid UTF-8 raw)."""
    peer = Peer()
    p = _run_client(peer.port, raw, 9, "--epoch-millis", "100", "--epoch-limit", "50")
    try:
        assert peer.recv() == lsp.NewConnect().marshal()
        peer.send(lsp.NewAck(7, 0).marshal())
        want = NewRequest(raw.decode("utf-8", "surrogateescape"), 0, 9).marshal()
        assert peer.recv(lsp.MsgData) == lsp.NewData(7, 1, want).marshal()
    finally:
        p.kill()
        p.communicate()
        peer.close()


def test_client_resends_each_epoch_then_disconnects():
    peer = Peer()
    t0 = time.monotonic()
    p = _run_client(peer.port, "x", 5, "--epoch-millis", "50", "--epoch-limit", "4")
    try:
        peer.recv(lsp.MsgConnect)
        peer.send(lsp.NewAck(3, 0).marshal())
        datas = [peer.recv(lsp.MsgData) for _ in range(3)]  # first send + resends, never acknowledged
        assert len(set(datas)) == 1 and Message.unmarshal(lsp.Message.unmarshal(datas[0]).Payload) == NewRequest("x", 0, 5)
        out, _ = p.communicate(timeout=30)
        assert out == b"Disconnected\n"
        assert time.monotonic() - t0 < 20
    finally:
        if p.poll() is None:
            p.kill()
        peer.close()


def test_client_no_answer_to_connect():
    peer = Peer()  # receives, never answers
    p = _run_client(peer.port, "x", 5, "--epoch-millis", "50", "--epoch-limit", "3")
    out, _ = p.communicate(timeout=30)
    peer.close()
    assert out == b"Disconnected\n"


def test_client_rejects_bad_max_nonce():
    for bad in ("-1", "18446744073709551616", "12x", "", " 5", "+5", "5_0", "0x10", "\u0665"):
        r = subprocess.run([_client(), "127.0.0.1:1", "m", bad], capture_output=True, timeout=30)
        assert r.returncode == 2, bad


class _OracleSearcher:
    def __init__(self, oracle):
        self.oracle = oracle

    def search(self, data, lower, upper):
        return self.oracle.search(_as_bytes(data), lower, upper)


def _start_server(p, chunk):
    srv = lsp.NewServer(0, p)
    bs = BitcoinServer(srv, chunk=chunk)
    t = threading.Thread(target=bs.serve, daemon=True)
    t.start()
    return srv, bs, t


@pytest.mark.parametrize("window", [1, 4])
def test_cpp_client_against_python_system_with_drops(oracle, window):
    p = lsp.Params(EpochLimit=200, EpochMillis=20, WindowSize=window)
    srv, bs, t = _start_server(p, 1000)
    m = threading.Thread(target=miner.run, args=(f"127.0.0.1:{srv.port}", p, _OracleSearcher(oracle)), daemon=True)
    m.start()
    lspnet.SetReadDropPercent(10)
    lspnet.SetWriteDropPercent(10)
    flags = ["--epoch-millis", "20", "--epoch-limit", "200", "--window-size", str(window), "--drop-read", "10",
             "--drop-write", "10"]
    procs = [(_run_client(srv.port, msg, n, *flags), want) for msg, n, want in KNOWN]
    try:
        for proc, want in procs:
            out, err = proc.communicate(timeout=120)
            assert out.decode() == want + "\n", err
    finally:
        for proc, _ in procs:
            if proc.poll() is None:
                proc.kill()
        lspnet.ResetDropPercent()
        bs.close()
        t.join(timeout=15)
        m.join(timeout=15)


def test_miner_without_gpu_fails_before_connecting():
    from distributed_bitcoin_minter_amd import device_count
    if device_count() > 0:
        pytest.skip("a GPU is present")
    peer = Peer()
    peer.s.settimeout(0.5)
    r = subprocess.run([_exe(), f"127.0.0.1:{peer.port}"], capture_output=True, timeout=60)
    assert r.returncode == 2 and r.stdout.startswith(b"error -2 ")
    with pytest.raises(socket.timeout):  # it never sent a Connect
        peer.recv()
    peer.close()


@pytest.mark.gpu
def test_cpp_gpu_miner_in_the_system(oracle):
    """Python LSP server + scheduler, two C++ GPU miner processes on device 0,
    C++ and Python clients, 10% drops everywhere."""
    from distributed_bitcoin_minter_amd import client
    p = lsp.Params(EpochLimit=200, EpochMillis=20, WindowSize=2)
    srv, bs, t = _start_server(p, 1 << 20)
    flags = ["--epoch-millis", "20", "--epoch-limit", "200", "--window-size", "2"]
    miners = [subprocess.Popen([_exe(), f"127.0.0.1:{srv.port}", "--device", "0", "-v", "--drop-read", "10",
                                "--drop-write", "10", *flags], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
              for _ in range(2)]
    cproc = []
    try:
        t0 = time.monotonic()
        while bs.stats["joins"] < 2:
            assert time.monotonic() - t0 < 60, [m.poll() for m in miners]
            time.sleep(0.01)
        lspnet.SetReadDropPercent(10)
        lspnet.SetWriteDropPercent(10)
        jobs = [("bradfitz", 9999), ("msg", 2), ("cpp-gpu-client", (1 << 24) + 12345), ("py-gpu-client", 3_000_000)]
        cproc = [_run_client(srv.port, msg, n, *flags, "--drop-read", "10", "--drop-write", "10")
                 for msg, n in jobs[:3]]
        py = client.request(f"127.0.0.1:{srv.port}", jobs[3][0], jobs[3][1], p)
        want = [oracle.search(m.encode(), 0, n, threads=8) for m, n in jobs]
        assert py == want[3]
        for proc, (h, n) in zip(cproc, want):
            out, err = proc.communicate(timeout=120)
            assert out.decode() == f"Result {h} {n}\n", err
    finally:
        for proc in cproc:
            if proc.poll() is None:
                proc.kill()
        lspnet.ResetDropPercent()
        bs.close()
        t.join(timeout=15)
    for m in miners:  # the server is gone: each miner shuts itself down (README:412)
        try:
            out, err = m.communicate(timeout=60)
        except subprocess.TimeoutExpired:
            m.kill()
            raise
        assert m.returncode == 0, err
        assert b"lost contact with the server" in err


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["C5"])
def test_c5_native_at_size(cfg):
    """BASELINE C5 at full size with every process native: the C++ server,
    4 C++ GPU miners on device 0, 16 C++ clients asking for [0, 2^34-1] of
    "client-%02d", 2^32-nonce jobs, 10% read and write drop at every endpoint
    (tools/bench_c5_native.py).  Every answer equals the full CPU scan of
    that client's range (tests/golden/c5_clients.json)."""
    import json
    _exe(), _client(), _build(os.path.join(ROOT, "examples", "bm_server"),
                              os.path.join(ROOT, "examples", "bm_server.cpp"), False)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_c5_native.py"), "--timeout", "200"],
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["all_answered"] and out["golden_ok"] and out["golden_checked"] == 16, out
    print(f"C5 native: {out['GHs']} GH/s end to end over {out['seconds']} s")
