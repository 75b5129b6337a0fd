"""The Part B programs as processes, the way the reference's graders ran them
(README:476-488: start ./server, ./miner, ./client and match the client's
stdout).  CPU: server and client processes, with an in-test miner searching
with the CPU oracle.  The all-process run with a GPU miner process is in
tests/test_system_gpu.py."""
import os
import subprocess
import sys
import threading

import pytest

from conftest import ROOT
from distributed_bitcoin_minter_amd import lsp, lspnet, miner

PKG = "distributed_bitcoin_minter_amd"
FAST = ["--epoch-millis", "20", "--epoch-limit", "100"]


def free_udp_port():
    c = lspnet.listen(0)
    port = c.local_port()
    c.close()
    return port


def py(*args, **kw):
    return subprocess.Popen([sys.executable, "-m", *args], cwd=ROOT, stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True, **kw)


@pytest.mark.parametrize("prog", ["server", "miner", "client"])
def test_help(prog):
    p = py(f"{PKG}.{prog}", "--help")
    out, _ = p.communicate(timeout=60)
    assert p.returncode == 0 and "usage" in out.lower()


def test_server_and_client_processes(oracle):
    port = free_udp_port()
    srv = py(f"{PKG}.server", str(port), "--chunk", "1000", *FAST)
    try:
        class Searcher:  # stands in for the GPU miner (test infrastructure)
            def search(self, data, lo, hi):
                return oracle.search(data.encode(), lo, hi)

        p = lsp.Params(EpochLimit=100, EpochMillis=20, WindowSize=1)
        t = threading.Thread(target=miner.run, args=(f"127.0.0.1:{port}", p), kwargs={"searcher": Searcher()},
                             daemon=True)
        t.start()
        cl = py(f"{PKG}.client", f"127.0.0.1:{port}", "bradfitz", "9999", *FAST)
        out, err = cl.communicate(timeout=60)
        assert cl.returncode == 0, err
        assert out == "Result 1419516646206828 9898\n"  # C1 (README:395-401 format)
    finally:
        srv.terminate()
        srv.wait(timeout=30)


def test_client_process_disconnected():
    port = free_udp_port()  # nobody listens
    cl = py(f"{PKG}.client", f"127.0.0.1:{port}", "msg", "2", "--epoch-millis", "20", "--epoch-limit", "3")
    out, _ = cl.communicate(timeout=60)
    assert out == "Disconnected\n"


def test_miner_process_without_gpu_fails_loudly():
    """No CPU fallback: a miner on a host with no GPU exits non-zero
    before joining (BM_ENODEV)."""
    from distributed_bitcoin_minter_amd import _lib
    if _lib.device_count() > 0:
        pytest.skip("a GPU is present")
    m = py(f"{PKG}.miner", "127.0.0.1:9", *FAST, env=dict(os.environ))
    _, err = m.communicate(timeout=60)
    assert m.returncode != 0 and "no usable gfx950 device" in err


def test_client_rejects_max_nonce_go_would_reject():
    """maxNonce as strconv.ParseUint(s, 10, 64): ASCII digits only, at most
    2^64-1 (Python's int() alone would take spaces, a sign, underscores and
    other scripts' digits).  Leading zeros are fine, as in Go."""
    from distributed_bitcoin_minter_amd import client
    for bad in ("-1", "18446744073709551616", "12x", "", " 5", "+5", "5_0", "0x10", "٥",
                "9" * 21, "1" * 5000):  # past Python's 4300-digit int() limit too
        assert client.main(["127.0.0.1:1", "m", bad]) == 2, bad
    # in range with leading zeros (Go's ParseUint takes them): past the usage check
    import unittest.mock
    with unittest.mock.patch.object(client, "request", return_value=(1, 2)) as req:
        import io
        buf = io.StringIO()
        assert client.main(["127.0.0.1:1", "m", "0" * 4400 + "18446744073709551615"], out=buf) == 0
        assert req.call_args[0][2] == 2 ** 64 - 1 and buf.getvalue() == "Result 1 2\n"
