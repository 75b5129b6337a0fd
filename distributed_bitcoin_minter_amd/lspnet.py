"""UDP shim with fault injection, mirroring the reference's lspnet package.

Reference: project2/lspnet/staff.go:7-82 (per-role read/write drop
percentages, package-global, atomic), conn.go:34-117 (reads/writes dropped
with probability p%, a 2,000-byte read buffer), net.go:14-88 (a global map
from connection to role: server or client).

Here a connection's role is fixed when it is created (``listen`` -> server,
``dial`` -> client).  Dropping is decided per packet with a module-level RNG
that tests may seed (``seed``), so a fault-injection run can be replayed.
"""
import os
import random
import socket
import threading

MAX_PACKET = 2000  # conn.go:35

_lock = threading.Lock()
_drop = {"client_read": 0, "client_write": 0, "server_read": 0, "server_write": 0}
_rng = random.Random()
_debug = False


def _set(key, p):
    if 0 <= p <= 100:
        with _lock:
            _drop[key] = int(p)


def SetClientReadDropPercent(p):  # staff.go:31-36
    _set("client_read", p)


def SetClientWriteDropPercent(p):  # staff.go:38-43
    _set("client_write", p)


def SetServerReadDropPercent(p):  # staff.go:45-50
    _set("server_read", p)


def SetServerWriteDropPercent(p):  # staff.go:52-57
    _set("server_write", p)


def SetReadDropPercent(p):  # staff.go:15-19
    SetClientReadDropPercent(p)
    SetServerReadDropPercent(p)


def SetWriteDropPercent(p):  # staff.go:21-25
    SetClientWriteDropPercent(p)
    SetServerWriteDropPercent(p)


def ResetDropPercent():  # staff.go:59-63
    SetReadDropPercent(0)
    SetWriteDropPercent(0)


def EnableDebugLogs(enable):  # conn.go:11-19
    global _debug
    _debug = bool(enable)


def seed(s):
    """Seed the drop RNG (the Go runtime seeds math/rand itself)."""
    with _lock:
        _rng.seed(s)


def _drop_it(key):
    with _lock:
        p = _drop[key]
        return p > 0 and _rng.randrange(100) < p  # conn.go:115-117


class UDPConn:
    """A UDP socket with lspnet's drop semantics for its role."""

    def __init__(self, sock, is_server, peer=None):
        # Always in timeout mode (CPython then keeps the fd O_NONBLOCK and
        # emulates blocking with poll), so a second handle on the same socket
        # can read without blocking: read_from(block=False) uses it, and
        # CPython's timeout path would first poll for up to the timeout.
        if sock.gettimeout() is None:
            sock.settimeout(3600.0)
        self._sock = sock
        self._nb = socket.socket(sock.family, sock.type, sock.proto, fileno=os.dup(sock.fileno()))
        self._nb.setblocking(False)
        self._server = is_server
        self._peer = peer
        self._closed = False

    @property
    def is_server(self):
        return self._server

    def local_port(self):
        return self._sock.getsockname()[1]

    def settimeout(self, t):
        self._sock.settimeout(t if t is not None else 3600.0)

    def read_from(self, block=True):
        """Next packet not dropped: (bytes, addr).  Raises socket.timeout /
        OSError; with block=False, None when nothing is queued."""
        key = "server_read" if self._server else "client_read"
        while True:
            try:
                data, addr = (self._sock if block else self._nb).recvfrom(MAX_PACKET)
            except (BlockingIOError, InterruptedError):
                return None
            except ConnectionRefusedError:
                # a connected client socket reports an earlier send's ICMP
                # port-unreachable here: for UDP that is only a lost packet
                continue
            if _drop_it(key):
                if _debug:
                    print(f"DROPPING read packet of length {len(data)}", flush=True)
                continue
            return data, addr

    def write_to(self, data, addr=None):
        """Send unless dropped.  Returns len(data) either way (conn.go:86-102)."""
        key = "server_write" if self._server else "client_write"
        if _drop_it(key):
            if _debug:
                print(f"DROPPING written packet of length {len(data)}", flush=True)
            return len(data)
        try:
            if addr is None:
                self._sock.send(data)
            else:
                self._sock.sendto(data, addr)
        except OSError:
            pass  # UDP: a send error is just a lost packet
        return len(data)

    def close(self):
        if not self._closed:
            self._closed = True
            self._nb.close()
            self._sock.close()


# Receive buffers.  One server socket takes every client's datagrams, and a
# Python reader that is descheduled for a few tens of ms (GC, a busy host) lets
# the kernel's default ~200 KB fill up: the overflow drops look like network
# loss and the retransmissions they trigger add load.  The kernel caps these
# at net.core.rmem_max.
SERVER_RCVBUF = 4 << 20
CLIENT_RCVBUF = 1 << 20


def _rcvbuf(s, n):
    try:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, n)
    except OSError:
        pass  # the default buffer still works


def listen(port, host="127.0.0.1"):
    """ListenUDP for a server (net.go:37-52).  port 0 picks a free port."""
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    _rcvbuf(s, SERVER_RCVBUF)
    s.bind((host, port))
    return UDPConn(s, True)


def dial(hostport):
    """DialUDP for a client (net.go:58-76)."""
    host, port = hostport.rsplit(":", 1)
    if host in ("", "localhost"):
        host = "127.0.0.1"
    peer = (socket.gethostbyname(host), int(port))
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    _rcvbuf(s, CLIENT_RCVBUF)
    s.bind(("0.0.0.0" if peer[0] != "127.0.0.1" else "127.0.0.1", 0))
    # connected, as Go's DialUDP: the kernel then delivers only the server's
    # datagrams, never a stale peer's that still targets a reused local port
    s.connect(peer)
    return UDPConn(s, False, peer)
