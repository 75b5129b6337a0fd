"""Live Sequence Protocol: reliable, windowed, epoch-driven messaging over UDP.

The transport the reference's miner, server and client talk over
(project2/README.md:67-239).  The API mirrors the Go package:

* ``Params`` (params.go:8-35): EpochLimit K = 5, EpochMillis d = 2000, WindowSize w = 1.
* ``Message`` (message.go:10-66): Connect / Data / Ack, with ConnID, SeqNum and
  Payload.  It marshals to the JSON Go's encoding/json produces: a nil
  ``[]byte`` is ``null``, any other payload is base64.
* ``NewClient(hostport, params) -> Client`` (client_api.go:6-30):
  ``ConnID``, ``Read``, ``Write``, ``Close``.
* ``NewServer(port, params) -> Server`` (server_api.go:6-39): ``Read``,
  ``Write``, ``CloseConn``, ``Close``.

Protocol rules, following README:67-138:
* Connection. A client sends (Connect, 0, 0); the server answers
  (Ack, id, 0), numbering ids from 1.  A repeated Connect from the same
  host:port gets the same id back.
* Sending. Data sequence numbers start at 1.  At most w messages may be
  unacknowledged: from the oldest unacked sequence number n, only n .. n+w-1
  may be sent.
* Receiving. Data inside [expected, expected+w) is buffered and delivered in
  order.  Every Data message at or below the window is acknowledged, duplicates
  included, so a lost Ack is repaired.
* Epochs. Every d ms an endpoint:
  * resends the Connect, or Ack 0 if no Data has arrived yet;
  * resends every unacknowledged Data;
  * re-acks the last w distinct Data messages it received.
  After K epochs with nothing received, the connection is declared lost.
* Closing. ``Close`` / ``CloseConn`` keep sending until every pending message
  is acknowledged, or the connection is lost.

Threads stand in for the Go goroutines: one socket reader and one epoch
timer per endpoint, with all state behind one lock.  No thread outlives
``Close``.
"""
import base64
import collections
import json
import socket
import threading
import time

from . import lspnet

MsgConnect, MsgData, MsgAck = 0, 1, 2  # message.go:8-13

DefaultEpochLimit = 5      # params.go:8-12
DefaultEpochMillis = 2000
DefaultWindowSize = 1


class Params:
    """params.go:15-35."""

    def __init__(self, EpochLimit=DefaultEpochLimit, EpochMillis=DefaultEpochMillis, WindowSize=DefaultWindowSize):
        self.EpochLimit = EpochLimit
        self.EpochMillis = EpochMillis
        self.WindowSize = WindowSize

    def String(self):
        return f"[EpochLimit: {self.EpochLimit}, EpochMillis: {self.EpochMillis}, WindowSize: {self.WindowSize}]"

    __str__ = String


def NewParams():
    return Params()


class Message:
    """message.go:16-66."""
    __slots__ = ("Type", "ConnID", "SeqNum", "Payload")

    def __init__(self, Type, ConnID=0, SeqNum=0, Payload=None):
        self.Type = Type
        self.ConnID = ConnID
        self.SeqNum = SeqNum
        self.Payload = Payload

    def marshal(self) -> bytes:
        p = None if self.Payload is None else base64.b64encode(self.Payload).decode()
        return json.dumps({"Type": self.Type, "ConnID": self.ConnID, "SeqNum": self.SeqNum, "Payload": p},
                          separators=(",", ":")).encode()

    @classmethod
    def unmarshal(cls, raw):
        """json.Unmarshal into a Message.  Anything that is not an object with
        integer Type/ConnID/SeqNum and a base64 (or null) Payload raises
        ValueError, so a stray datagram can never stop an endpoint's reader."""
        try:
            d = json.loads(raw)
        except (UnicodeDecodeError, RecursionError) as e:
            raise ValueError(f"not a JSON message: {e!r}") from None
        if not isinstance(d, dict):
            raise ValueError("LSP message is not a JSON object")
        vals = []
        for f in ("Type", "ConnID", "SeqNum"):
            v = d.get(f)
            if v is None:
                v = 0
            if isinstance(v, bool) or not isinstance(v, int) or not -(1 << 63) <= v < 1 << 63:
                raise ValueError(f"LSP field {f} is not an int")
            vals.append(v)
        p = d.get("Payload")
        if p is not None:
            if not isinstance(p, str):
                raise ValueError("LSP Payload is not a base64 string")
            p = base64.b64decode(p, validate=True)  # binascii.Error is a ValueError
        return cls(vals[0], vals[1], vals[2], p)

    def String(self):
        name = {MsgConnect: "Connect", MsgData: "Data", MsgAck: "Ack"}.get(self.Type, "")
        payload = " " + (self.Payload or b"").decode(errors="replace") if self.Type == MsgData else ""
        return f"[{name} {self.ConnID} {self.SeqNum}{payload}]"

    __str__ = String


def NewConnect():
    return Message(MsgConnect)


def NewData(connID, seqNum, payload):
    return Message(MsgData, connID, seqNum, bytes(payload))


def NewAck(connID, seqNum):
    return Message(MsgAck, connID, seqNum)


class LSPError(Exception):
    """A non-nil error of the Go API.  conn_id is the connection it concerns
    (0 for the server itself, server_api.go:13-17)."""

    def __init__(self, msg, conn_id=0):
        super().__init__(msg)
        self.conn_id = conn_id


def _next_tick(due, period):
    """The deadline after the tick that was due at `due`.  Like Go's
    time.Ticker, ticks missed while the process was descheduled are dropped,
    not fired back to back: a burst of K catch-up epochs would declare a
    connection lost that was silent for one stall, not for K epochs."""
    nxt = due + period
    now = time.monotonic()
    return nxt if nxt > now else now + period


def _drain(conn, handle, limit=4096):
    """Before an epoch counts silence, handle the datagrams already queued in
    the socket (lock held).  The reader thread may not have been scheduled
    for a while (GIL, a busy host); what waits unread was heard, and an epoch
    that ignored it could declare a live peer lost.  UDP hands each datagram
    to one reader, so the reader thread and this drain never both see one;
    the reordering between them is what LSP's sequence numbers absorb."""
    for _ in range(limit):
        try:
            got = conn.read_from(block=False)
        except OSError:
            return
        if got is None:
            return
        handle(*got)


class _Endpoint:
    """Protocol state of one end of one connection (no I/O of its own)."""

    def __init__(self, conn_id, params, send):
        self.id = conn_id
        self.w = max(1, params.WindowSize)
        self.k = max(1, params.EpochLimit)
        self.send = send
        self.next_seq = 1                         # next outgoing data sequence number
        self.pending = collections.deque()        # payloads waiting for the window
        self.unacked = collections.OrderedDict()  # seq -> Message, sent and not acked
        self.expect = 1                           # next in-order incoming seq
        self.ooo = {}                             # buffered out-of-order payloads
        self.recent = collections.deque(maxlen=self.w)  # last w distinct data seqs received
        self.got_data = False
        self.idle = 0                             # epochs since anything was received
        self.lost = False

    def _window_open(self):
        base = next(iter(self.unacked)) if self.unacked else self.next_seq
        return self.next_seq < base + self.w

    def pump(self):
        while self.pending and self._window_open():
            m = NewData(self.id, self.next_seq, self.pending.popleft())
            self.unacked[self.next_seq] = m
            self.next_seq += 1
            self.send(m)

    def write(self, payload):
        self.pending.append(bytes(payload))
        self.pump()

    def on_message(self, m):
        """Feed one received message; returns the payloads now deliverable."""
        self.idle = 0
        if m.Type == MsgAck:
            if m.SeqNum in self.unacked:
                del self.unacked[m.SeqNum]
                self.pump()
            return []
        if m.Type != MsgData or m.SeqNum < 1:
            return []
        s = m.SeqNum
        if s >= self.expect + self.w:
            return []  # beyond the receive window: the sender cannot be there, discard
        self.send(NewAck(self.id, s))
        if s not in self.recent:
            self.recent.append(s)
        self.got_data = True
        if s >= self.expect and s not in self.ooo:
            self.ooo[s] = m.Payload if m.Payload is not None else b""
        out = []
        while self.expect in self.ooo:
            out.append(self.ooo.pop(self.expect))
            self.expect += 1
        return out

    def on_epoch(self):
        """One epoch; returns True when the connection is (now) lost."""
        if self.lost:
            return True
        self.idle += 1
        if self.idle >= self.k:
            self.lost = True
            return True
        if not self.got_data:
            self.send(NewAck(self.id, 0))
        for m in list(self.unacked.values()):
            self.send(m)
        for s in list(self.recent):
            self.send(NewAck(self.id, s))
        return False

    def drained(self):
        return not self.pending and not self.unacked


class Client:
    """client_api.go:6-30.  Create with NewClient."""

    def __init__(self, conn, conn_id, params):
        self._conn = conn
        self._params = params
        self._lock = threading.Condition()
        self._ep = _Endpoint(conn_id, params, self._send)
        self._reads = collections.deque()
        self._closing = False
        self._stop = False
        self._threads = [threading.Thread(target=self._reader, daemon=True),
                         threading.Thread(target=self._epochs, daemon=True)]
        for t in self._threads:
            t.start()

    def _send(self, m):
        self._conn.write_to(m.marshal())

    def _reader(self):
        self._conn.settimeout(0.05)
        while not self._stop:
            try:
                data, _ = self._conn.read_from()
            except socket.timeout:
                continue
            except OSError:
                break
            with self._lock:
                self._handle(data)

    def _handle(self, data):  # lock held
        try:
            m = Message.unmarshal(data)
        except (ValueError, KeyError):
            return
        if m.ConnID != self._ep.id or self._ep.lost:
            return
        self._reads.extend(self._ep.on_message(m))
        self._lock.notify_all()

    def _epochs(self):
        period = self._params.EpochMillis / 1000.0
        nxt = time.monotonic() + period
        with self._lock:
            while not self._stop:
                left = nxt - time.monotonic()
                if left > 0:
                    self._lock.wait(timeout=left)  # woken early by other events: re-check the deadline
                    continue
                nxt = _next_tick(nxt, period)
                _drain(self._conn, lambda data, addr: self._handle(data))
                self._ep.on_epoch()
                self._lock.notify_all()

    def ConnID(self):
        return self._ep.id

    def Read(self):
        """Blocks for the next payload; LSPError once closed or lost with nothing left."""
        with self._lock:
            while not self._reads and not self._ep.lost and not self._closing:
                self._lock.wait()
            if self._reads:
                return self._reads.popleft()
            raise LSPError("connection lost" if self._ep.lost else "connection closed", self._ep.id)

    def Write(self, payload):
        """Non-blocking; LSPError only if the connection has been lost."""
        with self._lock:
            if self._ep.lost:
                raise LSPError("connection lost", self._ep.id)
            self._ep.write(payload)

    def Close(self):
        """Blocks until every pending message is acknowledged (or the
        connection is lost), then stops the background threads."""
        with self._lock:
            self._closing = True
            self._lock.notify_all()
            while not self._ep.drained() and not self._ep.lost:
                self._lock.wait(timeout=0.05)
            lost = self._ep.lost and not self._ep.drained()
            self._stop = True
            self._lock.notify_all()
        for t in self._threads:
            t.join()
        self._conn.close()
        if lost:
            raise LSPError("connection lost before pending messages were acknowledged", self._ep.id)


def NewClient(hostport, params=None):
    """Blocks until the server acknowledges the connection; LSPError after
    K epochs without an Ack (client_impl.go:52; README:111-138)."""
    params = params or NewParams()
    conn = lspnet.dial(hostport)
    period = params.EpochMillis / 1000.0
    conn.settimeout(period)
    connect = NewConnect().marshal()
    for _ in range(max(1, params.EpochLimit)):
        conn.write_to(connect)
        deadline = time.monotonic() + period
        while True:
            left = deadline - time.monotonic()
            if left <= 0:
                break
            conn.settimeout(left)
            try:
                data, _ = conn.read_from()
            except socket.timeout:
                break
            except OSError:
                conn.close()
                raise LSPError("cannot reach server")
            try:
                m = Message.unmarshal(data)
            except (ValueError, KeyError):
                continue
            if m.Type == MsgAck and m.SeqNum == 0 and m.ConnID > 0:
                return Client(conn, m.ConnID, params)
    conn.close()
    raise LSPError(f"could not connect to {hostport}")


class _ServerConn:
    def __init__(self, ep, addr):
        self.ep = ep
        self.addr = addr
        self.closing = False      # CloseConn / Close: finish sending, then drop
        self.user_closed = False  # CloseConn: deliver nothing more from it


class Server:
    """server_api.go:6-39.  Create with NewServer."""

    def __init__(self, conn, params):
        self._conn = conn
        self._params = params
        self.port = conn.local_port()
        self._lock = threading.Condition()
        self._conns = {}
        self._by_addr = {}
        self._next_id = 1
        self._reads = collections.deque()  # (conn_id, payload) or (conn_id, None) for an error
        self._closed = False
        self._stop = False
        self._lost_any = False
        self._threads = [threading.Thread(target=self._reader, daemon=True),
                         threading.Thread(target=self._epochs, daemon=True)]
        for t in self._threads:
            t.start()

    def _sender(self, addr):
        def send(m):
            self._conn.write_to(m.marshal(), addr)
        return send

    def _drop_if_done(self, cid):
        c = self._conns.get(cid)
        if c is not None and c.closing and c.ep.drained():
            self._forget(cid)

    def _forget(self, cid):
        c = self._conns.pop(cid, None)
        if c is not None:
            self._by_addr.pop(c.addr, None)

    def _reader(self):
        self._conn.settimeout(0.05)
        while not self._stop:
            try:
                data, addr = self._conn.read_from()
            except socket.timeout:
                continue
            except OSError:
                break
            with self._lock:
                self._handle(data, addr)

    def _handle(self, data, addr):  # lock held
        try:
            m = Message.unmarshal(data)
        except (ValueError, KeyError):
            return
        if m.Type == MsgConnect:
            cid = self._by_addr.get(addr)
            if cid is None:
                if self._closed:
                    return
                cid = self._next_id
                self._next_id += 1
                self._conns[cid] = _ServerConn(_Endpoint(cid, self._params, self._sender(addr)), addr)
                self._by_addr[addr] = cid
            self._conns[cid].ep.send(NewAck(cid, 0))  # a duplicate Connect gets the same id
            return
        c = self._conns.get(m.ConnID)
        if c is None or c.addr != addr or c.ep.lost:
            return
        out = c.ep.on_message(m)
        if not c.user_closed:
            self._reads.extend((m.ConnID, p) for p in out)
        self._drop_if_done(m.ConnID)
        self._lock.notify_all()

    def _epochs(self):
        period = self._params.EpochMillis / 1000.0
        nxt = time.monotonic() + period
        with self._lock:
            while not self._stop:
                left = nxt - time.monotonic()
                if left > 0:
                    self._lock.wait(timeout=left)
                    continue
                nxt = _next_tick(nxt, period)
                _drain(self._conn, self._handle)
                for cid, c in list(self._conns.items()):
                    if c.ep.on_epoch():
                        if not c.ep.drained():
                            self._lost_any = True
                        if not c.user_closed:
                            self._reads.append((cid, None))
                        self._forget(cid)
                    else:
                        self._drop_if_done(cid)
                self._lock.notify_all()

    def Read(self):
        """-> (conn_id, payload).  Raises LSPError(conn_id) when a client
        connection is lost, LSPError(conn_id=0) once the server is closed."""
        with self._lock:
            while not self._reads and not self._closed:
                self._lock.wait()
            if self._reads:
                cid, p = self._reads.popleft()
                if p is None:
                    raise LSPError(f"connection {cid} lost", cid)
                return cid, p
            raise LSPError("server closed", 0)

    def Write(self, connID, payload):
        """Non-blocking; LSPError if the connection does not exist or is lost."""
        with self._lock:
            c = self._conns.get(connID)
            if c is None or c.ep.lost or c.user_closed:
                raise LSPError(f"connection {connID} does not exist", connID)
            c.ep.write(payload)

    def CloseConn(self, connID):
        """Non-blocking: pending messages still go out; nothing more is read."""
        with self._lock:
            c = self._conns.get(connID)
            if c is None or c.user_closed:
                raise LSPError(f"connection {connID} does not exist", connID)
            c.user_closed = True
            c.closing = True
            self._reads = collections.deque(r for r in self._reads if r[0] != connID)
            self._drop_if_done(connID)

    def Close(self):
        """Blocks until every client's pending messages are acknowledged or
        that client is lost; LSPError if any was lost meanwhile."""
        with self._lock:
            self._closed = True
            for c in self._conns.values():
                c.closing = True
            self._lock.notify_all()
            while any(not c.ep.drained() and not c.ep.lost for c in self._conns.values()):
                self._lock.wait(timeout=0.05)
            self._stop = True
            self._lock.notify_all()
        for t in self._threads:
            t.join()
        self._conn.close()
        if self._lost_any:
            raise LSPError("a client was lost with messages pending", 0)


def NewServer(port, params=None):
    """Starts listening (port 0 = any free port, see Server.port) and returns
    without blocking (server_impl.go:48)."""
    params = params or NewParams()
    try:
        conn = lspnet.listen(port)
    except OSError as e:
        raise LSPError(f"cannot listen on port {port}: {e}")
    return Server(conn, params)
