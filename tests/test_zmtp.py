"""Wire path: libgeeps' ZMTP/3.0 ROUTER transport
(geeps_amd/csrc/geeps/net.cpp) against a stock libzmq ROUTER socket.

The reference moves pushes and refreshes between ZeroMQ ROUTER sockets named
"client-<i>" and "tablet-<i>" (/root/reference/src/client/clientlib.cpp:107-120,
/root/reference/src/server/server-entry.cpp:56-68, router-handler.cpp:69-120),
one message being a multipart of its structs: CLOCK_WITH_UPDATES_BATCH
[header][RowKey x n][RowOpVal x n] (client/encoder-decoder.cpp:105-124) and
READ_ROW_BATCH [header][RowKey x n][RowData x n]
(server/server-encoder-decoder.cpp:228-250).  Here libzmq (the image's
/opt/conda/lib/libzmq.so.5, driven through ctypes) plays the reference's socket
and tests/apps/zmtp_peer plays libgeeps' end, in both directions.  CPU only.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os
import socket
import struct
import subprocess
import time

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ZMTP_PEER: another build of the same program, e.g. an ASan/UBSan one
PEER = os.environ.get("ZMTP_PEER") or os.path.join(REPO, "build", "tests", "zmtp_peer")

ZMQ_ROUTER, ZMQ_ROUTING_ID, ZMQ_SNDMORE, ZMQ_RCVMORE = 6, 5, 2, 13
ZMQ_LINGER, ZMQ_RCVTIMEO, ZMQ_SNDTIMEO, ZMQ_ROUTER_MANDATORY = 17, 27, 28, 33
W = 128
READ_ROW_BATCH, CLOCK_WITH_UPDATES_BATCH, SHUTDOWN = 1, 3, 6


def _libzmq():
    for cand in ("/opt/conda/lib/libzmq.so.5", ctypes.util.find_library("zmq")):
        if cand and (not cand.startswith("/") or os.path.exists(cand)):
            try:
                lib = ctypes.CDLL(cand)
            except OSError:
                continue
            lib.zmq_ctx_new.restype = ctypes.c_void_p
            lib.zmq_socket.restype = ctypes.c_void_p
            lib.zmq_socket.argtypes = [ctypes.c_void_p, ctypes.c_int]
            for f in ("zmq_bind", "zmq_connect"):
                getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_char_p]
            lib.zmq_setsockopt.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
            lib.zmq_send.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            lib.zmq_msg_init.argtypes = [ctypes.c_void_p]
            lib.zmq_msg_recv.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
            lib.zmq_msg_data.restype = ctypes.c_void_p
            lib.zmq_msg_data.argtypes = [ctypes.c_void_p]
            lib.zmq_msg_size.restype = ctypes.c_size_t
            lib.zmq_msg_size.argtypes = [ctypes.c_void_p]
            lib.zmq_msg_more.argtypes = [ctypes.c_void_p]
            lib.zmq_msg_gets.restype = ctypes.c_char_p
            lib.zmq_msg_gets.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
            lib.zmq_msg_close.argtypes = [ctypes.c_void_p]
            lib.zmq_close.argtypes = [ctypes.c_void_p]
            lib.zmq_ctx_term.argtypes = [ctypes.c_void_p]
            lib.zmq_strerror.restype = ctypes.c_char_p
            return lib
    return None


ZMQ = _libzmq()
pytestmark = [
    pytest.mark.skipif(ZMQ is None, reason="libzmq not in this image"),
    pytest.mark.skipif(not os.path.exists(PEER), reason="build/tests/zmtp_peer not built (build())"),
]


class Router:
    """A libzmq ROUTER socket: what the reference's RouterHandler holds."""

    def __init__(self, identity: bytes):
        self.ctx = ZMQ.zmq_ctx_new()
        self.s = ZMQ.zmq_socket(self.ctx, ZMQ_ROUTER)
        self._opt(ZMQ_ROUTING_ID, identity)
        self._int(ZMQ_LINGER, 0)
        self._int(ZMQ_RCVTIMEO, 20000)
        self._int(ZMQ_SNDTIMEO, 20000)
        self._int(ZMQ_ROUTER_MANDATORY, 1)  # an unknown peer is an error, not a silent drop

    def _opt(self, opt, val: bytes):
        assert ZMQ.zmq_setsockopt(self.s, opt, val, len(val)) == 0

    def _int(self, opt, v):
        c = ctypes.c_int(v)
        assert ZMQ.zmq_setsockopt(self.s, opt, ctypes.byref(c), 4) == 0

    def send(self, parts, retry_s=0.0):
        """ROUTER send: routing id first, then the message parts."""
        deadline = time.time() + retry_s
        while True:
            rc = ZMQ.zmq_send(self.s, parts[0], len(parts[0]), ZMQ_SNDMORE)
            if rc >= 0 or time.time() > deadline:
                break
            time.sleep(0.05)  # EHOSTUNREACH until the peer's handshake is in
        assert rc >= 0, ZMQ.zmq_strerror(ZMQ.zmq_errno())
        for i, p in enumerate(parts[1:]):
            flags = ZMQ_SNDMORE if i + 2 < len(parts) else 0
            buf = ctypes.create_string_buffer(bytes(p), len(p)) if len(p) else None
            assert ZMQ.zmq_send(self.s, buf, len(p), flags) == len(p)

    def recv(self, props=()):
        """One message: [routing id, part, ...] and the peer metadata asked for."""
        parts, meta = [], {}
        msg = ctypes.create_string_buffer(64)  # zmq_msg_t
        while True:
            ZMQ.zmq_msg_init(msg)
            n = ZMQ.zmq_msg_recv(msg, self.s, 0)
            assert n >= 0, ZMQ.zmq_strerror(ZMQ.zmq_errno())
            size = ZMQ.zmq_msg_size(msg)
            parts.append(ctypes.string_at(ZMQ.zmq_msg_data(msg), size) if size else b"")
            if len(parts) == 2:
                for p in props:
                    v = ZMQ.zmq_msg_gets(msg, p.encode())
                    meta[p] = v.decode() if v is not None else None
            more = ZMQ.zmq_msg_more(msg)
            ZMQ.zmq_msg_close(msg)
            if not more:
                return parts, meta

    def close(self):
        ZMQ.zmq_close(self.s)
        ZMQ.zmq_ctx_term(self.ctx)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def update_rows(n):
    """The peer's update rows: row i, element j = i*128 + j + 0.25."""
    return (np.arange(n * W, dtype=np.float64).reshape(n, W) + 0.25).astype(np.float32)


def keys(n):
    return np.array([(0, 1000 + i) for i in range(n)], dtype=np.uint64).reshape(n, 2)


@pytest.mark.parametrize("rows", [0, 1, 300])
def test_libgeeps_client_pushes_to_a_libzmq_tablet(rows):
    """libgeeps' client end -> a libzmq ROUTER named tablet-3: the push arrives
    as the reference decodes it (server-encoder-decoder.cpp:86-101), the
    client's READY properties are visible as message metadata, and a reply
    routed by identity reaches the client (which checks it)."""
    port = free_port()
    r = Router(b"tablet-3")
    assert ZMQ.zmq_bind(r.s, f"tcp://127.0.0.1:{port}".encode()) == 0
    p = subprocess.Popen([PEER, "client", str(port), "5", "3", str(rows)], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        parts, meta = r.recv(props=("Socket-Type", "Identity", "X-Geeps-Ipc", "X-Geeps-Pci-Bus-Id"))
        assert parts[0] == b"client-5"
        assert meta == {"Socket-Type": "ROUTER", "Identity": "client-5", "X-Geeps-Ipc": "0",
                        "X-Geeps-Pci-Bus-Id": "0000:00:00.0"}
        assert len(parts) == 4
        cmd, client_id, clock, table_id, _, _ = struct.unpack("<B3xIiIii", parts[1])
        assert (cmd, client_id, clock, table_id) == (CLOCK_WITH_UPDATES_BATCH, 5, 7, 0)
        np.testing.assert_array_equal(np.frombuffer(parts[2], np.uint64).reshape(-1, 2), keys(rows))
        vals = np.frombuffer(parts[3], np.float32).reshape(-1, W)
        np.testing.assert_array_equal(vals, update_rows(rows))
        hdr = struct.pack("<B3xIiiIi", READ_ROW_BATCH, 3, 7, 7, 0, 0)
        r.send([b"client-5", hdr, parts[2], (vals + vals).tobytes()])
        parts, _ = r.recv()  # the client's SHUTDOWN
        assert parts[0] == b"client-5" and parts[1][0] == SHUTDOWN
        out, err = p.communicate(timeout=30)
        assert p.returncode == 0, err
        assert "identity=tablet-3" in out and f"client ok rows={rows}" in out
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
        r.close()


@pytest.mark.parametrize("rows", [0, 2, 300])
def test_libzmq_client_pushes_to_a_libgeeps_tablet(rows):
    """A libzmq ROUTER named client-2 (the reference's client socket) connects
    to libgeeps' server end named tablet-4: its push is decoded, and the
    READ_ROW_BATCH reply comes back routed from tablet-4."""
    port = free_port()
    p = subprocess.Popen([PEER, "server", str(port), "4"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
    r = Router(b"client-2")
    try:
        assert p.stdout.readline().strip() == "listening"
        assert ZMQ.zmq_connect(r.s, f"tcp://127.0.0.1:{port}".encode()) == 0
        hdr = struct.pack("<B3xIiIii", CLOCK_WITH_UPDATES_BATCH, 2, 11, 0, 0, 0)
        vals = update_rows(rows)
        r.send([b"tablet-4", hdr, keys(rows).tobytes(), vals.tobytes()], retry_s=20)
        parts, _ = r.recv()
        assert parts[0] == b"tablet-4" and len(parts) == 4
        cmd, server_id, data_age, self_clock, table_id, _ = struct.unpack("<B3xIiiIi", parts[1])
        assert (cmd, server_id, data_age, self_clock, table_id) == (READ_ROW_BATCH, 4, 11, 11, 0)
        np.testing.assert_array_equal(np.frombuffer(parts[2], np.uint64).reshape(-1, 2), keys(rows))
        np.testing.assert_array_equal(np.frombuffer(parts[3], np.float32).reshape(-1, W), vals + vals)
        r.send([b"tablet-4", struct.pack("<B3xIiIi", SHUTDOWN, 2, 0, 0, 0)])
        out, err = p.communicate(timeout=30)
        assert p.returncode == 0, err
        assert "identity=client-2" in out and "prop Socket-Type=ROUTER" in out and "served=1" in out
    finally:
        r.close()
        if p.poll() is None:
            p.kill()
            p.wait()


def test_non_zmtp_peer_fails_the_handshake_loudly():
    """A peer that is not a ZMTP 3 endpoint ends the handshake with a message
    naming why (the product aborts with it; GP_CHECK_MSG in client_net.cpp)."""
    port = free_port()
    ls = socket.socket()
    ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    ls.bind(("127.0.0.1", port))
    ls.listen(1)
    p = subprocess.Popen([PEER, "client", str(port), "1", "0", "1"], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        c, _ = ls.accept()
        c.sendall(b"GPS1" + bytes(60))  # the old libgeeps framing's magic
        _, err = p.communicate(timeout=30)
        assert p.returncode != 0 and "ZMTP handshake: peer is not a ZMTP 2+ endpoint" in err
        c.close()
    finally:
        ls.close()
        if p.poll() is None:
            p.kill()
            p.wait()


def test_curve_mechanism_is_refused():
    """A greeting that asks for another security mechanism is refused by name."""
    port = free_port()
    ls = socket.socket()
    ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    ls.bind(("127.0.0.1", port))
    ls.listen(1)
    p = subprocess.Popen([PEER, "client", str(port), "1", "0", "1"], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        c, _ = ls.accept()
        greeting = b"\xff" + bytes(8) + b"\x7f" + b"\x03\x00" + b"CURVE".ljust(20, b"\0") + b"\x00" + bytes(31)
        c.sendall(greeting)
        _, err = p.communicate(timeout=30)
        assert p.returncode != 0 and "mechanism 'CURVE'" in err
        c.close()
    finally:
        ls.close()
        if p.poll() is None:
            p.kill()
            p.wait()


def test_silent_peer_times_out_the_handshake():
    """A peer that accepts and then says nothing fails the handshake after the
    time limit (libgeeps uses its connect timeout) instead of hanging."""
    port = free_port()
    ls = socket.socket()
    ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    ls.bind(("127.0.0.1", port))
    ls.listen(1)
    env = dict(os.environ, ZMTP_PEER_HANDSHAKE_S="1")
    t0 = time.time()
    p = subprocess.Popen([PEER, "client", str(port), "1", "0", "1"], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True, env=env)
    try:
        c, _ = ls.accept()
        _, err = p.communicate(timeout=30)
        assert p.returncode != 0 and "no greeting from the peer within 1 s" in err
        assert time.time() - t0 < 20
        c.close()
    finally:
        ls.close()
        if p.poll() is None:
            p.kill()
            p.wait()


ZMQ_DEALER = 5


def test_libzmq_dealer_client_and_a_large_push():
    """A ROUTER talks to DEALER peers too: a libzmq DEALER named client-6
    pushes a 20,000-row CLOCK_WITH_UPDATES_BATCH (10 MiB in one frame) to a
    libgeeps tablet-1 and gets the READ_ROW_BATCH back, no routing frames on
    the DEALER side."""
    port = free_port()
    rows = 20000
    p = subprocess.Popen([PEER, "server", str(port), "1"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
    r = Router(b"client-6")
    try:
        ZMQ.zmq_close(r.s)  # the same options on a DEALER socket instead
        r.s = ZMQ.zmq_socket(r.ctx, ZMQ_DEALER)
        r._opt(ZMQ_ROUTING_ID, b"client-6")
        r._int(ZMQ_LINGER, 0)
        r._int(ZMQ_RCVTIMEO, 20000)
        r._int(ZMQ_SNDTIMEO, 20000)
        assert p.stdout.readline().strip() == "listening"
        assert ZMQ.zmq_connect(r.s, f"tcp://127.0.0.1:{port}".encode()) == 0
        vals = update_rows(rows)
        hdr = struct.pack("<B3xIiIii", CLOCK_WITH_UPDATES_BATCH, 6, 3, 0, 0, 0)
        parts = [hdr, keys(rows).tobytes(), vals.tobytes()]
        for i, part in enumerate(parts):  # a DEALER sends the message parts only
            buf = ctypes.create_string_buffer(part, len(part))
            assert ZMQ.zmq_send(r.s, buf, len(part), ZMQ_SNDMORE if i + 1 < len(parts) else 0) == len(part)
        got, _ = r.recv()
        assert len(got) == 3
        cmd, server_id, data_age, _, table_id, _ = struct.unpack("<B3xIiiIi", got[0])
        assert (cmd, server_id, data_age, table_id) == (READ_ROW_BATCH, 1, 3, 0)
        np.testing.assert_array_equal(np.frombuffer(got[2], np.float32).reshape(-1, W), vals + vals)
        r.close()
        r = None
        out, err = p.communicate(timeout=30)  # the DEALER closed: the server reads EOF
        assert p.returncode == 0, err
        assert "prop Socket-Type=DEALER" in out and "served=1" in out
    finally:
        if r is not None:
            r.close()
        if p.poll() is None:
            p.kill()
            p.wait()


def test_incompatible_socket_type_is_refused():
    """A peer whose READY names a socket type a ROUTER cannot talk to (PUB) is
    refused by name."""
    port = free_port()
    ls = socket.socket()
    ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    ls.bind(("127.0.0.1", port))
    ls.listen(1)
    p = subprocess.Popen([PEER, "client", str(port), "1", "0", "1"], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        c, _ = ls.accept()
        greeting = b"\xff" + bytes(8) + b"\x7f" + b"\x03\x00" + b"NULL".ljust(20, b"\0") + b"\x00" + bytes(31)
        body = b"\x05READY" + b"\x0bSocket-Type" + struct.pack(">I", 3) + b"PUB"
        c.sendall(greeting + bytes([0x04, len(body)]) + body)
        _, err = p.communicate(timeout=30)
        assert p.returncode != 0 and "a ROUTER cannot talk to a 'PUB' socket" in err
        c.close()
    finally:
        ls.close()
        if p.poll() is None:
            p.kill()
            p.wait()


def test_chunked_send_and_receive_match_the_plain_forms():
    """send_frame_chunked / recv_frame_chunked (libgeeps' socket pushes and
    refreshes, sent and landed piece by piece) against send_frame /
    recv_frame over a socketpair: the same bytes on the wire, one ready() per
    piece in order, landed() pieces tiling every part (tests/apps/wire_chunks.cpp)."""
    exe = os.path.join(REPO, "build", "tests", "wire_chunks")
    assert os.path.exists(exe), "run __graft_entry__.build() first"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "wire_chunks ok" in r.stdout, r.stdout + r.stderr
