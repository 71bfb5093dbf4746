"""CPU tests of the framed payload transport (flpytorch_amd/transport.py) and the host-side
message check (Compressor.validatePayload -> flc_payload_validate): the CommSocket framing
(comm_socket.py:16-82: ``<len>:<bytes>``), refusal of malformed prefixes / lengths, and every
rule of the check on hand-built messages of each wire format (include/flcodec.h layouts).
No device work: the library is loaded, the check is host code."""
import socket
import struct

import numpy as np
import pytest

from flpytorch_amd import transport
from flpytorch_amd.aggregation import initCompressor

F32, Q8, Q16, NAT16, SPARSE = 1, 2, 3, 4, 5


def a16(b):
    return (b + 15) & ~15


def header(fmt, count, norm=1.0, bad=0):
    return struct.pack("<IIfI", fmt, count, norm, bad)


def dense_msg(fmt, d, body):
    raw = header(fmt, d) + body
    return raw + bytes(16 + a16(len(body)) - len(raw))


def sparse_msg(k, idx, val, count=None):
    cap = bytearray(a16(4 * k))
    cap[:4 * len(idx)] = np.asarray(idx, np.uint32).tobytes()
    vb = bytearray(a16(4 * k))
    vb[:4 * len(val)] = np.asarray(val, np.float32).tobytes()
    return header(SPARSE, len(idx) if count is None else count, 0.0) + bytes(cap) + bytes(vb)


def test_framing_is_commsocket():
    a, b = socket.socketpair()
    pa = transport.PayloadSocket(a)
    pa.rawSend(b"\x00\x01hello")
    pa.rawSendString("result_of_local_training")
    b.settimeout(5)
    data = b""
    while len(data) < len(b"7:\x00\x01hello24:result_of_local_training"):
        data += b.recv(4096)
    assert data == b"7:\x00\x01hello24:result_of_local_training"
    assert pa.bytes_sent == len(data)


def test_roundtrip_and_refusals():
    c, s = transport.socket_pair()
    c.rawSend(bytes(range(256)) * 40)
    assert bytes(s.rawRecv()) == bytes(range(256)) * 40
    c.rawSendString("non_local_training")
    assert s.rawRecvString() == "non_local_training"
    c.sock.sendall(b"12x:")
    with pytest.raises(ValueError, match="prefix"):
        s.rawRecv()
    c2, s2 = transport.socket_pair()
    c2.sock.sendall(b"999999999999:")
    with pytest.raises(ValueError, match="exceeds"):
        s2.rawRecv(max_bytes=1 << 20)
    c3, s3 = transport.socket_pair()
    c3.sock.sendall(b"123456789012345678901234:")
    with pytest.raises(ValueError, match="prefix"):
        s3.rawRecv()
    c4, s4 = transport.socket_pair()
    c4.sock.close()
    with pytest.raises(RuntimeError, match="broken"):
        s4.rawRecv()


def test_recv_payload_refuses_wrong_length_before_the_body():
    comp = initCompressor("qsgd:10", 100)
    c, s = transport.socket_pair()
    c.sock.sendall(b"64:")                        # the codec's message is 16 + 112 bytes
    with pytest.raises(ValueError, match="128"):
        s.recvPayload(comp)
    # the body was never read, so the stream is out of step: the receiver ends the connection
    with pytest.raises(RuntimeError, match="broken"):
        s.recvPayload(comp)


def test_refused_length_unblocks_a_large_pending_send():
    """A wrong-length message larger than the socket buffer: the receiver refuses it from the prefix
    and shuts the connection down, so the sender's sendall fails instead of blocking forever."""
    import threading
    comp = initCompressor("qsgd:10", 100)
    c, s = transport.socket_pair()
    big = np.zeros(64 << 20, np.uint8)
    err = []

    def send():
        try:
            c.rawSend(big)
        except OSError as e:
            err.append(e)
    t = threading.Thread(target=send, daemon=True)
    t.start()
    with pytest.raises(ValueError, match="128"):
        s.recvPayload(comp)
    t.join(timeout=30)
    assert not t.is_alive() and err


def test_validate_dense_formats():
    d = 37
    q = initCompressor("qsgd:10", d)
    q.validatePayload(dense_msg(Q8, d, bytes([0x80 | 10, 0, 5] + [1] * (d - 3))))
    for bad, why in [(dense_msg(Q8, d, bytes([11] + [0] * (d - 1))), "exceeds s"),
                     (dense_msg(Q16, d, bytes(2 * d)), "format"),
                     (header(Q8, d - 1) + bytes(a16(d)), "count"),
                     (header(Q8, d, bad=2) + bytes(a16(d)), "unrepresentable"),
                     (dense_msg(Q8, d, bytes(d))[:-16], "bytes")]:
        with pytest.raises(ValueError, match=why):
            q.validatePayload(bad)
    s300 = initCompressor("std.dithering:300:2", d)         # Q16: level codes up to s = 300
    codes = np.zeros(d, np.uint16)
    codes[0], codes[1] = 300 | 0x8000, 7
    s300.validatePayload(dense_msg(Q16, d, codes.tobytes()))
    codes[2] = 301
    with pytest.raises(ValueError, match="exceeds s"):
        s300.validatePayload(dense_msg(Q16, d, codes.tobytes()))
    nat = initCompressor("natural", d)
    nat.validatePayload(dense_msg(NAT16, d, np.full(d, 0x7FFF, np.uint16).tobytes()))
    ident = initCompressor("ident", d)
    ident.validatePayload(dense_msg(F32, d, np.ones(d, np.float32).tobytes()), d)
    with pytest.raises(ValueError, match="count"):
        ident.validatePayload(header(F32, d + 1) + bytes(a16(4 * d)), d)


@pytest.mark.parametrize("spec", ["randk:4", "topk:4"])
def test_validate_sparse(spec):
    d = 50
    c = initCompressor(spec, d)
    c.validatePayload(sparse_msg(4, [0, 7, 8, 49], [1, 2, 3, 4]))
    c.validatePayload(sparse_msg(4, [3], [1.5]))                 # fewer entries than K (zeros kept)
    c.validatePayload(sparse_msg(4, [], []))
    for msg, why in [(sparse_msg(4, [0, 7, 7, 9], [1] * 4), "ascending"),
                     (sparse_msg(4, [9, 7], [1] * 2), "ascending"),
                     (sparse_msg(4, [1, 50], [1] * 2), "ascending"),        # index == d
                     (sparse_msg(4, [1, 2], [1] * 2, count=5), "at most"),
                     (header(F32, 4) + bytes(32), "format")]:
        with pytest.raises(ValueError, match=why):
            c.validatePayload(msg)


def test_validate_accepts_tensors_and_arrays():
    import torch
    d = 20
    q = initCompressor("qsgd:4", d)
    msg = dense_msg(Q8, d, bytes([1, 2, 3, 4] * 5))
    q.validatePayload(np.frombuffer(msg, np.uint8))
    q.validatePayload(torch.frombuffer(bytearray(msg), dtype=torch.uint8))
    with pytest.raises(TypeError):
        q.validatePayload(torch.zeros(len(msg), dtype=torch.int32))
