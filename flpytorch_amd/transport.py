"""Framed transport for wire messages between a remote client and the server.

The reference moves a remote client's work over ``CommSocket`` (comm_socket.py:16-82): each
message is ``<len>:<bytes>`` with the length in ASCII, and the bytes are a pickle of the whole
training result including the dense model (model_funcs.py:391-456 ``non_local_training``;
``pickle.loads`` of whatever the peer sent).  Here the same framing carries the codec's wire
message (``Compressor.compressPayload``: include/flcodec.h's 16-B header + body, e.g. 1 byte per
element for qsgd:127 instead of 4, 8 bytes per kept element for RandK / TopK), and the receiver
checks it against the codec before anything reaches the GPU (``flc_payload_validate``): exact
size, header format, count, level codes, ascending in-range sparse indices.  Nothing is unpickled.

``PayloadSocket`` keeps CommSocket's method names (``rawSend`` / ``rawRecv`` /
``rawSendString`` / ``rawRecvString``), so either end can be a CommSocket peer for framing.
"""
import socket

import numpy as np
import torch

_MAX_PREFIX = 20                        # digits of a length prefix (2**64 has 20)


class PayloadSocket:
    def __init__(self, sock=None):
        self.sock = sock if sock is not None else socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.settimeout(None)                                   # comm_socket.py:13-14
        self.bytes_sent = 0
        self.bytes_received = 0

    # -- framing (comm_socket.py:16-82) ---------------------------------------------------------
    def rawSend(self, msg):
        """Send ``<len>:<bytes>`` (bytes-like ``msg``)."""
        view = memoryview(msg).cast("B")
        head = f"{view.nbytes}:".encode("ascii")
        self.sock.sendall(head)
        self.sock.sendall(view)
        self.bytes_sent += len(head) + view.nbytes

    def rawSendString(self, msg):
        self.rawSend(msg.encode("utf-8"))

    def _recv_prefix(self):
        digits = bytearray()
        while True:
            ch = self.sock.recv(1)
            if ch == b"":
                raise RuntimeError("socket connection broken")
            if ch == b":":
                break
            if not ch.isdigit() or len(digits) >= _MAX_PREFIX:
                raise ValueError(f"malformed length prefix {bytes(digits + ch)!r}")
            digits += ch
        if not digits:
            raise ValueError("empty length prefix")
        self.bytes_received += len(digits) + 1
        return int(digits)

    def _recv_exact(self, n):
        buf = bytearray(n)
        view, got = memoryview(buf), 0
        while got < n:
            k = self.sock.recv_into(view[got:], n - got)
            if k == 0:
                raise RuntimeError("socket connection broken")
            got += k
        self.bytes_received += n
        return buf

    def rawRecv(self, max_bytes=1 << 30):
        """Receive one ``<len>:<bytes>`` message (refusing lengths above ``max_bytes``)."""
        n = self._recv_prefix()
        if n > max_bytes:
            raise ValueError(f"message of {n} bytes exceeds the {max_bytes}-byte limit")
        return self._recv_exact(n)

    def rawRecvString(self):
        return bytes(self.rawRecv()).decode("utf-8")

    def abort(self):
        """Shut the connection down in both directions (after a protocol error)."""
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass

    # -- wire messages ---------------------------------------------------------------------------
    def sendPayload(self, payload):
        """Send one wire message (a uint8 tensor on the GPU or the host, or bytes)."""
        if torch.is_tensor(payload):
            if payload.dtype != torch.uint8:
                raise TypeError("sendPayload: payload must be uint8")
            payload = payload.detach().reshape(-1).cpu().numpy()
        self.rawSend(payload)

    def recvPayload(self, compressor, d=None, device=None):
        """Receive one wire message for ``compressor`` (rows of ``d`` elements), check it
        (``validatePayload``: nothing malformed reaches the decode) and return it as a uint8
        tensor on ``device`` (host when None), ready for ``decompressPayload`` /
        ``PayloadReducer``.  The expected size is known up front: any other length is refused
        before the body is read."""
        want = compressor.payloadBytes(d)
        n = self._recv_prefix()
        if n != want:
            # the body is never read, so the stream is out of step: end the connection (the peer's
            # pending send fails instead of blocking on a full socket buffer)
            self.abort()
            raise ValueError(f"recvPayload: message of {n} bytes, the codec's payload is {want}")
        buf = self._recv_exact(n)
        compressor.validatePayload(buf, d)
        t = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8))
        return t if device is None else t.to(device)


def socket_pair():
    """Two connected PayloadSockets (client end, server end) on this host."""
    a, b = socket.socketpair()
    return PayloadSocket(a), PayloadSocket(b)
