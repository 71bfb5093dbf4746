"""Wire messages over the framed socket transport (flpytorch_amd/transport.py) on the MI355X:
flc_pack on the GPU -> CommSocket framing over a real socket -> host check (flc_payload_validate)
-> flc_unpack, bit for bit compressVector's output for every sparse and dense wire format; the
round harness with wire="socket" reproduces the reference runs; and the decode kernels stay inside
the row and the level table whatever bytes a malformed message holds."""
import ctypes

import numpy as np
import pytest
import torch

from tests.harness_cases import META, RUN_NAMES, check_history, simulation

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ag():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from flpytorch_amd import aggregation
    return aggregation


@pytest.mark.parametrize("spec", ["ident", "qsgd:127", "std.dithering:300:2", "natural", "randk:5%", "topk:5%",
                                  "bernulli:0.5", "terngrad"])
def test_payload_over_socket_decodes_bit_exact(ag, spec):
    from flpytorch_amd import transport
    d = 100_003
    x = torch.from_numpy(np.random.default_rng(3).standard_normal(d).astype(np.float32)).cuda()
    c = ag.initCompressor(spec, d)
    c.generateCompressPattern(np.random.RandomState(11), "cuda", 0, {})
    want = c.compressVector(x)
    msg = c.compressPayload(x)
    client, server = transport.socket_pair()
    import threading
    t = threading.Thread(target=client.sendPayload, args=(msg,))
    t.start()
    got_msg = server.recvPayload(c, d)
    t.join()
    assert bytes(got_msg.numpy()) == bytes(msg.cpu().numpy())
    assert server.bytes_received == client.bytes_sent == len(f"{msg.numel()}:") + msg.numel()
    got = c.decompressPayload(got_msg, d)                # host message: crosses to the device first
    assert torch.equal(got.view(torch.int32), want.view(torch.int32))


@pytest.mark.parametrize("name", [n for n in RUN_NAMES if META[n]["algorithm"] == "dcgd"])
def test_harness_socket_wire_reproduces_reference(ag, name):
    base = simulation(name, "cuda", record_iterates=True)
    base.run()
    sim = simulation(name, "cuda", record_iterates=True, wire="socket")
    H = sim.run()
    check_history(name, H, rel=1e-6)
    for a, b in zip(base.iterates, sim.iterates):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    client, server = sim.link
    per_msg = ag.initCompressor(META[name]["client_compressor"], META[name]["D"]).payloadBytes()
    n_msgs = sum(len(r["client_states"]) for r in H["history"].values()) * META[name]["local_iters"]
    assert server.bytes_received == client.bytes_sent == n_msgs * (per_msg + len(f"{per_msg}:"))


def _unpack_into_guarded(comp, payload_bytes, d):
    """flc_unpack of a (malformed) message into the first d floats of a d + 64 buffer of sentinels."""
    from flpytorch_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda")
    prm, keep = comp.codec_params(dev)
    p = torch.frombuffer(bytearray(payload_bytes), dtype=torch.uint8).to(dev)
    buf = torch.full((d + 64,), 7.0, dtype=torch.float32, device=dev)
    rc = lib.flc_unpack(ctypes.byref(prm), ctypes.c_void_p(p.data_ptr()), d, ctypes.c_void_p(buf.data_ptr()),
                        _lib.stream_ptr())
    assert rc == 0
    torch.cuda.synchronize()
    return buf.cpu().numpy()


def test_decode_kernels_stay_in_bounds(ag):
    import struct
    d = 50
    # sparse: an index just past the row (a wrong one inside the guard band) is dropped
    c = ag.initCompressor("randk:4", d)
    idx = np.array([1, d + 3, 0, 0], np.uint32).tobytes()
    val = np.array([2.5, 9.0, 0, 0], np.float32).tobytes()
    msg = struct.pack("<IIfI", 5, 2, 0.0, 0) + idx + val
    with pytest.raises(ValueError):
        c.validatePayload(msg)
    out = _unpack_into_guarded(c, msg, d)
    assert out[1] == 2.5 and np.count_nonzero(out[:d]) == 1 and np.all(out[d:] == 7.0)
    # Q8: level codes past s decode as the top level (levels[s] = 1), never past the table
    q = ag.initCompressor("qsgd:10", d)
    codes = bytes([0x7F, 0x80 | 0x7F, 0x80 | 10, 10]) + bytes(d - 4)
    msg = struct.pack("<IIfI", 2, d, 2.0, 0) + codes + bytes(16 - d % 16)
    with pytest.raises(ValueError):
        q.validatePayload(msg)
    out = _unpack_into_guarded(q, msg, d)
    assert list(out[:4]) == [2.0, -2.0, -2.0, 2.0] and np.all(out[d:] == 7.0)
    # a header claiming another format is decoded as the codec's own (no read past the Q8 body)
    msg = struct.pack("<IIfI", 1, d, 2.0, 0) + codes + bytes(16 - d % 16)
    out = _unpack_into_guarded(q, msg, d)
    assert list(out[:4]) == [2.0, -2.0, -2.0, 2.0] and np.all(out[d:] == 7.0)
