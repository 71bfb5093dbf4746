"""SURVEY §8b threading contract: the library is reentrant across host threads that use distinct
streams (the reference's worker threads call compressVector concurrently, worker_thread.py:60-64).
Eight threads, each on its own HIP stream, run every codec family at once; every result equals the
same call made alone."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SPECS = ["topk:1%", "qsgd:127", "randk:1%", "natural", "std.dithering:8:2", "rank_k:4", "qsgd:16", "ident"]


def test_concurrent_threads_distinct_streams():
    assert torch.cuda.is_available()
    from flpytorch_amd import aggregation as ag
    n, d = 6, 200003
    g = torch.Generator(device="cuda").manual_seed(3)
    rows = [torch.randn(n, d, generator=g, device="cuda") for _ in SPECS]

    def run(i, stream=None):
        red = ag.UplinkReducer(ag.initCompressor(SPECS[i], d), seed=100 + i)
        if stream is None:
            return red(rows[i]).clone()
        with torch.cuda.stream(stream):
            out = red(rows[i], stream=stream)
            c = ag.initCompressor(SPECS[i], d)
            c.device_rng = (100 + i, 0)
            one = c.compressVector(rows[i][0])
        stream.synchronize()
        return out.clone(), one.clone()

    want = [run(i) for i in range(len(SPECS))]
    want_one = []
    for i in range(len(SPECS)):
        c = ag.initCompressor(SPECS[i], d)
        c.device_rng = (100 + i, 0)
        want_one.append(c.compressVector(rows[i][0]).clone())
    torch.cuda.synchronize()
    got, errors = [None] * len(SPECS), []

    def worker(i):
        try:
            s = torch.cuda.Stream()
            for _ in range(3):
                got[i] = run(i, s)
        except Exception as e:          # surfaced below
            errors.append((i, repr(e)))
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(len(SPECS))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors
    for i, spec in enumerate(SPECS):
        out, one = got[i]
        if spec.startswith("rank_k"):
            assert (out - want[i]).norm().item() <= 1e-5 * (1 + want[i].norm().item())
        else:
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want[i].cpu().numpy().view(np.uint32)), spec
            assert np.array_equal(one.cpu().numpy().view(np.uint32), want_one[i].cpu().numpy().view(np.uint32)), spec


def test_one_thread_two_streams_interleaved():
    """ONE host thread queues TopK on stream A and QSGD on stream B back to back,
    several times, without synchronising in between, with row sizes that make the second call's
    workspace grow.  The scratch is per stream (_lib.WORKSPACE keyed by (device, stream)), so the
    two calls cannot share or free each other's workspace; each result is bit-exact vs the oracle
    (TopK: oracle encode + sequential fold; QSGD: compat uniforms, oracle encode)."""
    assert torch.cuda.is_available()
    from flpytorch_amd import aggregation as ag
    from oracle import codecs as oc
    from oracle.rng import OracleRandomState

    n = 4
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for d in (50_003, 300_007):                      # the second size grows both streams' scratch
        rng = np.random.default_rng([d, 11])
        rows = rng.standard_normal((n, d)).astype(np.float32)
        rt = torch.from_numpy(rows).cuda()
        want = {}
        uni = None
        for spec in ("topk:1%", "qsgd:127"):
            rs = OracleRandomState(7)
            enc, us = [], []
            for i in range(n):
                o = oc.OracleCompressor(spec, d)
                o.generate(rs)
                rs.randint31()
                enc.append(o.compress(rows[i]))
                if o.type == oc.STD_DITHERING:
                    us.append(o.testp)
            want[spec] = oc.reduce_plain(enc)
            if us:
                uni = torch.from_numpy(np.stack(us)).cuda()
        torch.cuda.synchronize()
        red_t = ag.UplinkReducer(ag.initCompressor("topk:1%", d))
        red_q = ag.UplinkReducer(ag.initCompressor("qsgd:127", d))
        outs = []
        for _ in range(3):
            with torch.cuda.stream(sa):
                ot = red_t(rt, stream=sa)
            with torch.cuda.stream(sb):
                oq = red_q(rt, uniforms=uni, stream=sb)
            outs.append((ot, oq))
        sa.synchronize()
        sb.synchronize()
        for ot, oq in outs:
            assert np.array_equal(ot.cpu().numpy().view(np.uint32), want["topk:1%"].view(np.uint32))
            assert np.array_equal(oq.cpu().numpy().view(np.uint32), want["qsgd:127"].view(np.uint32))


def test_resident_compressvector_threads_distinct_streams():
    """The register-resident lone TopK select (k_lone_resident) needs its whole grid on the chip at
    once; two of its grids running together could each hold part of it and wait for the other.  Its
    launches are serialised across streams (each waits for the previous one's completion event), so
    four host threads on four streams calling compressVector at once all finish, bit-exact vs the
    same call alone, with no barrier giving up (flag 1)."""
    from flpytorch_amd import aggregation as ag
    d = 4_000_003
    g = torch.Generator(device="cuda").manual_seed(5)
    xs = [torch.randn(d, generator=g, device="cuda") for _ in range(4)]
    want = [ag.initCompressor("topk:1%", d).compressVector(x).clone() for x in xs]
    torch.cuda.synchronize()
    got, errors = [None] * 4, []

    def worker(i):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                c = ag.initCompressor("topk:1%", d)
                outs = [c.compressVector(xs[i]) for _ in range(5)]
                f = int(ag.select_row_flags(c, 1, d)[0])
            s.synchronize()
            got[i] = ([o.clone() for o in outs], f)
        except Exception as e:          # surfaced below
            errors.append((i, repr(e)))
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors
    for i in range(4):
        outs, f = got[i]
        assert f & 16 and not f & 1, f"thread {i}: flags {f}"
        for o in outs:
            assert np.array_equal(o.cpu().numpy().view(np.uint32), want[i].cpu().numpy().view(np.uint32))


def test_workspace_keeps_a_bounded_number_of_streams():
    """the per-stream scratch is an LRU of _lib.Workspace.MAX_STREAMS streams —
    a pool that makes a stream per worker call does not keep one buffer per stream ever seen; the
    calls on every stream stay exact."""
    from flpytorch_amd import _lib
    from flpytorch_amd import aggregation as ag
    from oracle import codecs as oc
    d = 100_003
    x = torch.randn(d, generator=torch.Generator(device="cuda").manual_seed(2), device="cuda")
    want = oc.OracleCompressor("topk:1%", d).compress(x.cpu().numpy())
    _lib.WORKSPACE.release()
    streams = [torch.cuda.Stream() for _ in range(_lib.Workspace.MAX_STREAMS + 8)]
    for s in streams:
        with torch.cuda.stream(s):
            got = ag.initCompressor("topk:1%", d).compressVector(x)
        s.synchronize()
        np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want.view(np.uint32))
    assert len(_lib.WORKSPACE._bufs) <= _lib.Workspace.MAX_STREAMS
