"""GPU parity of the mixed per-client codec uplink (C5): each client against its constituent
codec's oracle under the group's device-RNG keys, combined in the stated group order."""
import numpy as np
import pytest
import torch

from oracle import codecs as oc
from oracle import devrng

pytestmark = pytest.mark.gpu

SPECS = ["randk:1%", "topk:1%", "qsgd:127"]


def bits(a):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else a
    return np.asarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("n,d,client0", [(7, 100003, 0), (12, 65536, 9), (3, 1 << 20, 3)])
def test_mixed_uplink_vs_oracle(n, d, client0):
    assert torch.cuda.is_available()
    from flpytorch_amd import _lib
    from flpytorch_amd.aggregation import MixedUplink
    lib = _lib.load()
    g = np.random.default_rng([n, d])
    rows = (g.standard_normal((n, d)) * 10.0 ** g.uniform(-1, 1, (n, 1))).astype(np.float32)
    up = MixedUplink(SPECS, d, seed=4242)
    G = len(SPECS)
    parts = []
    for gi, spec in enumerate(SPECS):
        acc = None
        for j, i in enumerate(range(gi, n, G)):
            cn = client0 // G + j
            o = oc.OracleCompressor(spec, d)
            if o.type == oc.RANDK:
                idx = np.empty(o.K, dtype=np.int64)
                assert lib.flc_device_randk_indices(up.seeds[gi], cn, d, o.K, idx.ctypes.data) == 0
                o.S = idx
            elif o.type == oc.STD_DITHERING:
                o.testp = devrng.uniforms(up.seeds[gi], cn, d)
            e = o.compress(rows[i])
            acc = e.copy() if acc is None else acc + e
        parts.append(acc if acc is not None else np.zeros(d, np.float32))
    want = parts[0].copy()
    for p in parts[1:]:
        want = want + p
    want = want / np.float32(n)
    t = torch.from_numpy(rows).cuda()
    got = up([t[i] for i in range(n)], client0=client0)
    assert np.array_equal(bits(got), bits(want))
    got2 = up(t, client0=client0)            # matrix rows: same bits
    assert np.array_equal(bits(got2), bits(want))
