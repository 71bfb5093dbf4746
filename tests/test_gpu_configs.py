"""BASELINE configs C4 and C5 exercised at their own row sizes ("not exercised").

* C4 — qsgd:127, D = 25 M: the fused uplink (the sparse one-read path the bench runs) on 3 full
  rows against the oracle, BIT-EXACT, norms included.  The oracle's level loop is O(s D); above
  oc.LOOP_MAX_D it uses its closed form, pinned equal to the loop and to the reference's outputs by
  tests/test_oracle_golden.py.
* C5 — the mixed uplink (randk:1% / topk:1% / qsgd:127, one client per codec) at D = 10^8, through
  MixedUplink's per-codec partials (one row each: the partial IS that client's encode):
    RandK  the device-RNG index set (host mirror of the Feistel sampler), values (D/K) x bit-exact;
    TopK   exactly K survivors, equal to x, each >= every dropped |x|;
    QSGD   the norm exactly rounded (float64 reference), every value (levels[k] sign) norm for an
           integer level k, and 2^20 random elements bit-exact against the oracle's formula with the
           device draws restated in numpy (oracle/devrng.py).
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import codecs as oc
from oracle import devrng

pytestmark = pytest.mark.gpu

SEED = 20241015


@pytest.fixture(scope="module")
def ag():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from flpytorch_amd import aggregation
    return aggregation


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_c4_qsgd127_uplink_full_rows_vs_oracle(ag):
    from flpytorch_amd import _lib
    n, d, client0 = 3, 25_000_000, 1536
    gen = torch.Generator(device="cuda").manual_seed(44)
    rows = torch.empty((n, d), device="cuda").normal_(generator=gen)
    rows[1] *= torch.pow(10.0, torch.empty(d, device="cuda").uniform_(-3, 3, generator=gen))   # heavy-tailed
    rows[2, ::1000] = 0.0                                                                         # exact zeros
    red = ag.UplinkReducer(ag.initCompressor("qsgd:127", d), seed=SEED)
    pn = torch.empty(n, device="cuda")
    _lib.profile_enable(True)
    try:
        _lib.profile_collect("k_ds_filter")
        got = red(rows, client0=client0, pnorms_out=pn)
        torch.cuda.synchronize()
        assert _lib.profile_collect("k_ds_filter")[1] >= 1          # the bench's sparse path ran (tuning row groups: more)
    finally:
        _lib.profile_enable(False)
    got = got.cpu().numpy()
    host = rows.cpu().numpy()
    del rows
    acc, norms = None, []
    for i in range(n):
        o = oc.OracleCompressor("qsgd:127", d)
        o.testp = devrng.uniforms(SEED, client0 + i, d)
        e = o.compress(host[i])
        norms.append(o.norm(host[i]))
        o.testp = None
        acc = e if acc is None else acc + e                           # reduce_plain, unit weights
    want = acc / np.float32(n)
    assert np.array_equal(bits(pn.cpu().numpy()), bits(norms))
    assert np.array_equal(bits(got), bits(want))
    assert 0.01 < np.count_nonzero(got) / d < 0.1


def test_c5_mixed_uplink_properties_at_1e8(ag):
    from flpytorch_amd import _lib
    d = 100_000_000
    K = 1_000_000
    up = ag.MixedUplink(["randk:1%", "topk:1%", "qsgd:127"], d, seed=SEED, device="cuda")
    gen = torch.Generator(device="cuda").manual_seed(55)
    rows = torch.empty((3, d), device="cuda").normal_(generator=gen)
    parts, _ = up.partials([rows[0], rows[1], rows[2]], client0=0)
    torch.cuda.synchronize()

    # RandK (group 0, client number 0): the device index set, values (D/K) * x
    idx = np.empty(K, dtype=np.int64)
    assert _lib.load().flc_device_randk_indices(up.seeds[0], 0, d, K, idx.ctypes.data_as(ctypes.c_void_p)) == 0
    it = torch.from_numpy(idx).cuda()
    p0 = parts[0]
    assert torch.equal(torch.sort(torch.nonzero(p0).flatten()).values, torch.sort(it).values)
    assert torch.equal(p0[it].view(torch.int32), (np.float32(d / K).item() * rows[0][it]).view(torch.int32))

    # TopK (group 1): exactly K survivors, equal to x, none smaller than a dropped |x|
    p1, x1 = parts[1], rows[1]
    keep = p1 != 0
    assert int(keep.sum()) == K
    assert torch.equal(p1[keep].view(torch.int32), x1[keep].view(torch.int32))
    assert float(x1[keep].abs().min()) >= float(x1[~keep].abs().max())

    # QSGD (group 2): exact norm, values on the level lattice, a random subset bit-exact
    p2, x2 = parts[2], rows[2]
    norm = np.float32(torch.linalg.vector_norm(x2.double()).item())
    lv = torch.arange(0.0, 1.0 + 1.0 / 127 * 0.5, 1.0 / 127).cuda()       # compressors.py:87
    k = torch.clamp(torch.round(p2.abs() / float(norm) * 127), 0, 127).long()
    lattice = (lv[k] * torch.sign(p2)) * torch.tensor(norm, device="cuda")
    nz = p2 != 0                                    # (signed zeros: checked bit-exactly below)
    assert torch.equal(lattice[nz].view(torch.int32), p2[nz].view(torch.int32))
    assert 0.01 < float((p2 != 0).float().mean()) < 0.05
    j = np.sort(np.random.default_rng(3).choice(d, 1 << 20, replace=False))
    xj = x2[torch.from_numpy(j).cuda()].cpu().numpy()
    u = devrng.dev_u32(up.seeds[2], 0, j.astype(np.uint32)).astype(np.float64) * (1.0 / 4294967296.0)
    with np.errstate(all="ignore"):
        lev = oc.dither_levels(np.abs(xj) / norm, u, oc.OracleCompressor("qsgd:127", d).levels)
        lev[xj == 0.0] = 0.0
        want = lev * np.sign(xj) * norm
    got = p2[torch.from_numpy(j).cuda()].cpu().numpy()
    assert np.array_equal(bits(got), bits(want))
