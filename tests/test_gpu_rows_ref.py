"""The HIP codecs against the REAL reference at BASELINE.json's row sizes (C3: topk:1 % of
D = 10 M; C4: qsgd:127 at D = 25 M).  Fixtures: tests/golden/rows.{npz,json}, made by
tests/golden/make_golden_rows.py from the reference's own compressors.py (torch 2.10 CPU); inputs
are regenerated here from their seeds and checked against the recorded digests first.

Tolerances, stated per codec:
* TopK (compressors.py:330-335): the index set and the dense output are bit-identical (no ties at
  the K-th magnitude in these rows).
* QSGD (compressors.py:270-299):
  - given the reference's own norm, the whole 25 M-element output is bit-identical (digest);
  - the kernel's norm is the exactly rounded one; the reference's torch CPU fp32 norm is
    `pnorm_ulps_from_exact` ulps away (-14 616 at D = 25 M on normal rows: torch accumulates in
    fp32) — asserted to be exactly that distance;
  - with its own norm every nonzero output is `lev * sign * norm`, so it differs from the
    reference's by the norms' ratio: relative `4 rel + 4 ulp` where rel = |n_gpu / n_ref - 1|;
    decisions flip only where the uniform falls between the two probabilities, whose expected
    count is E = s * rel * ||x||_1 / ||x||_2 (the sum over elements of |dp| = s |x_j| rel / n);
    at most E + 5 sqrt(E) + 3 elements may fall outside the ratio tolerance.
"""
import hashlib
import json
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
META = json.load(open(os.path.join(HERE, "golden", "rows.json")))
ARR = np.load(os.path.join(HERE, "golden", "rows.npz"))
CASES = {m["name"]: m for m in META}


def row(seed, d, dist):
    # the generator of tests/golden/make_golden_rows.py
    g = np.random.default_rng(seed)
    x = g.standard_normal(d, dtype=np.float32)
    if dist == "heavy":
        x *= np.power(np.float32(10.0), g.uniform(-3.0, 3.0, d).astype(np.float32))
    return x


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:32]


@pytest.fixture(scope="module")
def ag():
    from flpytorch_amd import aggregation
    return aggregation


def bits(f):
    return int(np.float32(f).view(np.uint32))


@pytest.mark.parametrize("name", ["topk_c3", "topk_c3_heavy"])
def test_topk_row_size_vs_reference(ag, name):
    m = CASES[name]
    x = row(m["seed"], m["D"], m["dist"])
    assert sha(x) == m["x_sha"], "row regeneration differs from the fixture's"
    c = ag.initCompressor(m["spec"], m["D"])
    xd = torch.from_numpy(x).cuda()
    out = c.compressVector(xd)
    got = out.cpu().numpy()
    np.testing.assert_array_equal(np.flatnonzero(got), ARR[f"{name}_ind"])
    assert sha(got) == m["out_sha"]
    assert c.last_need_to_send_advance == m["need"]
    # the fused uplink selects the same set (one row, divisor 1: the output itself)
    red = ag.UplinkReducer(ag.initCompressor(m["spec"], m["D"]))
    fused = red(xd.view(1, -1)).cpu().numpy()
    assert sha(fused) == m["out_sha"]


@pytest.mark.parametrize("name", ["qsgd_c4", "qsgd_c4_heavy"])
def test_qsgd_row_size_vs_reference(ag, name):
    m = CASES[name]
    D, s = m["D"], 127
    x = row(m["seed"], D, m["dist"])
    assert sha(x) == m["x_sha"], "row regeneration differs from the fixture's"
    c = ag.initCompressor(m["spec"], D)
    c.generateCompressPattern(np.random.RandomState(m["pattern_seed"]), "cuda", 0, None)
    assert sha(c.testp.numpy()) == m["testp_sha"], "numpy-stream uniforms differ from the reference's"
    xd = torch.from_numpy(x).cuda()
    pref = np.uint32(m["pnorm_bits"]).view(np.float32)

    # (a) the reference's norm in: the whole output bit-identical to the reference's
    ref_out = c._encode_gpu(xd, pnorm_in=torch.tensor([pref], dtype=torch.float32, device="cuda")).cpu().numpy()
    assert sha(ref_out) == m["out_sha"]
    idx = ARR[f"{name}_idx"]
    np.testing.assert_array_equal(ref_out[idx].view(np.uint32), ARR[f"{name}_val"].view(np.uint32))

    # (b) the kernel's own norm: exactly rounded, at the recorded distance from torch's
    pno = torch.empty(1, device="cuda")
    own = c._encode_gpu(xd, pnorm_out=pno).cpu().numpy()
    assert bits(pno.item()) == m["exact_norm_bits"]
    assert bits(pno.item()) - m["pnorm_bits"] == -m["pnorm_ulps_from_exact"]
    rel = abs(float(pno.item()) / float(pref) - 1.0)
    tol = 4 * rel + 4 * 2.0 ** -24
    off = ~np.isclose(own, ref_out, rtol=tol, atol=0)
    E = s * rel * m["l1_over_l2"]
    bound = E + 5 * math.sqrt(E) + 3
    assert off.sum() <= bound, (int(off.sum()), bound)
    # every element outside the ratio tolerance is one level apart (a flipped decision)
    if off.any():
        lv = float(np.float32(1.0 / s))
        step = np.abs(own[off].astype(np.float64) / float(pno.item()) - ref_out[off].astype(np.float64) / float(pref))
        assert np.all(np.abs(step - lv) <= 1e-3 * lv)
    assert np.count_nonzero(own) == pytest.approx(m["nnz"], abs=bound)
    # the fused encode+reduce of the row (compat uniforms, divisor 1) is the own-norm output
    red = ag.UplinkReducer(ag.initCompressor(m["spec"], D))
    fused = red(xd.view(1, -1), uniforms=c.testp.cuda().view(1, -1)).cpu().numpy()
    np.testing.assert_array_equal(fused.view(np.uint32), own.view(np.uint32))


@pytest.mark.parametrize("name", ["qsgd_c4", "qsgd_c4_heavy"])
def test_qsgd_norm_mode_torch_cpu_vs_reference(ag, name):
    """VERDICT r04 missing 3: the reference's QSGD bits through the PUBLIC drop-in.  With
    Compressor.norm_mode = "torch_cpu", compressVector computes torch.norm(x, 2) in torch's CPU
    fp32 reduction order on the GPU (flc_norm2_torch_cpu) and encodes with it: the norm equals the
    reference's recorded bits and the whole 25 M-element output the reference's (digest and the
    sampled values), bit for bit — no private pnorm_in."""
    m = CASES[name]
    D = m["D"]
    x = row(m["seed"], D, m["dist"])
    assert sha(x) == m["x_sha"]
    c = ag.initCompressor(m["spec"], D)
    c.norm_mode = "torch_cpu"
    c.generateCompressPattern(np.random.RandomState(m["pattern_seed"]), "cuda", 0, None)
    xd = torch.from_numpy(x).cuda()
    assert bits(c.torchNorm(xd).item()) == m["pnorm_bits"]
    out = c.compressVector(xd).cpu().numpy()
    assert sha(out) == m["out_sha"]
    np.testing.assert_array_equal(out[ARR[f"{name}_idx"]].view(np.uint32), ARR[f"{name}_val"].view(np.uint32))
    assert c.last_need_to_send_advance == m["need"]
