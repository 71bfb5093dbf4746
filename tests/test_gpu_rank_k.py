"""GPU parity of the Rank-K codec (compressors.py:336-364) through flc_encode / flc_encode_reduce.

Rank-K is the one floating-point-contraction codec: a thin SVD (rocSOLVER) and a GEMM (rocBLAS)
against the reference's torch LAPACK path, so parity is stated to a tolerance on the error norm,
relative to the input norm (inputs whose spectra have a gap at K, where U_K S_K Vt_K is unique):
"""
import numpy as np
import pytest
import torch

from oracle import codecs as oc
from tests.golden_io import load

pytestmark = pytest.mark.gpu

RANK_K_RTOL = 5e-5          # ||gpu - ref|| <= RANK_K_RTOL * ||x||   (fp32 SVD, rocSOLVER vs LAPACK)
RK_META, RK = load("rank_k")


@pytest.fixture(scope="module")
def ag():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from flpytorch_amd import aggregation
    return aggregation


def rel_err(got, want, x):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else got
    return float(np.linalg.norm(got.astype(np.float64) - want)) / max(float(np.linalg.norm(x)), 1e-30)


def low_rank(g, A, B, r, noise):
    u = g.standard_normal((A, r)) * np.linspace(3.0, 1.0, r)
    return ((u @ g.standard_normal((r, B))) + noise * g.standard_normal((A, B))).astype(np.float32).reshape(-1)


@pytest.mark.parametrize("i", range(len(RK_META)), ids=[f"{m['spec']}-{m['D']}" for m in RK_META])
def test_rank_k_golden(ag, i):
    m = RK_META[i]
    x, want = RK[f"x{i}"], RK[f"y{i}"]
    c = ag.initCompressor(m["spec"], m["D"])
    assert (c.A, c.B, c.K) == (m["A"], m["B"], m["K"])
    got = c.compressVector(torch.from_numpy(x.copy()).cuda())
    assert got.dtype == torch.float32 and got.shape == (m["D"],)
    assert torch.isfinite(got).all()
    err = rel_err(got, want, x)
    assert err <= RANK_K_RTOL, err
    assert c.last_need_to_send_advance == m["need"]
    assert c.last_input_advance == m["D"]


@pytest.mark.parametrize("n,A,B,K,r", [(5, 200, 150, 2, 2), (3, 85, 29, 3, 3), (4, 64, 64, 5, 3), (2, 1024, 1024, 16, 20),
                                       (3, 97, 1, 4, 1)])
def test_rank_k_encode_reduce_vs_oracle(ag, n, A, B, K, r):
    g = np.random.default_rng([n, A, B, K])
    d = A * B
    rows = np.stack([low_rank(g, A, B, r, 1e-3) for _ in range(n)])
    w = list(g.uniform(0.5, 2.0, n))
    enc = []
    for i in range(n):
        o = oc.OracleCompressor(f"rank_k:{K}", d)
        assert (o.A, o.B) == (A, B) or B == 1
        enc.append(o.compress(rows[i]))
    want = oc.reduce_plain(enc, w)
    red = ag.UplinkReducer(ag.initCompressor(f"rank_k:{K}", d))
    scale = sum(wi * float(np.linalg.norm(x)) for wi, x in zip(w, rows)) / sum(w)
    got = red(torch.from_numpy(rows).cuda(), weights=w)
    assert rel_err(got, want, np.array([scale])) <= RANK_K_RTOL
    rt = torch.from_numpy(rows).cuda()
    got2 = red([rt[i] for i in range(n)], weights=w)
    assert rel_err(got2, want, np.array([scale])) <= RANK_K_RTOL


def test_rank_k_full_rank_reproduces_input(ag):
    """K >= min(A, B): the full SVD reconstructs x to fp32 rounding."""
    g = np.random.default_rng(3)
    x = g.standard_normal(60 * 40).astype(np.float32)              # A = 48, B = 50
    c = ag.initCompressor("rank_k:100", x.size)
    assert min(c.A, c.B) == 48
    got = c.compressVector(torch.from_numpy(x).cuda())
    assert rel_err(got, x, x) <= RANK_K_RTOL


def test_rank_k_zero_input(ag):
    x = torch.zeros(4096, device="cuda")
    got = ag.initCompressor("rank_k:3", 4096).compressVector(x)
    assert torch.count_nonzero(got).item() == 0
