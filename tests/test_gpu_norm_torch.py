"""flc_norm2_torch_cpu (the reference's torch.norm(x, p=2) on a CPU fp32 tensor, compressors.py:272)
against the oracle's C restatement (oracle/torch_norm.c, itself pinned against torch on the
development host by tests/test_host.py and against the reference's recorded norms at D = 25 M by
tests/test_oracle_golden.py): bit-exact for every length class (D % 8 tails, chunk boundaries of
the kernel's 8192-element staging), several rows with a leading dimension, zeros, subnormals,
huge values (overflow to inf), inf and NaN."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def oracle_norm(x):
    from oracle import rng  # noqa: F401  (builds oracle/_build on first use)
    lib = ctypes.CDLL(rng._LIB_PATH)
    lib.orc_torch_norm2.restype = ctypes.c_float
    lib.orc_torch_norm2.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    x = np.ascontiguousarray(x, dtype=np.float32)
    return np.float32(lib.orc_torch_norm2(x.ctypes.data, x.size))


def gpu_norms(rows_np, ld=None):
    from flpytorch_amd import _lib
    n, d = rows_np.shape
    ld = ld or d
    buf = torch.zeros(n * ld + 4, dtype=torch.float32, device="cuda")
    for i in range(n):
        buf[i * ld:i * ld + d] = torch.from_numpy(rows_np[i])
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    _lib.check(_lib.load().flc_norm2_torch_cpu(buf.data_ptr(), ld, n, d, out.data_ptr(), _lib.stream_ptr()),
               "flc_norm2_torch_cpu")
    return out.cpu().numpy()


@pytest.mark.parametrize("d", [1, 7, 8, 9, 63, 4097, 8191, 8192, 8193, 8200, 65543, 1_000_003])
def test_torch_norm_lengths(d):
    g = np.random.default_rng(d)
    rows = (g.standard_normal((3, d)) * 10.0 ** g.uniform(-3, 3, (3, d))).astype(np.float32)
    got = gpu_norms(rows, ld=d + 5)
    want = np.array([oracle_norm(r) for r in rows], dtype=np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_torch_norm_specials():
    d = 20_011
    g = np.random.default_rng(5)
    rows = g.standard_normal((6, d)).astype(np.float32)
    rows[0] = 0.0
    rows[1] = np.float32(1e-41)                 # subnormal squares underflow
    rows[2, ::3] = np.float32(3e19)             # squares overflow to inf
    rows[3, 17] = np.inf
    rows[4, 5000] = np.nan
    rows[5] = -rows[5]
    got = gpu_norms(rows)
    for i in range(6):
        w = oracle_norm(rows[i])
        if np.isnan(w):
            assert np.isnan(got[i])
        else:
            assert got[i].view(np.uint32) == w.view(np.uint32), i


def test_compressvector_norm_mode_torch_cpu():
    """compressVector with norm_mode='torch_cpu' equals the oracle's encode with the oracle's
    torch-order norm (compat uniforms), and norm_mode='exact' stays the default."""
    from flpytorch_amd import aggregation as ag
    from oracle import codecs as oc
    from oracle.rng import OracleRandomState
    d = 300_007
    x = np.random.default_rng(11).standard_normal(d).astype(np.float32)
    c = ag.initCompressor("qsgd:127", d)
    assert c.norm_mode == "exact"
    c.norm_mode = "torch_cpu"
    rs = np.random.RandomState(3)
    c.generateCompressPattern(rs, "cuda", 0, None)
    o = oc.OracleCompressor("qsgd:127", d)
    o.generate(OracleRandomState(3))
    want = o.compress(x, pnorm=oracle_norm(x))
    got = c.compressVector(torch.from_numpy(x).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("spec", ["nat.dithering:4:2", "nat.dithering:8:2", "std.dithering:16:2"])
def test_compressvector_norm_mode_torch_cpu_dithering_p2(spec):
    """natural dithering (compressors.py:301-329) takes torch.norm(x, p) as well and
    its output y * sign * pnorm carries the norm's bits, so norm_mode='torch_cpu' applies to it (p = 2)
    like to standard dithering: bit-exact against the oracle given the torch-order norm; and the
    natural dithering output differs from the exact-norm one exactly where the norms differ."""
    from flpytorch_amd import aggregation as ag
    from oracle import codecs as oc
    from oracle.rng import OracleRandomState
    d = 200_003
    x = np.random.default_rng(len(spec)).standard_normal(d).astype(np.float32)
    c = ag.initCompressor(spec, d)
    c.norm_mode = "torch_cpu"
    c.generateCompressPattern(np.random.RandomState(4), "cuda", 0, None)
    o = oc.OracleCompressor(spec, d)
    o.generate(OracleRandomState(4))
    want = o.compress(x, pnorm=oracle_norm(x))
    got = c.compressVector(torch.from_numpy(x).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_norm_mode_torch_cpu_p1_not_restated():
    from flpytorch_amd import aggregation as ag
    c = ag.initCompressor("nat.dithering:4:1", 1000)
    c.norm_mode = "torch_cpu"
    with pytest.raises(NotImplementedError):
        c.compressVector(torch.ones(1000, device="cuda"))
