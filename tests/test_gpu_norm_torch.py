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


def gpu_norms(rows_np, ld=None, parallel=False):
    """flc_norm2_torch_cpu (the sequential chain) or, parallel=True, flc_norm2_torch_cpu_ws (the
    binade-segment maps: the same bits without the chain)."""
    from flpytorch_amd import _lib
    n, d = rows_np.shape
    ld = ld or d
    buf = torch.zeros(n * ld + 4, dtype=torch.float32, device="cuda")
    for i in range(n):
        buf[i * ld:i * ld + d] = torch.from_numpy(rows_np[i])
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    lib = _lib.load()
    if parallel:
        ws = torch.empty(max(1, lib.flc_norm2_torch_cpu_workspace_size(n, d)), dtype=torch.uint8, device="cuda")
        _lib.check(lib.flc_norm2_torch_cpu_ws(buf.data_ptr(), ld, n, d, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                              _lib.stream_ptr()), "flc_norm2_torch_cpu_ws")
    else:
        _lib.check(lib.flc_norm2_torch_cpu(buf.data_ptr(), ld, n, d, out.data_ptr(), _lib.stream_ptr()),
                   "flc_norm2_torch_cpu")
    return out.cpu().numpy()


def _assert_norms(got, rows):
    for i in range(rows.shape[0]):
        w = oracle_norm(rows[i])
        if np.isnan(w):
            assert np.isnan(got[i]), i
        else:
            assert got[i].view(np.uint32) == w.view(np.uint32), (i, got[i], w)


@pytest.mark.parametrize("parallel", [False, True])
@pytest.mark.parametrize("d", [1, 7, 8, 9, 63, 4097, 8191, 8192, 8193, 8200, 65543, 262_151, 1_000_003])
def test_torch_norm_lengths(d, parallel):
    g = np.random.default_rng(d)
    rows = (g.standard_normal((3, d)) * 10.0 ** g.uniform(-3, 3, (3, d))).astype(np.float32)
    got = gpu_norms(rows, ld=d + 5, parallel=parallel)
    want = np.array([oracle_norm(r) for r in rows], dtype=np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("parallel", [False, True])
def test_torch_norm_specials(parallel):
    d = 20_011
    g = np.random.default_rng(5)
    rows = g.standard_normal((6, d)).astype(np.float32)
    rows[0] = 0.0
    rows[1] = np.float32(1e-41)                 # subnormal squares underflow
    rows[2, ::3] = np.float32(3e19)             # squares overflow to inf
    rows[3, 17] = np.inf
    rows[4, 5000] = np.nan
    rows[5] = -rows[5]
    _assert_norms(gpu_norms(rows, parallel=parallel), rows)


def test_torch_norm_parallel_segments():
    """The parallel form (flc_norm2_torch_cpu_ws) on rows built against its own structure, bit-exact
    against the sequential restatement: ties to even at every binade (values 1.25, 1.5, 1.75 x 2^k
    whose squares sit exactly half an ulp off the accumulator's grid), a stagnating accumulator
    (one huge square, then squares below half its ulp: the float64 prediction is off by far), a
    tiny-then-normal ramp (the accumulator crosses ~250 binades from the subnormal grid), every
    element equal, NaN / inf after a long finite prefix, and a Gaussian row of C4's D = 25 M."""
    d = 1_000_003
    g = np.random.default_rng(77)
    rows = np.zeros((8, d), dtype=np.float32)
    rows[0] = (g.choice([1.25, 1.5, 1.75, -1.25, 0.75], d) * 2.0 ** g.integers(-3, 4, d)).astype(np.float32)
    rows[1] = (g.standard_normal(d) * 1e-4).astype(np.float32)
    rows[1, 3] = np.float32(3e15)
    rows[2] = (2.0 ** np.linspace(-140, 20, d)).astype(np.float32)
    rows[3] = np.float32(1.25)
    rows[4] = g.standard_normal(d).astype(np.float32)
    rows[4, d - 100] = np.nan
    rows[5] = g.standard_normal(d).astype(np.float32)
    rows[5, 700_000] = np.inf
    rows[6] = (g.integers(-4, 5, d) * 0.25).astype(np.float32)
    rows[7] = np.float32(1e-30) * g.standard_normal(d).astype(np.float32)
    _assert_norms(gpu_norms(rows, parallel=True), rows)
    big = g.standard_normal((1, 25_000_000)).astype(np.float32)
    _assert_norms(gpu_norms(big, parallel=True), big)


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
