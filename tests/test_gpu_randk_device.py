"""Device-RNG RandK (randk_tree.hpp sampler, k_randk_counts + the list-free k_randk_fold) against
the oracle: the index sets come from oracle/devrng.py's numpy restatement of the sampler (not from
the library), the expected fold from oracle/codecs.py's sequential fp32 reduction of the dense
compressVector outputs.  Bit-exact (uint32 compare) for every case: chunk-part splits (C < 256,
< 1024, >= 1024 chunks), short last chunks, rows with more than 64 members in a chunk (the fold's
in-place tail), 64-row batch boundaries, weights (negative / zero), both row entry points, and the
sign of zero where every row keeps a -0."""
import numpy as np
import pytest
import torch

from oracle import codecs as oc
from oracle import devrng

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ag():
    assert torch.cuda.is_available()
    from flpytorch_amd import aggregation
    return aggregation


def bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


def oracle_fold(rows, spec, seed, client0, weights=None):
    n, d = rows.shape
    enc = []
    for i in range(n):
        o = oc.OracleCompressor(spec, d)
        o.S = devrng.randk_indices(seed, client0 + i, d, o.K)
        enc.append(o.compress(rows[i]))
    return oc.reduce_plain(enc, weights)


@pytest.mark.parametrize("n,d,k", [(3, 100_003, 1001), (2, 1_000_000, 10_000), (70, 40_000, 400),
                                   (2, 9000, 9000), (4, 4096, 1), (1, 1, 1), (2, 5_000_003, 50_001)])
def test_device_randk_counts_kernel(ag, n, d, k):
    """k_randk_counts (the GPU's hypergeometric tree) == oracle/devrng.py's restatement, per chunk."""
    import ctypes
    from flpytorch_amd import _lib
    lib = _lib.load()
    seed, client0 = 20241015, 11
    C = (d + 4095) // 4096
    out = torch.zeros((C, n), dtype=torch.int32, device="cuda")
    wsb = lib.flc_device_randk_counts_workspace_size(n, d)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    rc = lib.flc_device_randk_counts(seed, client0, n, d, k, ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(ws.data_ptr()), wsb, _lib.stream_ptr())
    assert rc == 0
    got = out.cpu().numpy().astype(np.int64)
    for i in range(n):
        assert np.array_equal(got[:, i], devrng.randk_counts(seed, client0 + i, d, k)), i


CASES = [
    # (n, d, spec)                      chunks  parts  notes
    (3, 100_003, "randk:1%"),         # 25      4
    (5, 1_000_000, "randk:1%"),       # 245     4      C2's row size
    (2, 2_000_001, "randk:1%"),       # 489     2
    (2, 5_000_003, "randk:1%"),       # 1221    1
    (70, 40_000, "randk:1%"),         # 10      4      two 64-row batches
    (4, 50_000, "randk:5%"),          # ~205 members per chunk: the > 64 tail path
    (3, 9000, "randk:100%"),          # K = D: every column kept by every row
    (6, 4096, "randk:1"),             # K = 1
    (1, 12289, "randk:50%"),          # one row, short last chunk
]


@pytest.mark.parametrize("n,d,spec", CASES)
def test_device_randk_fold_vs_oracle(ag, n, d, spec):
    seed, client0 = 20241015, 11
    rows = np.random.default_rng([n, d]).standard_normal((n, d)).astype(np.float32)
    want = oracle_fold(rows, spec, seed, client0)
    red = ag.UplinkReducer(ag.initCompressor(spec, d), seed=seed)
    rt = torch.from_numpy(rows).cuda()
    got = red(rt, client0=client0).cpu().numpy()
    assert np.array_equal(bits(got), bits(want))
    got2 = red([rt[i] for i in range(n)], client0=client0).cpu().numpy()
    assert np.array_equal(bits(got2), bits(want))


def test_device_randk_weights(ag):
    n, d, spec, seed = 7, 70_001, "randk:2%", 99
    rows = np.random.default_rng(1).standard_normal((n, d)).astype(np.float32)
    w = [1.0, -0.5, 0.0, 2.25, 1.0, -3.0, 0.125]
    want = oracle_fold(rows, spec, seed, 0, w)
    got = ag.UplinkReducer(ag.initCompressor(spec, d), seed=seed)(torch.from_numpy(rows).cuda(), weights=w)
    assert np.array_equal(bits(got.cpu().numpy()), bits(want))


@pytest.mark.parametrize("w", [None, [1.0, 2.0, 0.5], [-1.0, -2.0, -0.5], [1.0, -1.0, 1.0]])
def test_device_randk_signed_zero(ag, w):
    """Columns where rows hold -0: with K = D every row keeps every column, so the reference's sum
    is -0 exactly where every row's term is -0; with K < D a row that skips the column adds
    w * (+0).  Both resolved bit-exactly (rk_resolve_neg_zero)."""
    n, d, seed = 3, 5000, 4
    rows = np.random.default_rng(2).standard_normal((n, d)).astype(np.float32)
    rows[:, :300] = -0.0                    # -0 in every row
    rows[0, 300:600] = -0.0                 # -0 in one row only
    rows[:, 600:700] = 0.0
    for spec in ("randk:100%", "randk:90%", "randk:1%"):
        want = oracle_fold(rows, spec, seed, 3, w)
        got = ag.UplinkReducer(ag.initCompressor(spec, d), seed=seed)(torch.from_numpy(rows).cuda(), client0=3,
                                                                        weights=w)
        assert np.array_equal(bits(got.cpu().numpy()), bits(want)), spec


@pytest.mark.parametrize("d,spec", [(1_000_000, "randk:1%"), (12289, "randk:50%"), (4096, "randk:1"), (1, "randk:1")])
def test_device_randk_compress_vector(ag, d, spec):
    """Single-row compressVector in device mode: out = 0, out[S] = (D/K) x[S] with S the sampler's set."""
    seed, client = 77, 5
    x = np.random.default_rng(d).standard_normal(d).astype(np.float32)
    c = ag.initCompressor(spec, d)
    c.device_rng = (seed, client)
    got = c.compressVector(torch.from_numpy(x).cuda()).cpu().numpy()
    o = oc.OracleCompressor(spec, d)
    o.S = devrng.randk_indices(seed, client, d, o.K)
    assert np.array_equal(bits(got), bits(o.compress(x)))


@pytest.mark.parametrize("n,d,spec", [(3, 100_003, "randk:1%"), (2, 5_000_003, "randk:1%"), (70, 40_000, "randk:1%")])
def test_device_randk_precomputed_counts(ag, n, d, spec):
    """flc_pattern.d_randk_counts: counts made ahead by flc_device_randk_counts on another stream
    (how MixedUplink overlaps them) give the same bits as the counts made inside the call, on both
    the short-row (lists) and the long-row (list-free fold) paths."""
    seed, client0 = 777, 5
    rows = np.random.default_rng([n, d, 1]).standard_normal((n, d)).astype(np.float32)
    want = oracle_fold(rows, spec, seed, client0)
    red = ag.UplinkReducer(ag.initCompressor(spec, d), seed=seed)
    rt = torch.from_numpy(rows).cuda()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        cnt = red.randk_counts(n, d, client0)
    torch.cuda.current_stream().wait_stream(side)
    got = red(rt, client0=client0, randk_counts=cnt).cpu().numpy()
    assert np.array_equal(bits(got), bits(want))
    assert int(cnt.sum()) == n * red.comp.K
