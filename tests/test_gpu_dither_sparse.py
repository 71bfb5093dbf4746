"""GPU parity of the sparse fused dithering path (flpytorch_amd/csrc/dither_sparse.hip).

QSGD / standard dithering with p = 2, fused encode + reduce: one pass per row
keeps the elements that could be nonzero (against a sampled lower bound of the norm), the chunk
owners encode them exactly.  Bar: BIT-EXACT (uint32 compare) against the oracle — the reference's
op order (oracle/codecs.py, compressors.py:270-299) with the device draws restated in numpy
(oracle/devrng.py) — including the sign of zero, and bit-identical to the dense two-pass path at
C4 scale.  Compressor.dither_path = "sparse" | "dense" (the flc_codec_params.flags hint) forces a
path; the automatic choice keeps small D dense.  Compat mode (the caller's float64 uniforms, the
reference's numpy stream) takes the same single pass reading the uniforms beside the rows.
"""
import zlib

import numpy as np
import pytest
import torch

from oracle import codecs as oc
from oracle import devrng

pytestmark = pytest.mark.gpu

SEED = 20240607


@pytest.fixture(scope="module")
def ag():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from flpytorch_amd import aggregation
    return aggregation


def bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


def assert_bitexact(got, want):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else got
    g, w = bits(got), bits(want)
    # NaN results must sit at the same positions; their payload / sign bit is not compared
    # (numpy on x86 and the GPU propagate different NaN encodings)
    same = (g == w) | (np.isnan(np.asarray(got, np.float32)).ravel() & np.isnan(np.asarray(want, np.float32)).ravel())
    if not same.all():
        bad = np.nonzero(~same)[0]
        raise AssertionError(f"{bad.size} of {g.size} elements differ; first {bad[:5]}: "
                             f"{np.asarray(got).ravel()[bad[:5]]} vs {np.asarray(want).ravel()[bad[:5]]}")


def oracle_uplink(spec, rows, client0, weights=None, seed=SEED, uniforms=None):
    d = rows.shape[1]
    enc, norms = [], []
    for i in range(rows.shape[0]):
        o = oc.OracleCompressor(spec, d)
        o.testp = devrng.uniforms(seed, client0 + i, d) if uniforms is None else uniforms[i]
        enc.append(o.compress(rows[i]))
        norms.append(o.norm(rows[i]))
    return oc.reduce_plain(enc, weights), np.array(norms, dtype=np.float32)


def sparse(ag, spec, d):
    """A compressor whose fused uplink is forced onto the sparse path (flags hint)."""
    c = ag.initCompressor(spec, d)
    c.dither_path = "sparse"
    return c


def make_rows(kind, n, d, g):
    if kind == "normal":
        return g.standard_normal((n, d)).astype(np.float32)
    if kind == "heavy":      # N(0,1) * 10^U(-3, 3): wide dynamic range
        return (g.standard_normal((n, d)) * 10.0 ** g.uniform(-3, 3, (n, d))).astype(np.float32)
    if kind == "sparse":     # mostly exact zeros: the sample sees nothing, the bound is +inf
        r = np.zeros((n, d), dtype=np.float32)
        for i in range(n):
            k = g.choice(d, size=max(1, d // 5000), replace=False)
            r[i, k] = g.standard_normal(k.size).astype(np.float32)
        return r
    if kind == "negative":   # every element < 0 and tiny vs the norm: many -0 columns
        r = -np.abs(g.standard_normal((n, d))).astype(np.float32) * 1e-3
        r[:, 0] = -50.0
        return r
    if kind == "clustered":  # the mass in one short run: lists overflow -> dense rows
        r = (g.standard_normal((n, d)) * 1e-4).astype(np.float32)
        r[:, d // 3: d // 3 + 20000] = g.standard_normal((n, 20000)).astype(np.float32) * 3
        return r
    if kind == "ones":       # flat rows: the s sqrt(D) bound is attained
        return np.sign(g.standard_normal((n, d))).astype(np.float32)
    if kind == "tiny":       # norms near FLT_MIN: levels * norm are subnormal (fold must keep them)
        return (g.standard_normal((n, d)) * 1e-41).astype(np.float32)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["normal", "heavy", "sparse", "negative", "clustered", "ones", "tiny"])
@pytest.mark.parametrize("spec", ["qsgd:4", "qsgd:127"])
def test_sparse_dither_vs_oracle(ag, monkeypatch, kind, spec):
    n, d, client0 = 5, 300_001, 11
    rows = make_rows(kind, n, d, np.random.default_rng(zlib.crc32(f"{kind}{spec}".encode())))
    want, wn = oracle_uplink(spec, rows, client0)
    red = ag.UplinkReducer(sparse(ag, spec, d), seed=SEED)
    pn = torch.empty(n, device="cuda")
    got = red(torch.from_numpy(rows).cuda(), client0=client0, pnorms_out=pn)
    assert_bitexact(pn, wn)
    assert_bitexact(got, want)


@pytest.mark.parametrize("d", [1, 3, 4096, 4097, 8192 * 3 + 5, 16384, 16385, 65536, 65537, 100_000])
def test_sparse_dither_shapes(ag, monkeypatch, d):
    """Chunk / item / sample boundaries, tiny rows (whole-row sample)."""
    n, client0 = 3, 0
    rows = np.random.default_rng(d).standard_normal((n, d)).astype(np.float32)
    want, _ = oracle_uplink("qsgd:16", rows, client0)
    red = ag.UplinkReducer(sparse(ag, "qsgd:16", d), seed=SEED)
    assert_bitexact(red(torch.from_numpy(rows).cuda(), client0=client0), want)
    # the pointer-array entry point reads the same rows
    rt = torch.from_numpy(rows).cuda()
    assert_bitexact(red([rt[i].clone() for i in range(n)], client0=client0), want)


@pytest.mark.parametrize("bad", [None, "nan", "inf"])
def test_sparse_dither_weights_nonfinite(ag, monkeypatch, bad):
    """Weights (some negative, one zero) flip zero signs; a row with a NaN (norm NaN: every
    output NaN, as in the reference) or an inf element (norm inf) is folded dense."""
    n, d, client0 = 6, 120_000, 5
    g = np.random.default_rng(3)
    rows = make_rows("negative", n, d, g)
    rows[1] = g.standard_normal(d).astype(np.float32)
    if bad == "nan":
        rows[4, 777] = np.nan
    if bad == "inf":
        rows[5, 31] = np.inf
    w = [0.5, -2.0, 1.0, 0.0, 3.0, 1.25]
    want, _ = oracle_uplink("qsgd:8", rows, client0, weights=w)
    red = ag.UplinkReducer(sparse(ag, "qsgd:8", d), seed=SEED)
    assert_bitexact(red(torch.from_numpy(rows).cuda(), client0=client0, weights=w), want)


@pytest.mark.parametrize("groups", [2, 3])
@pytest.mark.parametrize("weighted", [False, True])
def test_sparse_dither_row_groups(ag, monkeypatch, groups, weighted):
    """The row-group pipeline (filter of group g+1 beside the fold of group g on a side stream; the
    folds continue each other's sums) gives the same bits as the sequential fold."""
    n, d, client0 = 7, 150_001, 3
    g = np.random.default_rng(groups)
    rows = make_rows("normal", n, d, g)
    rows[2] = make_rows("negative", 1, d, g)[0]
    rows[5] = make_rows("clustered", 1, d, g)[0]          # a dense-folded row inside a group
    w = [1.0, -0.5, 2.0, 1.5, 0.25, 1.0, 3.0] if weighted else None
    want, wn = oracle_uplink("qsgd:16", rows, client0, weights=w)
    comp = sparse(ag, "qsgd:16", d)
    comp.row_groups = groups
    red = ag.UplinkReducer(comp, seed=SEED)
    pn = torch.empty(n, device="cuda")
    got = red(torch.from_numpy(rows).cuda(), client0=client0, weights=w, pnorms_out=pn)
    torch.cuda.synchronize()
    assert_bitexact(pn, wn)
    assert_bitexact(got, want)


@pytest.mark.parametrize("spec,d", [("qsgd:16", 40_003), ("qsgd:127", 300_007)])
@pytest.mark.parametrize("entry", ["matrix", "pointers"])
@pytest.mark.parametrize("weighted", [False, True])
def test_sparse_dither_default_row_groups(ag, monkeypatch, spec, d, entry, weighted):
    """Without a hint, 128 rows or more take the default two row groups (group 0's norm, resolve
    and fold on the side stream under group 1's filter, whose blocks carry the LDS pad): same bits
    as the oracle, through both entry points, with special rows on either side of the boundary."""
    n, client0 = 161, 11
    g = np.random.default_rng(161 + weighted)
    rows = make_rows("normal", n, d, g)
    for i, kind in ((0, "negative"), (79, "clustered"), (80, "clustered"), (81, "sparse"),
                    (120, "heavy"), (160, "ones")):
        rows[i] = make_rows(kind, 1, d, g)[0]
    w = g.uniform(-1.0, 2.0, n).astype(np.float32).tolist() if weighted else None
    want, wn = oracle_uplink(spec, rows, client0, weights=w)
    comp = sparse(ag, spec, d)
    assert getattr(comp, "row_groups", None) in (None, 0)
    red = ag.UplinkReducer(comp, seed=SEED)
    x = torch.from_numpy(rows).cuda()
    arg = x if entry == "matrix" else [x[i] for i in range(n)]
    pn = torch.empty(n, device="cuda")
    got = red(arg, client0=client0, weights=w, pnorms_out=pn)
    torch.cuda.synchronize()
    assert_bitexact(pn, wn)
    assert_bitexact(got, want)
    # one filter launch per row group (a second call, so the timing events stay out of the first)
    from flpytorch_amd import _lib
    _lib.profile_enable(True)
    _lib.profile_collect("k_ds_filter")
    again = red(arg, client0=client0, weights=w)
    torch.cuda.synchronize()
    launches = _lib.profile_collect("k_ds_filter")[1]
    _lib.profile_enable(False)
    assert launches == 2
    assert_bitexact(again, want)


@pytest.mark.parametrize("kind", ["normal", "heavy", "sparse", "negative", "clustered", "tiny", "nan"])
@pytest.mark.parametrize("compat", [False, True])
@pytest.mark.parametrize("spec", ["qsgd:16", "qsgd:127"])
def test_lone_compress_vector_sparse(ag, monkeypatch, kind, compat, spec):
    """A lone compressVector (compressors.py:270-299) forced onto the single-read sparse pass (one
    row folded with weight 1 is its encode, -0 included): bit-exact vs the oracle with device
    draws and with the caller's float64 uniforms, and so is the dense two-pass encode (the
    automatic choice for one row)."""
    d, client = 2_000_003, 9
    g = np.random.default_rng(zlib.crc32(f"lone{kind}{compat}{spec}".encode()))
    x = make_rows("normal" if kind == "nan" else kind, 1, d, g)[0]
    if kind == "nan":
        x[1234] = np.nan
    o = oc.OracleCompressor(spec, d)
    c = sparse(ag, spec, d)
    if compat:
        u = g.random(d)
        o.testp = u
        c.testp = torch.from_numpy(u).cuda()
    else:
        o.testp = devrng.uniforms(SEED, client, d)
        c.device_rng = (SEED, client)
    want = o.compress(x)
    xt = torch.from_numpy(x).cuda()
    pn = torch.empty(1, device="cuda")
    got = c._encode_gpu(xt, pnorm_out=pn)
    assert_bitexact(got, want)
    assert_bitexact(pn, np.array([o.norm(x)], dtype=np.float32))
    assert_bitexact(c.compressVector(xt), want)
    c.dither_path = "dense"
    assert_bitexact(c.compressVector(xt), want)


@pytest.mark.parametrize("compat", [False, True])
def test_lone_compress_vector_c4_scale(ag, monkeypatch, compat):
    """The drop-in call at C4's row length (qsgd:127, D = 25 M): the forced sparse pass and the
    dense two-pass encode (the automatic choice) give the same bits and the same norm."""
    d = 25_000_000
    x = torch.empty(d, device="cuda").normal_(generator=torch.Generator("cuda").manual_seed(7))
    c = ag.initCompressor("qsgd:127", d)
    if compat:
        c.testp = torch.rand(d, dtype=torch.float64, device="cuda", generator=torch.Generator("cuda").manual_seed(8))
    else:
        c.device_rng = (SEED, 3)
    outs, norms = {}, {}
    for path in ("sparse", "dense"):
        c.dither_path = path
        pn = torch.empty(1, device="cuda")
        outs[path] = c._encode_gpu(x, pnorm_out=pn).cpu().numpy()
        norms[path] = pn.cpu().numpy()
    assert_bitexact(norms["sparse"], norms["dense"])
    assert_bitexact(outs["sparse"], outs["dense"])
    assert 0 < np.count_nonzero(outs["sparse"]) < d


def test_sparse_equals_dense_c4_scale(ag, monkeypatch):
    """C4's row length (D = 25 M, qsgd:127): the sparse path and the dense two-pass path give
    the same bits, and the same norms (the oracle would take minutes at this size)."""
    n, d = 6, 25_000_000
    x = torch.empty((n, d), device="cuda").normal_(generator=torch.Generator("cuda").manual_seed(4))
    comp = ag.initCompressor("qsgd:127", d)
    red = ag.UplinkReducer(comp, seed=SEED)
    outs, norms = {}, {}
    for path in ("sparse", "dense"):
        comp.dither_path = path
        pn = torch.empty(n, device="cuda")
        outs[path] = red(x, client0=100, pnorms_out=pn).cpu().numpy()
        norms[path] = pn.cpu().numpy()
    assert_bitexact(norms["sparse"], norms["dense"])
    assert_bitexact(outs["sparse"], outs["dense"])
    nz = np.count_nonzero(outs["sparse"])
    assert 0 < nz < d


def test_auto_path_choice(ag, monkeypatch):
    """Without the override, C4's shape takes the sparse path and short rows the dense one
    (checked through the library's launch profiler); the environment never changes the path."""
    from flpytorch_amd import _lib
    monkeypatch.setenv("FLC_DITHER_PATH", "dense")       # read only by -DFLC_TUNING builds
    for d, want, other in ((25_000_000, "k_ds_filter", "k_ew_accum_vec"), (200_000, "k_ew_accum_vec", "k_ds_filter")):
        x = torch.randn((2, d), device="cuda")
        red = ag.UplinkReducer(ag.initCompressor("qsgd:127", d), seed=SEED)
        _lib.profile_enable(True)
        try:
            red(x)
            torch.cuda.synchronize()
            assert _lib.profile_collect(want)[1] >= 1, (d, want)     # >= 1: row groups (tuning builds)
            assert _lib.profile_collect(other)[1] == 0, (d, other)
        finally:
            _lib.profile_enable(False)


@pytest.mark.parametrize("big", [440, 470, 505, 530])
def test_sparse_dither_item_near_staging_capacity(ag, monkeypatch, big):
    """A filter item (8192 elements) whose candidate count lands just below, at and just past
    its 512-entry LDS staging: `big` elements of the first item at +-1 (kept at a level >= 1 for
    sure, so always candidates) plus ~1/256 of the small rest.  Below 512 the item's entries are
    staged exactly (slot = running count + lane prefix); past it the row is folded dense."""
    n, d, client0, spec = 3, 16384, 2, "qsgd:127"
    g = np.random.default_rng(big)
    rows = (g.standard_normal((n, d)) * 1e-3).astype(np.float32)
    for i in range(n):
        idx = g.choice(8192, size=big, replace=False)
        rows[i, idx] = np.where(g.random(big) < 0.5, -1.0, 1.0).astype(np.float32)
    want, wn = oracle_uplink(spec, rows, client0)
    red = ag.UplinkReducer(sparse(ag, spec, d), seed=SEED)
    pn = torch.empty(n, device="cuda")
    got = red(torch.from_numpy(rows).cuda(), client0=client0, pnorms_out=pn)
    assert_bitexact(pn, wn)
    assert_bitexact(got, want)


@pytest.mark.parametrize("many", [9, 10, 11, 12, 40, 128])
def test_sparse_dither_lane_overflow(ag, monkeypatch, many):
    """Per-lane candidate staging (each lane of the filter's wave appends to its own column,
    DS_PLS = 10 slots per item): `many` sure candidates among the 128 elements one lane reads in
    an item (lane 5: elements 4*5 + 256 L + q of each chunk; lane 40 gets many // 2), the rest
    small.  Past 10 the lane's extra candidates are re-read and appended after the compaction;
    bit-exact vs the oracle either way (and with the pooled staging of other builds)."""
    n, d, client0, spec = 3, 16384, 7, "qsgd:127"
    g = np.random.default_rng(many)
    rows = (g.standard_normal((n, d)) * 1e-3).astype(np.float32)
    for lane, cnt in ((5, many), (40, many // 2)):
        pos = np.array([sub * 4096 + L * 256 + lane * 4 + q for sub in range(2) for L in range(16) for q in range(4)])
        for i in range(n):
            pick = g.choice(pos, size=cnt, replace=False)
            rows[i, pick] = np.where(g.random(cnt) < 0.5, -1.0, 1.0).astype(np.float32)
    want, wn = oracle_uplink(spec, rows, client0)
    red = ag.UplinkReducer(sparse(ag, spec, d), seed=SEED)
    pn = torch.empty(n, device="cuda")
    got = red(torch.from_numpy(rows).cuda(), client0=client0, pnorms_out=pn)
    assert_bitexact(pn, wn)
    assert_bitexact(got, want)


def compat_uniforms(n, d, g):
    """float64 draws in [0, 1) as numpy's random() makes them, with the edges planted: exact 0,
    the largest double below 1, and values a few ulps either side of 1/2."""
    u = g.random((n, d))
    u[:, 5] = 0.0
    u[:, 6] = np.nextafter(1.0, 0.0)
    u[:, 7:11] = 0.5 + np.array([-2, -1, 1, 2]) * 2.0 ** -53
    return u


@pytest.mark.parametrize("kind", ["normal", "heavy", "sparse", "negative", "clustered", "ones", "tiny"])
@pytest.mark.parametrize("spec", ["qsgd:4", "qsgd:127"])
def test_sparse_dither_compat_vs_oracle(ag, monkeypatch, kind, spec):
    """Compat draws (float64 uniforms, resident [N, D], a padded row stride) through the single
    pass: bit-exact against the oracle's `testp < p` with the same uniforms, norms included."""
    n, d, client0 = 5, 300_001, 11
    g = np.random.default_rng(zlib.crc32(f"compat{kind}{spec}".encode()))
    rows = make_rows(kind, n, d, g)
    uni = compat_uniforms(n, d, g)
    want, wn = oracle_uplink(spec, rows, client0, uniforms=uni)
    red = ag.UplinkReducer(sparse(ag, spec, d))
    pad = torch.zeros((n, d + 3), dtype=torch.float64, device="cuda")   # uniforms_ld = d + 3
    pad[:, :d] = torch.from_numpy(uni)
    pn = torch.empty(n, device="cuda")
    got = red(torch.from_numpy(rows).cuda(), client0=client0, pnorms_out=pn, uniforms=pad[:, :d])
    assert_bitexact(pn, wn)
    assert_bitexact(got, want)


@pytest.mark.parametrize("d", [1, 3, 4097, 8192 * 3 + 5, 16385])
def test_sparse_dither_compat_shapes_and_weights(ag, monkeypatch, d):
    """Compat draws at chunk / item / sample boundaries, weighted (negative and zero weights), and
    through the pointer-array entry point."""
    n = 4
    g = np.random.default_rng(d + 7)
    rows = g.standard_normal((n, d)).astype(np.float32)
    rows[2] = -np.abs(rows[2]) * 1e-3
    uni = g.random((n, d))
    w = [1.0, -0.5, 0.0, 2.0]
    want, _ = oracle_uplink("qsgd:16", rows, 0, weights=w, uniforms=uni)
    red = ag.UplinkReducer(sparse(ag, "qsgd:16", d))
    ud = torch.from_numpy(uni).cuda()
    rt = torch.from_numpy(rows).cuda()
    assert_bitexact(red(rt, weights=w, uniforms=ud), want)
    assert_bitexact(red([rt[i].clone() for i in range(n)], weights=w, uniforms=ud), want)


@pytest.mark.parametrize("groups", [1, 3])
def test_sparse_dither_compat_row_groups_nonfinite(ag, monkeypatch, groups):
    """Compat draws through the row-group pipeline, with a NaN row and a clustered (dense-folded)
    row: the dense fold reads the uniforms too."""
    n, d = 7, 150_001
    g = np.random.default_rng(groups + 40)
    rows = make_rows("normal", n, d, g)
    rows[2, 99] = np.nan
    rows[5] = make_rows("clustered", 1, d, g)[0]
    uni = g.random((n, d))
    want, wn = oracle_uplink("qsgd:16", rows, 0, uniforms=uni)
    comp = sparse(ag, "qsgd:16", d)
    comp.row_groups = groups
    red = ag.UplinkReducer(comp)
    pn = torch.empty(n, device="cuda")
    got = red(torch.from_numpy(rows).cuda(), pnorms_out=pn, uniforms=torch.from_numpy(uni).cuda())
    torch.cuda.synchronize()
    assert_bitexact(pn, wn)
    assert_bitexact(got, want)


def test_sparse_equals_dense_compat_c4_scale(ag, monkeypatch):
    """C4's row length with compat draws: the single pass and the dense two-pass path agree bit
    for bit, and the automatic choice takes the single pass."""
    from flpytorch_amd import _lib
    n, d = 4, 25_000_000
    gen = torch.Generator("cuda").manual_seed(9)
    x = torch.empty((n, d), device="cuda").normal_(generator=gen)
    uni = torch.empty((n, d), device="cuda", dtype=torch.float64).uniform_(generator=gen)
    comp = ag.initCompressor("qsgd:127", d)
    red = ag.UplinkReducer(comp)
    outs, norms = {}, {}
    for path in ("auto", "dense"):
        comp.dither_path = None if path == "auto" else path
        pn = torch.empty(n, device="cuda")
        _lib.profile_enable(True)
        try:
            outs[path] = red(x, pnorms_out=pn, uniforms=uni).cpu().numpy()
            launched = _lib.profile_collect("k_ds_filter")[1]
        finally:
            _lib.profile_enable(False)
        assert (launched >= 1) == (path == "auto"), (path, launched)
        norms[path] = pn.cpu().numpy()
    assert_bitexact(norms["auto"], norms["dense"])
    assert_bitexact(outs["auto"], outs["dense"])
    assert 0 < np.count_nonzero(outs["auto"]) < d
