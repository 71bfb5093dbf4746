"""GPU parity: libflcodec (HIP, gfx950) against the oracle and the reference's golden vectors.

Bars (stated per test):
  * reduction, RandK, TopK (no ambiguous tie), ident, lazy, natural, dithering given the same
    norm: BIT-EXACT (uint32 compare);
  * dithering with the kernel's own norm vs the reference's torch-CPU norm: relative error of
    every element <= 4*|n_gpu/n_ref - 1| + 4 ulp, with <= 1 % of elements allowed one level off;
    vs the oracle's exactly rounded norm: bit-exact;
  * TopK with ambiguous ties: same multiset of magnitudes as the reference (torch's tie order is
    unspecified); against the oracle (lowest index first): bit-exact.
"""
import math

import numpy as np
import pytest
import torch

from oracle import codecs as oc
from oracle import devrng
from oracle.rng import OracleRandomState
from tests.golden_io import load

pytestmark = pytest.mark.gpu

CODEC_META, CODEC = load("codecs")
RUN_META, RUNS = load("runs")


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
    if not np.array_equal(g, w):
        bad = np.nonzero(g != w)[0]
        raise AssertionError(f"{bad.size} of {g.size} elements differ; first {bad[:5]}: "
                             f"{np.asarray(got).ravel()[bad[:5]]} vs {np.asarray(want).ravel()[bad[:5]]}")


# ---------------------------------------------------------------------------------------------
# reduction (serverGradient core)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", sorted(RUN_META))
def test_server_gradient_golden_runs(ag, name):
    """run.py captures: the GPU fold equals the reference's gs bit for bit (incl. host round trip)."""

    class Buf:  # the reference Buffer's read protocol (buffer.py:59-102)
        def __init__(self, items):
            self.items, self.waits = items, 0

        def waitForItem(self):
            self.waits += 1

        def get(self, i):
            return self.items[i]

    for r in range(RUN_META[name]["rounds"]):
        x = RUNS[f"{name}_r{r}_x"]
        models = RUNS[f"{name}_r{r}_models"]
        want = RUNS[f"{name}_r{r}_gs"]
        for on_gpu in (True, False):
            dev = "cuda" if on_gpu else "cpu"
            items = [{"model": torch.from_numpy(m.copy()).to(dev), "client_state": {"weight": 1.0}} for m in models]
            buf = Buf(items)
            H = {"fl_dtype": torch.float32}
            gs = ag.reduce_client_models(buf, len(items), torch.from_numpy(x.copy()).to(dev), H)
            assert buf.waits == len(items)
            assert gs.device.type == dev
            assert_bitexact(gs, want)
            l2 = math.sqrt(float(np.sum(gs.cpu().numpy().astype(np.float64) ** 2)))
            assert abs(l2 - RUN_META[name]["grad_sgd_server_l2"][r]) <= 1e-6 * l2


@pytest.mark.parametrize("n,d", [(1, 1), (2, 3), (3, 4), (17, 1000), (64, 4099), (5, 262147), (300, 4096)])
@pytest.mark.parametrize("relative", [True, False])
@pytest.mark.parametrize("weighted", [False, True])
def test_reduce_vs_oracle(ag, n, d, relative, weighted):
    g = np.random.default_rng([n, d, relative, weighted])
    x = g.standard_normal(d).astype(np.float32)
    rows = (g.standard_normal((n, d)) * 10.0 ** g.uniform(-3, 3, (n, d))).astype(np.float32)
    w = list(g.uniform(0.1, 3.0, n)) if weighted else None
    want = oc.server_gradient(x, list(rows), w) if relative else oc.reduce_plain(list(rows), w)
    xt = torch.from_numpy(x).cuda()
    rt = torch.from_numpy(rows).cuda()
    # strided matrix entry and pointer-array entry
    got_m = ag.reduce_rows(xt, rt, w, relative=relative)
    got_p = ag.reduce_rows(xt, [rt[i] for i in range(n)], w, relative=relative)
    assert_bitexact(got_m, want)
    assert_bitexact(got_p, want)


def test_reduce_zero_clients(ag):
    x = torch.ones(10, device="cuda")
    assert torch.equal(ag.reduce_rows(x, [], None), torch.zeros(10, device="cuda"))


# ---------------------------------------------------------------------------------------------
# dense encode (compressVector) vs the reference's golden outputs
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("i", range(len(CODEC_META)))
@pytest.mark.parametrize("where", ["cuda", "cpu"])
def test_compress_vector_golden(ag, i, where):
    m = CODEC_META[i]
    X, OUT = CODEC[f"c{i:02d}_x"], CODEC[f"c{i:02d}_out"]
    pn = CODEC[f"c{i:02d}_pnorm"]
    stats = CODEC[f"c{i:02d}_stats"]
    rs = np.random.RandomState(m["seed"])
    for c in range(m["n_clients"]):
        comp = ag.initCompressor(m["spec"], m["D"])
        comp.generateCompressPattern(rs, where, c, None)
        assert int(rs.randint(2 ** 31)) == m["client_seeds"][c]       # stream position kept
        x = torch.from_numpy(X[c].copy()).to(where)
        out = comp.compressVector(x)
        assert out.device.type == where and out.shape == x.shape
        want = OUT[c]
        if m["type"] == 7:
            key = oc.topk_keys(X[c])
            kth = np.sort(key)[::-1][m["K"] - 1]
            if np.sum(key == kth) > 1:
                np.testing.assert_array_equal(np.sort(np.abs(out.cpu().numpy())), np.sort(np.abs(want)))
                # and exactly the oracle's lowest-index tie rule
                o = oc.OracleCompressor(m["spec"], m["D"])
                assert_bitexact(out, o.compress(X[c]))
            else:
                assert_bitexact(out, want)
        elif m["type"] in (5, 6):
            # (a) given the reference's own norm: bit-exact
            comp2 = ag.initCompressor(m["spec"], m["D"])
            comp2.testp = comp.testp
            got = comp2._encode_gpu(x.cuda(), pnorm_in=torch.tensor([pn[c]], dtype=torch.float32, device="cuda"))
            assert_bitexact(got, want)
            # (b) own norm: within the norms' ratio, except for decisions the norm difference flips.
            # A flip needs the uniform between the two probabilities; for std dithering (levels
            # 1/s apart) |dp_j| = s |x_j| rel / n, so E[flips] = s rel ||x||_1 / n.  Natural
            # dithering's output is y * sign * pnorm whatever the level (compressors.py:326): none.
            pno = torch.empty(1, device="cuda")
            own = comp2._encode_gpu(x.cuda(), pnorm_out=pno)
            rel = abs(float(pno.item()) / pn[c] - 1.0)
            ok = np.isclose(own.cpu().numpy(), want, rtol=4 * rel + 4 * 2.0 ** -24, atol=0)
            E = 0.0
            if m["type"] == 5 and pn[c] > 0:
                E = comp2.s * rel * float(np.abs(X[c]).astype(np.float64).sum()) / float(pn[c])
            assert np.sum(~ok) <= E + 5 * math.sqrt(E) + 3, (int(np.sum(~ok)), E)
            # (c) own norm == the oracle's exactly rounded norm -> bit-exact vs the oracle
            o = oc.OracleCompressor(m["spec"], m["D"])
            o.testp = comp.testp.cpu().numpy()
            assert float(pno.item()) == float(o.norm(X[c]))
            assert_bitexact(own, o.compress(X[c]))
        else:
            assert_bitexact(out, want)
        assert [comp.total_input_components, comp.really_need_to_send_components,
                comp.last_input_advance, comp.last_need_to_send_advance] == list(stats[c])


# ---------------------------------------------------------------------------------------------
# fused encode + reduce vs oracle (encode each row, sequential fp32 reduce)
# ---------------------------------------------------------------------------------------------
SPECS = ["ident", "randk:1%", "randk:10%", "topk:1%", "topk:5", "qsgd:127", "qsgd:3", "std.dithering:8",
         "std.dithering:5:1", "terngrad", "natural", "nat.dithering:6:2", "bernulli:0.5"]


def oracle_uplink(spec, rows, seed, weights=None):
    """Oracle: numpy-stream patterns in client order, encode, sequential reduce."""
    rs = OracleRandomState(seed)
    enc, pats = [], []
    for x in rows:
        o = oc.OracleCompressor(spec, x.size)
        o.generate(rs)
        rs.randint31()
        enc.append(o.compress(x))
        pats.append(o)
    return oc.reduce_plain(enc, weights), pats


@pytest.mark.parametrize("spec", SPECS)
@pytest.mark.parametrize("n,d", [(1, 4099), (5, 4099), (7, 65536 + 12), (3, 300001)])
def test_encode_reduce_compat_vs_oracle(ag, spec, n, d):
    g = np.random.default_rng([n, d, len(spec)])
    rows = (g.standard_normal((n, d)) * 10.0 ** g.uniform(-2, 2, (n, d))).astype(np.float32)
    rows[:, :7] = 0.0
    w = list(g.uniform(0.5, 2.0, n)) if n > 1 else None
    want, pats = oracle_uplink(spec, list(rows), seed=99 + n, weights=w)
    comp = ag.initCompressor(spec, d)
    red = ag.UplinkReducer(comp)
    kw = {}
    t = pats[0].type
    if t == oc.RANDK:
        kw["randk_idx"] = torch.from_numpy(np.stack([p.S for p in pats])).cuda()
    if t in (oc.NATURAL, oc.STD_DITHERING, oc.NAT_DITHERING):
        kw["uniforms"] = torch.from_numpy(np.stack([p.testp for p in pats])).cuda()
    if t == oc.LAZY:
        kw["lazy_u"] = torch.tensor([p.testp for p in pats], dtype=torch.float64, device="cuda")
    got = red(torch.from_numpy(rows).cuda(), weights=w, **kw)
    assert_bitexact(got, want)
    # row-pointer entry point gives the same bits
    rt = torch.from_numpy(rows).cuda()
    got2 = red([rt[i] for i in range(n)], weights=w, **kw)
    assert_bitexact(got2, want)


@pytest.mark.parametrize("spec", ["randk:1%", "qsgd:127", "natural", "std.dithering:4"])
def test_encode_reduce_device_rng(ag, spec):
    """Device-RNG mode: the kernels' counter-based draws == the host mirror of the generator."""
    from flpytorch_amd import _lib
    lib = _lib.load()
    n, d, seed, client0 = 4, 20000, 12345, 77
    g = np.random.default_rng(5)
    rows = g.standard_normal((n, d)).astype(np.float32)
    enc = []
    for i in range(n):
        o = oc.OracleCompressor(spec, d)
        if o.type == oc.RANDK:
            idx = np.empty(o.K, dtype=np.int64)
            assert lib.flc_device_randk_indices(seed, client0 + i, d, o.K, idx.ctypes.data) == 0
            assert np.unique(idx).size == o.K and idx.min() >= 0 and idx.max() < d
            o.S = idx
        else:
            o.testp = devrng.uniforms(seed, client0 + i, d)
        enc.append(o.compress(rows[i]))
    want = oc.reduce_plain(enc)
    red = ag.UplinkReducer(ag.initCompressor(spec, d), seed=seed)
    got = red(torch.from_numpy(rows).cuda(), client0=client0)
    assert_bitexact(got, want)


# ---------------------------------------------------------------------------------------------
# TopK: fast path, exact fallback, ties, structured rows, sizes around the chunking
# ---------------------------------------------------------------------------------------------
def _topk_rows(kind, n, d, g):
    if kind == "normal":
        return g.standard_normal((n, d)).astype(np.float32)
    if kind == "ties":
        return (g.integers(-3, 4, (n, d)) * 0.5).astype(np.float32)
    if kind == "zeros":
        r = np.zeros((n, d), dtype=np.float32)
        r[:, ::97] = 1.0
        return r
    if kind == "clustered":          # all the mass in one region: the spread sample misjudges it
        r = (g.standard_normal((n, d)) * 1e-3).astype(np.float32)
        r[:, d // 3: d // 3 + d // 50] *= 1e4
        return r
    if kind == "fewnz":              # fewer than K nonzeros: the K-th magnitude is 0 (zeros admitted)
        r = np.zeros((n, d), dtype=np.float32)
        r[:, ::97] = g.standard_normal((n, len(range(0, d, 97)))).astype(np.float32)
        r[:, ::3 * 97] = 0.0
        return r
    if kind == "nan_inf":
        r = g.standard_normal((n, d)).astype(np.float32)
        r[:, 5] = np.inf
        r[:, 11] = -np.inf
        return r
    if kind == "heavy":              # SURVEY 8d's second distribution: N(0,1) * 10^U(-3,3)
        r = g.standard_normal((n, d), dtype=np.float32)
        r *= np.float32(10.0) ** g.uniform(-3, 3, (n, d)).astype(np.float32)
        return r
    raise ValueError(kind)


def _topk_enc(rows, k):
    """The oracle's dense TopK outputs (compressors.py:330-335, lowest-index ties)."""
    enc = []
    for r in rows:
        out = np.zeros(r.size, dtype=np.float32)
        ind = oc.topk_indices_fast(r, k)
        out[ind] = r[ind]
        enc.append(out)
    return enc


class _FilterVariants:
    """Counts the TopK filter launches by variant (flc_profile_*: k_topk_filter_g4 / _g2) over a block."""

    def __enter__(self):
        from flpytorch_amd import _lib
        self._lib = _lib
        _lib.profile_enable(True)
        for v in ("k_topk_filter_g4", "k_topk_filter_g2"):
            _lib.profile_collect(v)
        return self

    def __exit__(self, *exc):
        torch.cuda.synchronize()
        self.g4 = self._lib.profile_collect("k_topk_filter_g4")[1]
        self.g2 = self._lib.profile_collect("k_topk_filter_g2")[1]
        self._lib.profile_enable(False)
        return False


@pytest.mark.parametrize("kind", ["normal", "ties", "zeros", "clustered", "nan_inf", "fewnz"])
@pytest.mark.parametrize("n,d,k", [(3, 4096, 41), (4, 100003, 1000), (2, 1 << 20, 10486), (3, 50000, 20000)])
def test_topk_vs_oracle(ag, kind, n, d, k):
    g = np.random.default_rng([d, k])
    rows = _topk_rows(kind, n, d, g)
    enc = []
    for i in range(n):
        out = np.zeros(d, dtype=np.float32)
        ind = oc.topk_indices(rows[i], k)
        out[ind] = rows[i][ind]
        enc.append(out)
    want = oc.reduce_plain(enc)
    red = ag.UplinkReducer(ag.initCompressor(f"topk:{k}", d))
    got = red(torch.from_numpy(rows).cuda())
    assert_bitexact(got, want)
    # single-row dense encode (compressVector path)
    c = ag.initCompressor(f"topk:{k}", d)
    one = c.compressVector(torch.from_numpy(rows[0].copy()).cuda())
    assert_bitexact(one, enc[0])


@pytest.mark.parametrize("kind", ["normal", "ties", "fewnz"])
@pytest.mark.parametrize("n,d,k", [(256, 65548, 655), (130, 20011, 300)])
def test_topk_tail_groups_vs_oracle(ag, kind, n, d, k):
    """Many rows (n >= 128): the TopK uplink in tail row groups (4 groups at n = 256, 2 at 130) —
    each group's candidate select and exact fallback on the side stream under the next group's
    filter, the last group's select in 1024-thread workgroups, the fold split in two launches
    (rows of the first groups beside the last select, tiles carried) — bit-exact vs the oracle,
    with weights and through both entry points."""
    g = np.random.default_rng([n, d, k, len(kind)])
    rows = _topk_rows(kind, n, d, g)
    enc = []
    for i in range(n):
        out = np.zeros(d, dtype=np.float32)
        ind = oc.topk_indices(rows[i], k)
        out[ind] = rows[i][ind]
        enc.append(out)
    w = [float(v) for v in g.uniform(0.5, 2.0, n)]
    red = ag.UplinkReducer(ag.initCompressor(f"topk:{k}", d))
    rt = torch.from_numpy(rows).cuda()
    assert_bitexact(red(rt), oc.reduce_plain(enc))
    want_w = oc.reduce_plain(enc, w)
    assert_bitexact(red(rt, weights=w), want_w)
    assert_bitexact(red([rt[i] for i in range(n)], weights=w), want_w)


@pytest.mark.parametrize("d", [2_000_000, 10_000_000])
def test_topk_few_rows_kth_ties_vs_oracle(ag, d):
    """Few rows (the sharded lists + k_cs_pass path of a lone compressVector and of n <= 16 uplinks)
    whose K-th magnitude is tied by entries in different shards, with fewer places left than ties:
    the last arriver gathers the tie indices and admits the lowest (torch.topk's CPU order, the
    oracle's), instead of the exact path.  Bit-exact for the fused uplink (weighted too) and for
    compressVector of each row."""
    n, k = 3, d // 100
    g = np.random.default_rng([d, 7])
    rows = g.standard_normal((n, d)).astype(np.float32)
    for i, top in enumerate([0, 2, 5]):                  # ties straddle: 1, 3, 6 places left
        mags = np.sort(np.abs(rows[i]))[::-1]
        v = mags[k - 1 - top]
        below = np.flatnonzero(np.abs(rows[i]) < mags[k + 10])
        pos = below[np.linspace(0, len(below) - 1, 6 + i).astype(np.int64)]
        rows[i, pos] = v * np.where(g.random(len(pos)) < 0.5, -1.0, 1.0).astype(np.float32)
    enc = []
    for i in range(n):
        out = np.zeros(d, dtype=np.float32)
        ind = oc.topk_indices(rows[i], k)
        out[ind] = rows[i][ind]
        enc.append(out)
    red = ag.UplinkReducer(ag.initCompressor(f"topk:{k}", d))
    rt = torch.from_numpy(rows).cuda()
    assert_bitexact(red(rt), oc.reduce_plain(enc))
    # the tie cut ran on the fast path (F_TIES, 4) and no row fell back to the exact path (8), which
    # would give the same bits
    fl = ag.select_row_flags(red.comp, n, d).tolist()
    assert all(f & 8 == 0 and f & 4 for f in fl), f"row flags {fl}: expected the fast path's tie cut"
    w = [0.75, 1.5, 1.0]
    assert_bitexact(red(rt, weights=w), oc.reduce_plain(enc, w))
    c = ag.initCompressor(f"topk:{k}", d)
    for i in range(n):
        assert_bitexact(c.compressVector(rt[i]), enc[i])
        f = int(ag.select_row_flags(c, 1, d)[0])
        assert f & 8 == 0 and f & 4, f"compressVector row {i}: flags {f}, expected the fast path's tie cut"


@pytest.mark.parametrize("kind", ["normal", "heavy", "ties", "zeros", "clustered", "nan_inf", "fewnz"])
@pytest.mark.parametrize("d,k", [((1 << 21) + 3, 20_000), (10_000_000, 100_000), (4_000_000, 80_000)])
def test_topk_lone_row_vs_oracle(ag, kind, d, k):
    """A lone compressVector row (compressors.py:330-335) on its own pipeline: up to 16.7 M
    elements held in the chip's registers (k_lone_resident: exact radix select with grid barriers,
    the dense output written from the registers; flag 16).  Bit-exact vs the oracle (lowest-index
    ties) on every kind; never the exact fallback."""
    g = np.random.default_rng([d, k, len(kind)])
    x = _topk_rows(kind, 1, d, g)[0]
    want = _topk_enc([x], k)[0]
    c = ag.initCompressor(f"topk:{k}", d)
    xt = torch.from_numpy(x).cuda()
    assert_bitexact(c.compressVector(xt), want)
    f = int(ag.select_row_flags(c, 1, d)[0])
    assert f & 16 and f & 8 == 0 and f & 1 == 0, f"flags {f}: expected the register-resident select"
    # the same row at a 4-byte offset (scalar loads; the exact fallback's non-vector variant)
    buf = torch.zeros(d + 1, device="cuda")
    buf[1:] = xt
    assert_bitexact(c.compressVector(buf[1:]), want)


@pytest.mark.parametrize("kind", ["normal", "heavy"])
def test_topk_lone_row_three_passes(ag, kind):
    """A lone row longer than FLC_CS_TWO_MAXD (64 Mi): the candidate select keeps its third
    k_cs_pass launch (the first digit's bin may hold more entries than list mode ranks).
    Bit-exact vs the oracle, off the exact path."""
    d, k = (64 << 20) + 4099, 700_001
    g = np.random.default_rng([d, len(kind)])
    x = _topk_rows(kind, 1, d, g)[0]
    want = _topk_enc([x], k)[0]
    c = ag.initCompressor(f"topk:{k}", d)
    assert_bitexact(c.compressVector(torch.from_numpy(x).cuda()), want)
    f = int(ag.select_row_flags(c, 1, d)[0])
    assert f & 8 == 0, f"flags {f}: the row took the exact path"


@pytest.mark.parametrize("ties", [20, 600, 1500, 3000])
def test_topk_lone_row_tie_capacity(ag, ties):
    """The lone row's tie cut: `ties` extra entries equal to the K-th magnitude (signs mixed, spread
    over the row) straddle the cut.  The register-resident select (flag 16) ranks them over the grid
    whatever their number (F_TIES set, no exact path); the list path's TIECAP = 2048 bound (k_cs_pass)
    applies to rows longer than 16.7 M only.  Bit-exact vs the oracle."""
    d, k = 4_000_000, 40_000
    g = np.random.default_rng([ties, 3])
    x = g.standard_normal(d).astype(np.float32)
    mags = np.sort(np.abs(x))[::-1]
    v = mags[k - 1 - 7]                                   # 8 places left at the cut
    below = np.flatnonzero(np.abs(x) < mags[k + 10])
    pos = below[np.linspace(0, len(below) - 1, ties).astype(np.int64)]
    x[pos] = v * np.where(g.random(ties) < 0.5, -1.0, 1.0).astype(np.float32)
    want = _topk_enc([x], k)[0]
    c = ag.initCompressor(f"topk:{k}", d)
    assert_bitexact(c.compressVector(torch.from_numpy(x).cuda()), want)
    f = int(ag.select_row_flags(c, 1, d)[0])
    assert f & 16 and f & 4 and f & 8 == 0, f"flags {f}: expected the resident select's tie cut"


def test_topk_few_rows_stay_on_fast_path(ag):
    """Path guard for the few-row path (n <= 16: sharded lists + k_cs_pass): Gaussian rows at
    D = 10 M must not fall back to the exact selection (~8 ms per failed row against ~0.1 ms).  Two
    round-3 builds did: the fused uplink's interleaved item order put each of n rows' groups into
    64 / n shards (overflow), and ambiguous ties at the K-th key (~1 row in 8) went to the exact path.
    Asserted on the rows' path flags (flc_select_row_flags), not on wall-clock time; the device
    times are printed for information."""
    n, d = 8, 10_000_000
    k = d // 100
    gen = torch.Generator(device="cuda").manual_seed(9)
    rows = torch.randn(n, d, generator=gen, device="cuda")
    red = ag.UplinkReducer(ag.initCompressor(f"topk:{k}", d))
    c = ag.initCompressor(f"topk:{k}", d)

    def dev_ms(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    fused = dev_ms(lambda: red(rows))
    fl = ag.select_row_flags(red.comp, n, d).tolist()
    assert all(f & 8 == 0 for f in fl), f"fused {n}-row uplink: row flags {fl} (8 = exact path)"
    times = []
    for i in range(n):
        times.append(dev_ms(lambda: c.compressVector(rows[i])))
        f = int(ag.select_row_flags(c, 1, d)[0])
        assert f & 8 == 0, f"compressVector of row {i}: flags {f} (8 = exact path)"
    print(f"fused {n}-row uplink {fused:.3f} ms; compressVector " + " ".join(f"{t:.3f}" for t in times) + " ms")


@pytest.mark.parametrize("kind", ["normal", "heavy", "ties", "fewnz"])
def test_topk_c3_variant_vs_oracle(ag, kind):
    """The C3 bench's own TopK kernel variant: many rows (n > 16) with
    n * D >= 64 Mi take k_topk_filter_fast<16, 4> (4-chunk work items) in 4 tail row groups, each
    group's select and exact fallback on the side stream under the next group's filter.  n = 256,
    D = 300 007 (ragged last chunk and group), K = 1 %: bit-exact vs the oracle, weighted, through
    both entry points; the profile counters show the 4-chunk filter ran (4 launches per call) and,
    for normal / heavy-tailed rows, the path flags show no row fell back to the exact path."""
    n, d = 256, 300_007
    k = math.ceil(0.01 * d)
    g = np.random.default_rng([n, d, len(kind), 4])
    rows = _topk_rows(kind, n, d, g)
    enc = _topk_enc(rows, k)
    w = [float(v) for v in g.uniform(0.5, 2.0, n)]
    red = ag.UplinkReducer(ag.initCompressor("topk:1%", d))
    assert red.comp.K == k
    rt = torch.from_numpy(rows).cuda()
    with _FilterVariants() as fv:
        got = red(rt)
    assert (fv.g4, fv.g2) == (4, 0), f"filter variants g4={fv.g4} g2={fv.g2}: not the C3 bench's path"
    assert_bitexact(got, oc.reduce_plain(enc))
    if kind in ("normal", "heavy"):
        fl = np.asarray(ag.select_row_flags(red.comp, n, d))
        assert not np.any(fl & 8), f"{int(np.sum((fl & 8) != 0))} rows took the exact path"
    want_w = oc.reduce_plain(enc, w)
    assert_bitexact(red(rt, weights=w), want_w)
    with _FilterVariants() as fv:
        got = red([rt[i] for i in range(n)], weights=w)
    assert (fv.g4, fv.g2) == (4, 0)
    assert_bitexact(got, want_w)


@pytest.mark.parametrize("kind", ["ties", "zeros", "fewnz", "clustered"])
def test_topk_exact_fallback_in_side_select(ag, kind):
    """Rows that fall back to the exact path inside a NON-last row group of >= 128 rows: their select
    (k_cand_select_x) runs in 512-thread workgroups, so exact_row rewrites each 4096-column chunk in
    sub-blocks of NT * 4 = 2048 columns (it used to cover only the first 2048 columns
    of every chunk there).  n = 256 rows in 2 row groups (FLC_ROW_GROUPS(2)), D = 300 007 (ragged
    last chunk), K = 1 %: bit-exact vs the oracle, and group 0's rows are asserted to have taken the
    exact path (flag 8) for the structured rows."""
    n, d = 256, 300_007
    k = math.ceil(0.01 * d)
    g = np.random.default_rng([n, d, len(kind), 5])
    rows = _topk_rows(kind, n, d, g)
    enc = _topk_enc(rows, k)
    comp = ag.initCompressor("topk:1%", d)
    comp.row_groups = 2
    red = ag.UplinkReducer(comp)
    rt = torch.from_numpy(rows).cuda()
    assert_bitexact(red(rt), oc.reduce_plain(enc))
    fl = np.asarray(ag.select_row_flags(red.comp, n, d))
    assert np.any(fl[:128] & 8), f"{kind}: no row of group 0 took the exact path; flags {np.unique(fl)}"
    w = [float(v) for v in g.uniform(0.5, 2.0, n)]
    assert_bitexact(red([rt[i] for i in range(n)], weights=w), oc.reduce_plain(enc, w))


@pytest.mark.parametrize("m", [448, 511, 512, 513, 576, 700])
def test_topk_4chunk_group_staging_capacity(ag, m):
    """The 512-entry LDS staging of a 4-chunk group (the C3 variant, n = 17 > 16 rows, n * D >=
    64 Mi).  Row i: K "big" entries (|x| >= 1), m_i of them in its first group (elements
    0..16383, otherwise zeros), the rest spread over the row among small nonzero entries
    (|x| < 1e-3).  The sample's threshold then falls among the small entries, so group 0 stages
    exactly its m_i big entries — just below, at or past the staging — while every other group
    stays far below it.  A group that fits does not overflow (path flag 1 clear); one past 512
    overflows (spare slots, flag 1) and its row is redone exactly (flag 8).  (A row may still take
    the exact path for another reason: the bimodal rows can put the sample's K-th estimate among
    the small entries, flag 2.)  Bit-exact vs the oracle either way."""
    n, d = 17, 4_000_000
    k = d // 100
    g = np.random.default_rng([m, 17])
    rows = (g.uniform(1e-4, 1e-3, (n, d)) * np.where(g.random((n, d)) < 0.5, -1.0, 1.0)).astype(np.float32)
    rows[:, :16384] = 0.0
    counts = [m if i % 2 == 0 else 256 for i in range(n)]     # odd rows: a quiet first group
    for i in range(n):
        head = g.choice(16384, size=counts[i], replace=False)
        tail = 16384 + g.choice(d - 16384, size=k - counts[i], replace=False)
        idx = np.concatenate([head, tail])
        rows[i, idx] = ((np.abs(g.standard_normal(idx.size)) + 1.0) *
                        np.where(g.random(idx.size) < 0.5, -1.0, 1.0)).astype(np.float32)
    enc = _topk_enc(rows, k)
    assert all(np.count_nonzero(np.abs(e) >= 1.0) == k for e in enc)
    red = ag.UplinkReducer(ag.initCompressor(f"topk:{k}", d))
    with _FilterVariants() as fv:
        got = red(torch.from_numpy(rows).cuda())
    assert fv.g4 >= 1 and fv.g2 == 0, f"filter variants g4={fv.g4} g2={fv.g2}"
    assert_bitexact(got, oc.reduce_plain(enc))
    fl = ag.select_row_flags(red.comp, n, d).tolist()
    for i in range(n):
        over = counts[i] > 512
        assert bool(fl[i] & 1) == over and (not over or fl[i] & 8), f"row {i} ({counts[i]} in group 0): flags {fl[i]}"


def test_randk_scale_inexact(ag):
    """D/K = 98.6 (not exact in fp32): the reference's fp32 scalar multiply is reproduced."""
    d = 2465
    rs = np.random.RandomState(7)
    c = ag.initCompressor("randk:1%", d)
    c.generateCompressPattern(rs, "cuda", 0, None)
    x = np.random.default_rng(1).standard_normal(d).astype(np.float32)
    out = c.compressVector(torch.from_numpy(x).cuda())
    want = np.zeros(d, dtype=np.float32)
    S = c.S.cpu().numpy()
    want[S] = np.float32(d / c.K) * x[S]
    assert_bitexact(out, want)


def test_fast_division_selftest(ag):
    """The dithering kernels' Markstein division == IEEE division for every float numerator in
    [2^-80, 2^80], for norms / level gaps of every kind (random, powers of two, all-ones mantissa,
    the qsgd:127 level gap)."""
    from flpytorch_amd import _lib
    lib = _lib.load()
    g = np.random.default_rng(11)
    bs = list(np.float32(g.uniform(1, 2, 24)) * np.float32(2.0) ** g.integers(-30, 60, 24).astype(np.float32))
    bs += [np.float32(1.0), np.float32(3.0), np.float32(0.1), np.uint32(0x3FFFFFFF).view(np.float32),
           np.uint32(0x4B7FFFFF).view(np.float32), -np.float32(1.0 / 127), np.float32(0.0078740157),
           -np.float32(np.float32(2.0 / 127) - np.float32(1.0 / 127))]
    b = torch.tensor(np.array(bs, dtype=np.float32), device="cuda")
    bad = torch.zeros(len(bs), dtype=torch.int64, device="cuda")
    _lib.check(lib.flc_selftest_division(b.data_ptr(), len(bs), bad.data_ptr(), _lib.stream_ptr()), "selftest")
    torch.cuda.synchronize()
    assert bad.cpu().tolist() == [0] * len(bs)


@pytest.mark.parametrize("mode", ["compat", "device", "skewed"])
@pytest.mark.parametrize("d,k", [(5_000_003, 50_001), (2_500_000, 20_000)])
def test_randk_large_rows(ag, mode, d, k):
    """RandK beyond one chunk per superchunk (D > 1 M: coarse + fine bucketing); 'skewed' compat
    lists put every index in the first superchunk (the fine kernel's in-memory path)."""
    from flpytorch_amd import _lib
    lib = _lib.load()
    n, seed, client0 = 3, 31337, 5
    g = np.random.default_rng([d, k])
    rows = g.standard_normal((n, d)).astype(np.float32)
    idx = []
    for i in range(n):
        if mode == "device":
            s = np.empty(k, dtype=np.int64)
            assert lib.flc_device_randk_indices(seed, client0 + i, d, k, s.ctypes.data) == 0
            assert np.unique(s).size == k and s.min() >= 0 and s.max() < d
        elif mode == "skewed":
            s = g.permutation(k + 7)[:k].astype(np.int64)        # all inside [0, k + 7)
        else:
            s = g.choice(d, k, replace=False).astype(np.int64)
        idx.append(s)
    enc = []
    for i in range(n):
        o = oc.OracleCompressor(f"randk:{k}", d)
        o.S = idx[i]
        enc.append(o.compress(rows[i]))
    want = oc.reduce_plain(enc)
    red = ag.UplinkReducer(ag.initCompressor(f"randk:{k}", d), seed=seed)
    kw = {} if mode == "device" else {"randk_idx": torch.from_numpy(np.stack(idx)).cuda()}
    got = red(torch.from_numpy(rows).cuda(), client0=client0, **kw)
    assert_bitexact(got, want)


@pytest.mark.parametrize("name", sorted(RUN_META))
def test_shifted_server_gradients(ag, name):
    """DIANA (algorithms.py:1395-1421) and COFIG (1273-1307) on the run captures: the fold is the
    reference's gs bit for bit, then the same torch tail."""

    class Buf:
        def __init__(self, items):
            self.items = items

        def waitForItem(self):
            pass

        def get(self, i):
            return self.items[i]
    x = RUNS[f"{name}_r0_x"]
    models = RUNS[f"{name}_r0_models"]
    gs_ref = torch.from_numpy(RUNS[f"{name}_r0_gs"].copy()).cuda()
    g = torch.Generator(device="cuda").manual_seed(1)
    h = torch.randn(x.size, generator=g, device="cuda")
    items = [{"model": torch.from_numpy(m.copy()).cuda(), "client_state": {"weight": 1.0, "alpha": 0.37}} for m in models]
    xt = torch.from_numpy(x.copy()).cuda()
    H = {"fl_dtype": torch.float32, "h": h}
    out = ag.serverGradientDIANA(Buf(items), len(items), None, xt, H)
    assert_bitexact(H["m"], gs_ref.cpu().numpy())
    assert_bitexact(out, (h + gs_ref).cpu().numpy())
    H = {"fl_dtype": torch.float32, "h_prev": h, "total_clients": 10}
    out = ag.serverGradientCOFIG(Buf(items), len(items), None, xt, H)
    assert_bitexact(out, (gs_ref + h).cpu().numpy())
    assert_bitexact(H["u_avg_update"], gs_ref.cpu().numpy())
    assert H["alpha_update"] == 0.37 * (len(items) / 10)


def _ref_fold_cpu(x, rows, weights):
    """algorithms.py:1753-1768 on CPU tensors (true fp32 division by the Python-float total)."""
    gs = weights[0] * (x - rows[0])
    tot = weights[0]
    for w, r in zip(weights[1:], rows[1:]):
        tot += w
        gs += w * (x - r)
    return gs / tot


def test_gradskip_and_frecon_server_gradients(ag):
    """GradSkip (algorithms.py:951-998) and FRECON (1124-1176) wrappers against the reference's
    bodies restated on CPU tensors."""
    import types

    class Buf:
        def __init__(self, items):
            self.items = items

        def waitForItem(self):
            pass

        def get(self, i):
            return self.items[i]
    g = np.random.default_rng(0)
    n, d = 5, 4099
    x = g.standard_normal(d).astype(np.float32)
    models = [g.standard_normal(d).astype(np.float32) for _ in range(n)]
    his = [g.standard_normal(d).astype(np.float32) for _ in range(n)]
    w = [1.0, 0.5, 2.0, 1.5, 1.0]
    # GradSkip
    gamma, p = 0.1, 0.5
    items = [{"model": torch.from_numpy(m).cuda(), "client_state": {
        "weight": w[i], "local_steps": [], "Ki": 3, "change_shift": i % 2 == 0, "hi": torch.from_numpy(his[i]).cuda(),
        "grad": torch.from_numpy(his[(i + 1) % n]).cuda(), "stats": {"send_scalars_to_master": 0}}} for i, m in enumerate(models)]
    H = {"fl_dtype": torch.float32, "args": types.SimpleNamespace(local_lr=gamma), "p": p}
    out = ag.serverGradientGradSkip(Buf(items), n, None, torch.from_numpy(x).cuda(), H)
    hi_ref = [his[(i + 1) % n] if i % 2 == 0 else his[i] for i in range(n)]
    rows = [torch.from_numpy(models[i]) - torch.from_numpy(hi_ref[i]) * gamma / p for i in range(n)]
    want = _ref_fold_cpu(torch.from_numpy(x), rows, w)
    assert_bitexact(out, want.numpy())
    for i in range(n):
        assert items[i]["client_state"]["local_steps"] == [3 + (1 if i % 2 == 0 else 0)]
        assert_bitexact(items[i]["client_state"]["delta_x"], (torch.from_numpy(x) - want - torch.from_numpy(models[i])).numpy())
    # FRECON with the lambda_ experiment option
    qs = [g.standard_normal(d).astype(np.float32) for _ in range(n)]
    items = [{"model": torch.from_numpy(m).cuda(), "client_state": {"weight": w[i], "alpha": 0.25,
                                                                   "qi": torch.from_numpy(qs[i]).cuda()}}
             for i, m in enumerate(models)]
    am = types.SimpleNamespace(has_experiment_option=lambda H, k: k == "lambda_",
                               get_experiment_option_f=lambda H, k: 0.3)
    gprev = g.standard_normal(d).astype(np.float32)
    hprev = g.standard_normal(d).astype(np.float32)
    H = {"fl_dtype": torch.float32, "h_prev": torch.from_numpy(hprev).cuda(), "g_server_prev": torch.from_numpy(gprev).cuda(),
         "total_clients": 20}
    out = ag.make_server_gradient_frecon(am)(Buf(items), n, None, torch.from_numpy(x).cuda(), H)
    u = _ref_fold_cpu(torch.from_numpy(x), [torch.from_numpy(m) for m in models], w)
    q = w[0] * torch.from_numpy(qs[0])
    tot = w[0]
    for wi, qi in zip(w[1:], qs[1:]):
        tot += wi
        q += wi * torch.from_numpy(qi)
    q = q / tot
    want = q + (1.0 - 0.3) * torch.from_numpy(gprev) + 0.3 * (u + torch.from_numpy(hprev))
    assert_bitexact(out, want.numpy())
    assert all("qi" not in it["client_state"] for it in items)
    assert H["alpha_update"] == 0.25 * (n / 20)


def test_frecon_with_host_params(ag):
    """FRECON's serverGradient with a HOST params_current (the simulator's CPU model, device rows):
    both folds run on the GPU and the result lands on the host, equal to the device-params run."""
    import types

    class Buf:
        def __init__(self, items):
            self.items = items

        def waitForItem(self):
            pass

        def get(self, i):
            return self.items[i]
    g = np.random.default_rng(7)
    n, d = 4, 2049
    x = g.standard_normal(d).astype(np.float32)
    models = [g.standard_normal(d).astype(np.float32) for _ in range(n)]
    qs = [g.standard_normal(d).astype(np.float32) for _ in range(n)]
    gprev = g.standard_normal(d).astype(np.float32)
    hprev = g.standard_normal(d).astype(np.float32)
    am = types.SimpleNamespace(has_experiment_option=lambda H, k: k == "lambda_",
                               get_experiment_option_f=lambda H, k: 0.3)
    outs = []
    for on_host in (False, True):
        dev = "cpu" if on_host else "cuda"
        items = [{"model": torch.from_numpy(m.copy()), "client_state": {"weight": 1.0, "alpha": 0.5,
                                                                        "qi": torch.from_numpy(qs[i].copy()).cuda()}}
                 for i, m in enumerate(models)]
        H = {"fl_dtype": torch.float32, "h_prev": torch.from_numpy(hprev).to(dev),
             "g_server_prev": torch.from_numpy(gprev).to(dev), "total_clients": 8}
        out = ag.make_server_gradient_frecon(am)(Buf(items), n, None, torch.from_numpy(x).to(dev), H)
        assert out.device.type == dev
        outs.append(out.cpu().numpy())
    assert_bitexact(outs[1], outs[0])


@pytest.mark.parametrize("spec", ["topk:3%", "randk:3%"])
@pytest.mark.parametrize("n", [1, 2, 5])
@pytest.mark.parametrize("weights", ["ones", "mixed", "negative"])
def test_signed_zero_in_sparse_fold(ag, spec, n, weights):
    """Columns whose every kept value is -0 (the chunk-owner fold gave +0).  The
    reference adds the dense rows, so the result is -0 iff EVERY term is -0: kept -0 values, and
    w_i * (+0) for the rows that did not keep the column (-0 only for negative-signed weights).
    Bit-exact against the oracle's sequential fold, untouched columns included."""
    d = 3 * 4096 + 77
    g = np.random.default_rng(n * 7 + len(weights))
    rows = np.zeros((n, d), dtype=np.float32)
    k = math.ceil(0.03 * d)
    idx = []
    for i in range(n):
        # 40 large values per row, the rest +0, and -0 at the lowest indices: TopK keeps the 40
        # large ones and fills K from the lowest-index zeros (ties by lowest index) -> the -0s
        big = g.choice(np.arange(200, d), 40, replace=False)
        rows[i, big] = g.standard_normal(40).astype(np.float32) * 10
        rows[i, :150] = -0.0
        rows[i, 150:160] = 0.0
        if i == n - 1 and n > 1:
            rows[i, 100:150] = 0.0                           # the last client: +0 at some of them
        # RandK (compat indices): every client keeps 0..199 plus its own random others
        rest = g.choice(np.arange(200, d), k - 200, replace=False)
        idx.append(np.concatenate([np.arange(200), rest]).astype(np.int64))
    w = {"ones": None, "mixed": [1.0, -2.0, 0.5, -0.0, 3.0][:n], "negative": [-1.0, -0.5, -2.0, -1.5, -3.0][:n]}[weights]
    enc = []
    for i in range(n):
        o = oc.OracleCompressor(spec, d)
        o.S = idx[i]
        enc.append(o.compress(rows[i]))
    want = oc.reduce_plain(enc, w)
    kw = {"randk_idx": torch.from_numpy(np.stack(idx)).cuda()} if spec.startswith("randk") else {}
    red = ag.UplinkReducer(ag.initCompressor(spec, d))
    got = red(torch.from_numpy(rows).cuda(), weights=w, **kw)
    assert (want[:100] == 0).all() and (want[200:] == 0).any()      # kept -0 columns and untouched ones
    if weights == "ones":
        assert np.signbit(want[:100]).all()                           # ... that the reference returns as -0
    assert_bitexact(got, want)
    # the pointer-array entry point and the wire path (sparse payloads) give the same bits
    rt = torch.from_numpy(rows).cuda()
    assert_bitexact(red([rt[i].clone() for i in range(n)], weights=w, **kw), want)


def test_weighted_fold_vs_reference(ag):
    """The fold with client weights != 1 against the reference's own DCGD / FedAvg serverGradient
    (tests/golden/weighted.*, make_golden_weighted.py): both entry points and the protocol body
    with a host params_current, bit-exact."""
    import json
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(gold, "weighted.json")))
    arr = np.load(os.path.join(gold, "weighted.npz"))
    for m in meta:
        c = m["case"]
        x, rows, w = arr[f"c{c}_x"], arr[f"c{c}_rows"], m["weights"]
        want = arr[f"c{c}_{m['algorithm']}_gs"]
        xt, rt = torch.from_numpy(x).cuda(), torch.from_numpy(rows).cuda()
        assert_bitexact(ag.reduce_rows(xt, rt, w), want)
        assert_bitexact(ag.reduce_rows(xt, [rt[i] for i in range(len(w))], w), want)

        class Buf:
            def waitForItem(self):
                pass

            def get(self, i, _r=rows, _w=w):
                return {"model": torch.from_numpy(_r[i].copy()), "client_state": {"weight": _w[i]}}
        H = {"fl_dtype": torch.float32, "compressor_master": ag.initCompressor("ident", x.size)}
        body = ag.serverGradientMaster if m["algorithm"] == "dcgd" else ag.serverGradientPlain
        got = body(Buf(), len(w), None, torch.from_numpy(x.copy()), H)
        assert got.device.type == "cpu"
        assert_bitexact(got, want)


@pytest.mark.parametrize("kind", ["ties", "clustered"])
def test_topk_exact_rows_unaligned(ag, kind):
    """Rows the fast path fails (massive ties / a misjudging sample) go through the one-launch exact
    selection (k_topk_exact_rows); rows given as pointers at 4-byte (not 16-byte) offsets take its
    scalar loads.  Bit-exact against the oracle, fused fold and single-row compressVector."""
    n, d, k = 3, 70001, 700
    g = np.random.default_rng([d, k, 7])
    rows = _topk_rows(kind, n, d, g)
    enc = []
    for i in range(n):
        out = np.zeros(d, dtype=np.float32)
        ind = oc.topk_indices(rows[i], k)
        out[ind] = rows[i][ind]
        enc.append(out)
    want = oc.reduce_plain(enc)
    flat = torch.zeros(n * d + 1, dtype=torch.float32, device="cuda")
    flat[1:] = torch.from_numpy(rows.reshape(-1)).cuda()
    views = [flat[1 + i * d: 1 + (i + 1) * d] for i in range(n)]
    red = ag.UplinkReducer(ag.initCompressor(f"topk:{k}", d))
    assert_bitexact(red(views), want)
    c = ag.initCompressor(f"topk:{k}", d)
    assert_bitexact(c.compressVector(views[1]), enc[1])


@pytest.mark.parametrize("k", [440, 490, 511, 512, 530])
def test_topk_group_near_staging_capacity(ag, k):
    """Every one of the top K magnitudes in the first filter group (2 chunks for small inputs):
    its candidate count sits just below, at or past the 512-entry LDS staging (exact slots below,
    the exact path past it).  D <= 16 K: the sample is the whole row, so the candidates are
    exactly the top K."""
    n, d = 3, 16384
    g = np.random.default_rng(k)
    rows = (g.standard_normal((n, d)) * 1e-3).astype(np.float32)
    for i in range(n):
        idx = g.choice(8192, size=k, replace=False)
        rows[i, idx] = (g.standard_normal(k) * 10).astype(np.float32)
    enc = []
    for i in range(n):
        out = np.zeros(d, dtype=np.float32)
        ind = oc.topk_indices(rows[i], k)
        out[ind] = rows[i][ind]
        enc.append(out)
    want = oc.reduce_plain(enc)
    red = ag.UplinkReducer(ag.initCompressor(f"topk:{k}", d))
    assert_bitexact(red(torch.from_numpy(rows).cuda()), want)
