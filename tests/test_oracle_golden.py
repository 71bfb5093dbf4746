"""Pin the oracle (oracle/) against the real reference's outputs (tests/golden/)."""
import math

import numpy as np
import pytest

from oracle import codecs as oc
from oracle.rng import OracleRandomState
from tests.golden_io import load

CODEC_META, CODEC = load("codecs")
RNG_META, RNG = load("rng")
RUN_META, RUNS = load("runs")


@pytest.mark.parametrize("i", range(len(RNG_META)))
def test_rng_stream(i):
    m = RNG_META[i]
    rs = OracleRandomState(m["seed"])
    want = RNG[f"r{i:02d}"]
    if m["kind"] == "choice":
        got = rs.choice(m["args"][0], m["args"][1])
    elif m["kind"] == "rand":
        got = rs.rand(m["args"][0])
    elif m["kind"] == "random":
        got = np.array([rs.random() for _ in range(m["args"][0])])
    elif m["kind"] == "randint31":
        got = np.array([rs.randint31() for _ in range(m["args"][0])])
    else:  # interleaved DCGD-like sequence
        vals = []
        for _ in range(2):
            vals.extend(rs.choice(10, 4).tolist())
        for _ in range(4):
            vals.extend(rs.choice(2465, 247).tolist())
            vals.append(rs.randint31())
        vals.extend(rs.rand(3).view(np.int64).tolist())
        got = np.array(vals, dtype=np.int64)
    np.testing.assert_array_equal(got, want)
    key, pos = rs.state()
    assert pos == m["end_pos"]
    np.testing.assert_array_equal(key[:8], RNG[f"r{i:02d}_endkey"])


def _case(i):
    m = CODEC_META[i]
    return m, CODEC[f"c{i:02d}_x"], CODEC[f"c{i:02d}_out"]


@pytest.mark.parametrize("i", range(len(CODEC_META)))
def test_codec_constants(i):
    m = CODEC_META[i]
    c = oc.OracleCompressor(m["spec"], m["D"])
    assert c.type == m["type"]
    assert c.K == m["K"]
    assert getattr(c, "w", None) == m["w"]
    assert getattr(c, "alpha", None) == m["alpha"]
    if m["type"] in (5, 6):
        np.testing.assert_array_equal(c.levels, CODEC[f"c{i:02d}_levels"])
        assert c.s == m["s"] and float(c.p) == m["p"]


@pytest.mark.parametrize("i", range(len(CODEC_META)))
def test_codec_outputs(i):
    """Bit-exact outputs, patterns and stats; dithering given the reference's own norm."""
    m, X, OUT = _case(i)
    rs = OracleRandomState(m["seed"])
    stats = CODEC[f"c{i:02d}_stats"]
    pn = CODEC[f"c{i:02d}_pnorm"]
    for c in range(m["n_clients"]):
        comp = oc.OracleCompressor(m["spec"], m["D"])
        comp.generate(rs)
        assert rs.randint31() == m["client_seeds"][c]
        if m["type"] == 3:
            np.testing.assert_array_equal(comp.S, CODEC[f"c{i:02d}_pat{c}"])
        if m["type"] == 2:
            assert comp.testp == CODEC[f"c{i:02d}_pat{c}"][0]
        if m["type"] in (4, 5, 6) and c == 0 and f"c{i:02d}_pat0" in CODEC.files:
            np.testing.assert_array_equal(comp.testp, CODEC[f"c{i:02d}_pat0"])
        x = X[c]
        if m["type"] == 7:
            out = comp.compress(x)
            want = OUT[c]
            # same nonzero set unless the K-th magnitude ties (reference tie order is torch's)
            kth = np.sort(oc.topk_keys(x))[::-1][m["K"] - 1] if m["K"] <= x.size else None
            tied = np.sum(oc.topk_keys(x) == kth) > 1
            if not tied:
                np.testing.assert_array_equal(out, want)
            else:
                np.testing.assert_array_equal(np.sort(np.abs(out)), np.sort(np.abs(want)))
        else:
            out = comp.compress(x, pnorm=(pn[c] if m["type"] in (5, 6) else None))
            np.testing.assert_array_equal(out.view(np.uint32), OUT[c].view(np.uint32))
        # per-call stats (compressors.py:223-224, 367-368); a fresh compressor per client
        assert [comp.total_input_components, comp.really_need_to_send_components,
                comp.last_input_advance, comp.last_need_to_send_advance] == list(stats[c])
    assert [rs.randint31() for _ in range(4)] == m["after_draws"]


@pytest.mark.parametrize("i", [i for i, m in enumerate(CODEC_META) if m["type"] in (5, 6)])
def test_dithering_own_norm(i):
    """With the oracle's own (exactly rounded) norm: outputs equal the reference's up to the
    norm's scale (torch's CPU fp32 norm is not exactly rounded) and rare level flips."""
    m, X, OUT = _case(i)
    rs = OracleRandomState(m["seed"])
    pn = CODEC[f"c{i:02d}_pnorm"]
    for c in range(m["n_clients"]):
        comp = oc.OracleCompressor(m["spec"], m["D"])
        comp.generate(rs)
        rs.randint31()
        mine = comp.norm(X[c])
        rel = abs(float(mine) / pn[c] - 1.0)
        assert rel < 64 * 2.0 ** -24 * max(1.0, math.sqrt(m["D"]) / 8)
        out = comp.compress(X[c])
        want = OUT[c]
        ok = np.isclose(out, want, rtol=4 * rel + 4 * 2.0 ** -24, atol=0)
        # derived flip bound (the bound tests/test_gpu_rows_ref.py uses): element j's
        # keep-probability moves by |dp_j| = y_j rel / gap_j (gap_j: its level interval's width),
        # so the expected flips are E = sum_j min(1, |dp_j|); at most E + 5 sqrt(E) + 3 elements
        # may fall outside the ratio tolerance
        y = np.abs(X[c].astype(np.float64)) / float(mine)
        lv = np.asarray(comp.levels, dtype=np.float64)
        k = np.clip(np.searchsorted(lv, y, side="right") - 1, 0, len(lv) - 2)
        gap = lv[k + 1] - lv[k]
        E = float(np.sum(np.minimum(1.0, y * rel / np.where(gap > 0, gap, np.inf))))
        assert int(np.sum(~ok)) <= E + 5 * math.sqrt(E) + 3, (int(np.sum(~ok)), E)


def _torch_norm_lib():
    import ctypes
    from oracle import rng
    rng._load()
    lib = ctypes.CDLL(rng._LIB_PATH)
    lib.orc_torch_norm2.restype = ctypes.c_float
    lib.orc_torch_norm2.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    return lambda x: np.float32(lib.orc_torch_norm2(np.ascontiguousarray(x, np.float32).ctypes.data, x.size))


@pytest.mark.parametrize("i", [i for i, m in enumerate(CODEC_META) if m["type"] in (5, 6)])
def test_torch_norm_order_vs_reference_norms(i):
    """oracle/torch_norm.c (torch's CPU fp32 2-norm order, compressors.py:272) reproduces every
    norm the reference recorded for its p = 2 dithering cases bit for bit; p = inf (a max) is
    order-free and the exact norm equals it."""
    m, X, OUT = _case(i)
    comp = oc.OracleCompressor(m["spec"], m["D"])
    if comp.p not in (2, math.inf):
        pytest.skip("p = 1: torch's L1 reduction order is not restated (exact norm + stated bound)")
    tn = _torch_norm_lib()
    pn = CODEC[f"c{i:02d}_pnorm"]
    for c in range(m["n_clients"]):
        got = tn(X[c]) if comp.p == 2 else comp.norm(X[c])
        assert np.float32(got).view(np.uint32) == np.float32(pn[c]).view(np.uint32), (c, got, pn[c])


@pytest.mark.parametrize("name", ["qsgd_c4", "qsgd_c4_heavy"])
def test_torch_norm_order_vs_reference_at_25m(name):
    """The same restatement at C4's row size: the reference's recorded torch.norm bits of the
    D = 25 M rows (tests/golden/rows.json pnorm_bits, 14 616 / 12 602 ulp below the exact norm)."""
    import json
    import os
    meta = {e["name"]: e for e in json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rows.json")))}
    e = meta[name]
    g = np.random.default_rng(e["seed"])
    x = g.standard_normal(e["D"], dtype=np.float32)
    if e["dist"] == "heavy":
        x *= np.power(np.float32(10.0), g.uniform(-3.0, 3.0, e["D"]).astype(np.float32))
    assert int(_torch_norm_lib()(x).view(np.uint32)) == e["pnorm_bits"]


@pytest.mark.parametrize("name", sorted(RUN_META))
def test_server_gradient_runs(name):
    """run.py captures (config C1 + DCGD): the sequential fp32 reduction is bit-exact."""
    meta = RUN_META[name]
    for r in range(meta["rounds"]):
        x = RUNS[f"{name}_r{r}_x"]
        models = RUNS[f"{name}_r{r}_models"]
        gs = oc.server_gradient(x, list(models))
        np.testing.assert_array_equal(gs.view(np.uint32), RUNS[f"{name}_r{r}_gs"].view(np.uint32))
        # history scalar (algorithms.py:2220), l2_norm_of_vec = sqrt(sum(g**2)) (mutils.py:395)
        l2 = math.sqrt(float(np.sum(gs.astype(np.float64) ** 2)))
        assert abs(l2 - meta["grad_sgd_server_l2"][r]) <= 1e-6 * meta["grad_sgd_server_l2"][r]
        xb = math.sqrt(float(np.sum(x.astype(np.float64) ** 2)))
        assert abs(xb - meta["x_before_round"][r]) <= 1e-6 * meta["x_before_round"][r]
        if r + 1 < meta["rounds"]:   # global SGD step, lr 1.0: x <- x - 1.0 * gs (model_funcs.py:605)
            nxt = x - np.float32(meta["global_lr"]) * gs
            np.testing.assert_array_equal(nxt, RUNS[f"{name}_r{r+1}_x"])


def test_run_patterns_follow_stream():
    """DCGD randk: the RandK sets drawn inside run.py follow the predicted stream order:
    seed(runtime) -> per-round client sampling -> per client choice(D,K) then randint(2**31)."""
    name = "dcgd_randk10"
    pats = RUNS[f"{name}_patterns"]
    D = RUN_META[name]["D"]
    K = math.ceil(0.1 * D)
    rs = OracleRandomState(456)
    for _ in range(3):
        rs.choice(4, 4)
    k = 0
    for _ in range(3):
        for _ in range(4):
            np.testing.assert_array_equal(rs.choice(D, K), pats[k])
            rs.randint31()
            k += 1


RK_META, RK = load("rank_k")
# Rank-K (compressors.py:336-364) goes through a floating-point SVD: the oracle (numpy LAPACK, fp32)
# and the reference (torch LAPACK, fp32) agree to rounding, not bits.  Tolerance on the error norm,
# relative to the input norm:
RANK_K_RTOL = 1e-5


@pytest.mark.parametrize("i", range(len(RK_META)), ids=[f"{m['spec']}-{m['D']}" for m in RK_META])
def test_rank_k_golden(i):
    m = RK_META[i]
    x, want = RK[f"x{i}"], RK[f"y{i}"]
    comp = oc.OracleCompressor(m["spec"], m["D"])
    assert (comp.A, comp.B, comp.K, comp.alpha) == (m["A"], m["B"], m["K"], m["alpha"])
    out = comp.compress(x)
    assert out.dtype == np.float32 and out.shape == want.shape
    err = float(np.linalg.norm(out.astype(np.float64) - want)) / max(float(np.linalg.norm(x)), 1e-30)
    assert err <= RANK_K_RTOL, err
    assert comp.last_need_to_send_advance == m["need"]


SH_META, SH = load("shift")


@pytest.mark.parametrize("i", range(len(SH_META)), ids=[f"{m['algo']}-{m['spec']}-{m['D']}" for m in SH_META])
def test_shift_step_golden(i):
    """The shift codecs' client step (DIANA / EF21 / MARINA) against the reference codecs driven by
    the algorithms' own torch expressions: bit-exact (dithering given the reference's norm)."""
    from tests.golden_io import shift_fingerprint, shift_inputs
    m = SH_META[i]
    a, b, x3 = shift_inputs(m["seed"], m["D"])
    assert shift_fingerprint(a, b, x3) == m["fingerprint"]
    comp = oc.OracleCompressor(m["spec"], m["D"])
    comp.generate(OracleRandomState(m["seed"]))
    base = {"b": b, "x3": x3, None: None}[m["base"]]
    pn = m["pnorm"] if comp.type in (oc.STD_DITHERING, oc.NAT_DITHERING) else None
    msg, h2 = oc.shift_step(comp, a, b, scale=m["scale"], base=base, alpha=m["alpha"],
                            h=b if m["alpha"] is not None else None, pnorm=pn)
    np.testing.assert_array_equal(msg.view(np.uint32), SH[f"msg{i}"].view(np.uint32))
    if m["alpha"] is not None:
        np.testing.assert_array_equal(h2.view(np.uint32), SH[f"h{i}"].view(np.uint32))
    assert comp.last_need_to_send_advance == m["need"]


@pytest.mark.parametrize("i", range(len(CODEC_META)), ids=[f"{m['spec']}-{m['D']}" for m in CODEC_META])
def test_wire_format_lossless_on_reference_outputs(i):
    """The wire format (oracle/wire.py == wire.hip's layout) reproduces every reference output of
    the golden codec cases bit for bit after pack -> unpack (dithering with the reference's norm)."""
    from oracle import wire
    m, X, OUT = _case(i)
    pn = CODEC[f"c{i:02d}_pnorm"]
    for c in range(m["n_clients"]):
        comp = oc.OracleCompressor(m["spec"], m["D"])
        out = OUT[c]
        p = pn[c] if m["type"] in (5, 6) else None
        pl = wire.pack(comp, out, p)
        assert pl.size == wire.payload_bytes(comp, m["D"]) and pl.size % 16 == 0
        assert pl[12:16].view(np.uint32)[0] == 0                 # no element without a code
        np.testing.assert_array_equal(wire.unpack(comp, pl, m["D"]).view(np.uint32), out.view(np.uint32))
        if m["type"] == 5 and comp.s <= 127:
            assert pl.size <= 16 + m["D"] + 15                   # one byte per element


@pytest.mark.parametrize("i", [i for i, m in enumerate(CODEC_META) if m["type"] == 5])
def test_dithering_closed_form_on_reference_outputs(i, monkeypatch):
    """The closed form the oracle uses above LOOP_MAX_D (oc.dither_levels) reproduces the
    reference's outputs bit for bit too (forced here at the fixtures' sizes)."""
    monkeypatch.setattr(oc, "LOOP_MAX_D", 0)
    m, X, OUT = _case(i)
    rs = OracleRandomState(m["seed"])
    pn = CODEC[f"c{i:02d}_pnorm"]
    for c in range(m["n_clients"]):
        comp = oc.OracleCompressor(m["spec"], m["D"])
        comp.generate(rs)
        rs.randint31()
        out = comp.compress(X[c], pnorm=pn[c])
        np.testing.assert_array_equal(out.view(np.uint32), OUT[c].view(np.uint32))


@pytest.mark.parametrize("spec", ["qsgd:127", "qsgd:4", "std.dithering:10:2", "std.dithering:7:1", "terngrad",
                                  "std.dithering:300:2"])
def test_dithering_closed_form_equals_loop(spec):
    """oc.dither_levels == the level loop of compressors.py:284-291 on inputs that hit every level
    exactly (boundaries are where the loop's later interval overwrites), zeros, the max element
    (y == 1), y just above 1 (a norm rounded below |x|), NaN and inf."""
    g = np.random.default_rng(abs(hash(spec)) % 2 ** 32)
    d = 50_000
    comp = oc.OracleCompressor(spec, d)
    lv = comp.levels
    y = g.random(d).astype(np.float32)
    y[: lv.size] = lv                                           # exact level hits
    y[lv.size: 2 * lv.size] = np.nextafter(lv, np.float32(2))   # one ulp above each level
    y[2 * lv.size: 3 * lv.size] = np.nextafter(lv, np.float32(-1))
    y[-1], y[-2], y[-3], y[-4] = 1.0, np.nextafter(np.float32(1), np.float32(2)), np.nan, np.inf
    u = g.random(d)
    u[: lv.size] = 0.0
    loop = np.zeros_like(y)
    with np.errstate(all="ignore"):
        for s in range(len(lv) - 1):
            c12 = (y >= lv[s]) & (y <= lv[s + 1])
            p = (y - lv[s + 1]) / (lv[s] - lv[s + 1])
            c3 = u < p.astype(np.float64)
            loop[c12 & c3] = lv[s]
            loop[c12 & ~c3] = lv[s + 1]
        fast = oc.dither_levels(y, u, lv)
    np.testing.assert_array_equal(fast.view(np.uint32), loop.view(np.uint32))


def _weighted():
    import json
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(gold, "weighted.json")))
    arr = np.load(os.path.join(gold, "weighted.npz"))
    return meta, arr


def test_oracle_weighted_fold_vs_reference():
    """The oracle's fold with Python-float weights != 1 (w * (x - x_i) in fp32, Python-float total
    as the divisor) equals the reference's DCGD / FedAvg serverGradient on the same inputs."""
    meta, arr = _weighted()
    for m in meta:
        c = m["case"]
        x, rows = arr[f"c{c}_x"], arr[f"c{c}_rows"]
        got = oc.server_gradient(x, list(rows), m["weights"])
        want = arr[f"c{c}_{m['algorithm']}_gs"]
        assert np.array_equal(np.asarray(got, np.float32).view(np.uint32), want.view(np.uint32)), m


@pytest.mark.parametrize("name", ["topk_c3", "topk_c3_heavy", "qsgd_c4", "qsgd_c4_heavy"])
def test_oracle_row_size_vs_reference(name):
    """The oracle against the reference at the config row sizes (tests/golden/rows.*, made by
    make_golden_rows.py): TopK's index set and dense output at D = 10 M; QSGD at D = 25 M given the
    reference's torch norm — the whole output bit-identical — and the oracle's own norm exactly
    rounded (the reference's fp32 torch norm sits `pnorm_ulps_from_exact` ulps from it)."""
    from tests.test_gpu_rows_ref import ARR, CASES, row, sha
    m = CASES[name]
    x = row(m["seed"], m["D"], m["dist"])
    assert sha(x) == m["x_sha"]
    o = oc.OracleCompressor(m["spec"], m["D"])
    if m["spec"].startswith("topk"):
        out = o.compress(x)
        np.testing.assert_array_equal(np.flatnonzero(out), ARR[f"{name}_ind"])
        assert sha(out) == m["out_sha"]
        return
    o.testp = np.random.RandomState(m["pattern_seed"]).rand(m["D"])
    assert sha(o.testp) == m["testp_sha"]
    pref = np.uint32(m["pnorm_bits"]).view(np.float32)
    assert sha(o.compress(x, pnorm=pref)) == m["out_sha"]
    assert int(np.float32(o.norm(x)).view(np.uint32)) == m["exact_norm_bits"]


@pytest.mark.parametrize("kind", ["normal", "ties", "zeros", "nan_inf", "fewnz"])
@pytest.mark.parametrize("d,k", [(1, 1), (17, 5), (4096, 41), (100003, 1000), (50000, 50000)])
def test_oracle_topk_fast_equals_sort(kind, d, k):
    """topk_indices_fast (selection; the large-row GPU tests) is the same set as topk_indices (the
    full lexsort restatement of compressors.py:330-335 with the lowest-index tie rule)."""
    g = np.random.default_rng([d, k, len(kind)])
    x = g.standard_normal(d).astype(np.float32)
    if kind == "ties":
        x = (g.integers(-3, 4, d) * 0.5).astype(np.float32)
    elif kind == "zeros":
        x[:] = 0.0
        x[::97] = 1.0
    elif kind == "nan_inf":
        x[d // 2] = np.inf
        x[d // 3] = -np.nan
    elif kind == "fewnz":
        x[x.size // 50:] = 0.0
    np.testing.assert_array_equal(oc.topk_indices_fast(x, k), oc.topk_indices(x, k))
