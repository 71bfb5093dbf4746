"""TopK tie rule in the ABI: flc_codec_params.tie chooses which of the
entries tied at the K-th magnitude are kept when fewer places are left than ties — FLC_TIE_LOWEST
(default; torch.topk's CPU order on the reference's rows, compressors.py:332) or FLC_TIE_HIGHEST.
Every selection path of select.hip is driven with tied rows under the highest-index rule and checked
bit-exactly against the oracle's topk_indices(tie="highest"), and shown to differ from the lowest-index
result: the many-row fast path's tie cut (k_cand_select / k_cand_select_x), its exact fallback
(exact_row, 512- and 1024-thread workgroups), the few-row spread select (k_cs_pass, list and
histogram modes), the lone compressVector row (k_assign_finish), the dense-K path (k_radix_select
FULLROW + k_topk_filter<EXACT>), both entry points and weights."""
import math

import numpy as np
import pytest
import torch

from oracle import codecs as oc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ag():
    from flpytorch_amd import aggregation
    return aggregation


def _straddle(rows, k, g, places=(1, 3, 6), nties=(6, 9, 12)):
    """Make row i's K-th magnitude tied by extra entries (mixed signs, spread over the row) with only
    places[i % 3] places left at the cut."""
    n, d = rows.shape
    for i in range(n):
        top, nt = places[i % 3] - 1, nties[i % 3]
        mags = np.sort(np.abs(rows[i]))[::-1]
        v = mags[k - 1 - top]
        below = np.flatnonzero(np.abs(rows[i]) < mags[k + 10])
        pos = below[np.linspace(0, len(below) - 1, nt).astype(np.int64)]
        rows[i, pos] = v * np.where(g.random(nt) < 0.5, -1.0, 1.0).astype(np.float32)
    return rows


def _enc(rows, k, tie):
    out = []
    for r in rows:
        e = np.zeros(r.size, dtype=np.float32)
        ind = oc.topk_indices_fast(r, k, tie)
        e[ind] = r[ind]
        out.append(e)
    return out


def _bits(a):
    return np.asarray(a.cpu().numpy() if torch.is_tensor(a) else a, dtype=np.float32).view(np.uint32)


def _comp(ag, spec, d, tie, **kw):
    c = ag.initCompressor(spec, d)
    c.tie_policy = tie
    for a, v in kw.items():
        setattr(c, a, v)
    return c


@pytest.mark.parametrize("n,d,groups", [(256, 300_007, None), (256, 300_007, 2), (3, 2_000_000, None), (5, 10_000_000, None)])
def test_fused_uplink_tie_rules(ag, n, d, groups):
    """Fused encode+reduce of rows whose K-th magnitude is tied across the cut: the fast path's tie
    cut (many rows: per-row-group selects; few rows: k_cs_pass) under both rules."""
    k = math.ceil(0.01 * d)
    g = np.random.default_rng([n, d, 3])
    rows = _straddle(g.standard_normal((n, d)).astype(np.float32), k, g)
    w = [float(v) for v in g.uniform(0.5, 2.0, n)]
    rt = torch.from_numpy(rows).cuda()
    got = {}
    for tie in ("lowest", "highest"):
        comp = _comp(ag, "topk:1%", d, tie, row_groups=groups)
        assert comp.K == k
        red = ag.UplinkReducer(comp)
        enc = _enc(rows, k, tie)
        got[tie] = red(rt)
        np.testing.assert_array_equal(_bits(got[tie]), _bits(oc.reduce_plain(enc)))
        np.testing.assert_array_equal(_bits(red([rt[i] for i in range(n)], weights=w)), _bits(oc.reduce_plain(enc, w)))
        fl = ag.select_row_flags(red.comp, n, d).tolist()
        assert all(f & 4 for f in fl), f"{tie}: expected the fast path's tie cut on every row, flags {sorted(set(fl))}"
    assert not np.array_equal(_bits(got["lowest"]), _bits(got["highest"]))


@pytest.mark.parametrize("kind", ["ties", "fewnz"])
def test_fused_exact_fallback_tie_rules(ag, kind):
    """Rows with more ties at the K-th key than the fast path gathers (or fewer than K nonzeros):
    the exact fallback (exact_row) in the side selects of 128-row groups (512 threads) and in the last
    group (1024 threads) keeps the tie rule."""
    n, d = 256, 300_007
    k = math.ceil(0.01 * d)
    g = np.random.default_rng([len(kind), 9])
    if kind == "ties":
        rows = (g.integers(-3, 4, (n, d)) * 0.5).astype(np.float32)
    else:
        rows = np.zeros((n, d), dtype=np.float32)
        rows[:, ::97] = g.standard_normal((n, len(range(0, d, 97)))).astype(np.float32)
        rows[:, ::3 * 97] = 0.0
    rt = torch.from_numpy(rows).cuda()
    got = {}
    for tie in ("lowest", "highest"):
        red = ag.UplinkReducer(_comp(ag, "topk:1%", d, tie, row_groups=2))
        got[tie] = red(rt)
        np.testing.assert_array_equal(_bits(got[tie]), _bits(oc.reduce_plain(_enc(rows, k, tie))))
        fl = np.asarray(ag.select_row_flags(red.comp, n, d))
        assert np.all(fl & 8), "expected the exact path on every row"
    if kind == "ties":                   # (fewnz: the tied K-th magnitude is 0, both rules add +0)
        assert not np.array_equal(_bits(got["lowest"]), _bits(got["highest"]))


@pytest.mark.parametrize("d,k,ties", [(2_000_003, 20_000, 40), (10_000_000, 100_000, 600), (4_000_000, 40_000, 3000)])
def test_compressvector_tie_rules(ag, d, k, ties):
    """A lone compressVector row (the drop-in), D <= 16.7 M: the register-resident exact select
    (k_lone_resident, flag 16) ranks the ties at the K-th key over the whole grid, any number of
    them, under either rule (F_TIES set, never the exact fallback)."""
    g = np.random.default_rng([d, ties])
    x = g.standard_normal(d).astype(np.float32)
    mags = np.sort(np.abs(x))[::-1]
    v = mags[k - 1 - 7]
    below = np.flatnonzero(np.abs(x) < mags[k + 10])
    pos = below[np.linspace(0, len(below) - 1, ties).astype(np.int64)]
    x[pos] = v * np.where(g.random(ties) < 0.5, -1.0, 1.0).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    outs = {}
    for tie in ("lowest", "highest"):
        c = _comp(ag, f"topk:{k}", d, tie)
        outs[tie] = c.compressVector(xt)
        want = _enc([x], k, tie)[0]
        np.testing.assert_array_equal(_bits(outs[tie]), _bits(want))
        f = int(ag.select_row_flags(c, 1, d)[0])
        assert f & 16 and f & 4 and not f & 8, f"{tie}: flags {f}"
    assert not np.array_equal(_bits(outs["lowest"]), _bits(outs["highest"]))


def test_dense_k_tie_rules(ag):
    """K > D / 16 (the multi-launch exact path: k_radix_select FULLROW, k_tie_count / k_tie_scan,
    k_topk_filter<EXACT>) on tied rows, fused (both entry points) and compressVector."""
    n, d = 4, 100_003
    k = d // 5
    g = np.random.default_rng(17)
    rows = (g.integers(-6, 7, (n, d)) * 0.25).astype(np.float32)
    rt = torch.from_numpy(rows).cuda()
    got = {}
    for tie in ("lowest", "highest"):
        enc = _enc(rows, k, tie)
        red = ag.UplinkReducer(_comp(ag, f"topk:{k}", d, tie))
        got[tie] = red(rt)
        np.testing.assert_array_equal(_bits(got[tie]), _bits(oc.reduce_plain(enc)))
        np.testing.assert_array_equal(_bits(red([rt[i] for i in range(n)])), _bits(oc.reduce_plain(enc)))
        c = _comp(ag, f"topk:{k}", d, tie)
        np.testing.assert_array_equal(_bits(c.compressVector(rt[1])), _bits(enc[1]))
    assert not np.array_equal(_bits(got["lowest"]), _bits(got["highest"]))


def test_tie_rule_validation(ag):
    c = ag.initCompressor("topk:1%", 1000)
    c.tie_policy = "middle"
    with pytest.raises(ValueError):
        c.codec_params(torch.device("cuda"))


@pytest.mark.parametrize("d", [2_000_003, 4_000_001, 10_000_000, 16_777_216, 16_777_217, 1_000])
@pytest.mark.parametrize("kind", ["fewnz", "ties", "normal"])
def test_compressvector_resident_edges(ag, d, kind):
    """The register-resident lone select (k_lone_resident) at its edges: rows whose length is not a
    multiple of 4 (the padding of the straddling float4 is +0, at the end of the index order, and must
    neither count nor be kept when the K-th magnitude is 0: fewnz under the highest-index rule), a
    row of exactly 16 float4 x 4096 x 256 elements and one past it (the list path), and a tiny row
    with K above D / 16 (one workgroup).  Both tie rules, bit-exact vs the oracle."""
    g = np.random.default_rng([d, len(kind)])
    k = max(1, d // 100) if d > 10_000 else 300
    x = g.standard_normal(d).astype(np.float32)
    if kind == "fewnz":
        x[np.argsort(g.random(d))[: d - k // 3]] = 0.0             # fewer nonzeros than K: zeros tie
    elif kind == "ties":
        x = _straddle(x[None, :].copy(), k, g)[0]
    xt = torch.from_numpy(x).cuda()
    for tie in ("lowest", "highest"):
        c = _comp(ag, f"topk:{k}", d, tie)
        got = c.compressVector(xt)
        np.testing.assert_array_equal(_bits(got), _bits(_enc([x], k, tie)[0]), err_msg=f"{tie}")
        f = int(ag.select_row_flags(c, 1, d)[0])
        assert not f & 1, f"{tie}: flags {f} (a barrier gave up)"
        if d <= 16_777_216 and d * 4 < 2**31:
            assert f & 16, f"{tie}: flags {f}, expected the register-resident select"


@pytest.mark.parametrize("where", ["between_pieces", "in_pieces"])
def test_compressvector_resident_speculation_miss(ag, where):
    """k_lone_resident guesses the K-th key's first digit from a fixed sample (32 pieces of 256
    elements spread over the row) and takes both digits from one round when the guess holds.  Rows
    built so that the sample misjudges the row: the large magnitudes only BETWEEN the sampled pieces
    (the sample sees none of them: the guess is far too low), or only INSIDE them (far too high).
    The result must not depend on the guess: bit-exact vs the oracle under both tie rules."""
    d = 4_000_003
    k = 40_000
    g = np.random.default_rng([d, len(where)])
    x = (g.standard_normal(d) * 1e-3).astype(np.float32)
    inside = np.zeros(d, dtype=bool)
    for p in range(32):
        a = p * (d - 256) // 31
        inside[a:a + 256] = True
    pool = np.flatnonzero(~inside if where == "between_pieces" else inside)
    big = g.choice(pool, size=min(2 * k, pool.size), replace=False)
    x[big] = (g.standard_normal(big.size) * 10.0).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    for tie in ("lowest", "highest"):
        c = _comp(ag, f"topk:{k}", d, tie)
        np.testing.assert_array_equal(_bits(c.compressVector(xt)), _bits(_enc([x], k, tie)[0]), err_msg=tie)
        f = int(ag.select_row_flags(c, 1, d)[0])
        assert f & 16 and not f & 1, f"{tie}: flags {f}"


def _debug_resident(mult, spin_ticks):
    from flpytorch_amd import _lib
    _lib.check(_lib.load().flc_debug_resident(mult, spin_ticks), "flc_debug_resident")


@pytest.mark.parametrize("d,kind", [(4_000_003, "normal"), (4_000_003, "ties"), (10_000_000, "normal"),
                                    (2_100_001, "fewnz"), (10_000_000, "ties")])
def test_compressvector_resident_not_coresident(ag, d, kind):
    """k_lone_resident's grid barrier assumes its workgroups are all resident; other kernels (another
    process, RCCL, a long kernel on a caller's stream) can hold CUs.  Forced
    here deterministically: flc_debug_resident(2, 1 ms) launches twice the grid (2 x CUs 1024-thread
    workgroups, one fits a CU), so the resident half waits for workgroups that cannot start, its
    waits give up after 1 ms and abort the call, and the last workgroup out re-selects the row
    exactly (F_REPAIR, 32).  The output must be the oracle's bits under both tie rules — never a
    silent wrong result — and the next call (the control block back to zero) clean and exact."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    g = np.random.default_rng([d, len(kind), 5])
    k = max(1, d // 100)
    x = g.standard_normal(d).astype(np.float32)
    if kind == "fewnz":
        x[np.argsort(g.random(d))[: d - k // 3]] = 0.0
    elif kind == "ties":
        x = _straddle(x[None, :].copy(), k, g, places=(3,), nties=(400,))[0]
    xt = torch.from_numpy(x).cuda()
    g2 = min(2 * cus, -(-d // 4096))
    e4 = -(-d // (g2 * 4096))
    gu = -(-d // (e4 * 4096))                                     # the forced grid (select.hip host code)
    for tie in ("lowest", "highest"):
        want = _bits(_enc([x], k, tie)[0])
        c = _comp(ag, f"topk:{k}", d, tie)
        _debug_resident(2, 100_000)
        try:
            got = c.compressVector(xt)
            torch.cuda.synchronize()
        finally:
            _debug_resident(1, 0)
        np.testing.assert_array_equal(_bits(got), want, err_msg=f"{tie}: forced non-resident grid")
        f = int(ag.select_row_flags(c, 1, d)[0])
        if gu > cus:
            assert f & 16 and f & 32, f"{tie}: flags {f}, expected the repaired resident call ({gu} workgroups, {cus} CUs)"
        # the next call on the default grid: the control block was left clean
        got2 = c.compressVector(xt)
        np.testing.assert_array_equal(_bits(got2), want, err_msg=f"{tie}: the call after a repaired one")
        f2 = int(ag.select_row_flags(c, 1, d)[0])
        assert f2 & 16 and not f2 & 32, f"{tie}: flags {f2} after the repair"


def test_debug_resident_validation(ag):
    from flpytorch_amd import _lib
    lib = _lib.load()
    assert lib.flc_debug_resident(0, 0) != 0
    assert lib.flc_debug_resident(2, -1) != 0
    assert lib.flc_debug_resident(1, 0) == 0


def test_compressvector_under_graph_capture(ag):
    """inside a stream capture a lone TopK compressVector must not use the
    register-resident launch (its call sequence number and cross-stream serialisation are host state
    a replayed graph would not redo): the captured graph runs the list path and every replay gives
    the oracle's bits, also on rows with ties at the K-th key."""
    d, k = 2_000_003, 20_000
    g = np.random.default_rng(41)
    x = _straddle(g.standard_normal(d).astype(np.float32)[None, :].copy(), k, g, places=(2,), nties=(9,))[0]
    xt = torch.from_numpy(x).cuda()
    c = _comp(ag, f"topk:{k}", d, "lowest")
    want = _bits(_enc([x], k, "lowest")[0])
    np.testing.assert_array_equal(_bits(c.compressVector(xt)), want)        # warm: workspace, level tables
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        np.testing.assert_array_equal(_bits(c.compressVector(xt)), want)    # the capture stream's workspace
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        out = c.compressVector(xt)
    for _ in range(3):
        out.zero_()
        graph.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_bits(out), want)


@pytest.mark.parametrize("tie", ["lowest", "highest"])
def test_compressvector_resident_list_overflow(ag, tie):
    """k_lone_resident's candidate finish lists the elements sharing the K-th key's 22-bit prefix:
    each workgroup's first RS_CS (4) in slots of its own, any beyond them in the shared list at an
    offset it reserves.  A row whose prefix group (~700 elements, some exactly tied) sits mostly in
    the first workgroup's slice (600 of them) and partly in another's drives both stores and the
    ranking workgroup's merge of the two: bit-exact vs the oracle, no abort, no repair."""
    d, k = 10_000_000, 100_000
    g = np.random.default_rng(4242)
    x = g.standard_normal(d).astype(np.float32)
    v = np.sort(np.abs(x))[::-1][k - 1 - 300]
    base = np.float32(v).view(np.uint32) & np.uint32(0xFFFFFE00)      # the 22-bit prefix of v
    low = g.integers(0, 512, 650).astype(np.uint32)
    low[::50] = low[0]                                                  # a few exact ties
    mags = (base | low).view(np.float32)
    small = np.abs(x) < 1.0
    first = np.flatnonzero(small[:30_000])[:600]                       # workgroup 0's slice
    other = np.flatnonzero(small[4_000_000:4_030_000])[:50] + 4_000_000
    pos = np.concatenate([first, other])
    x[pos] = mags * np.where(g.random(pos.size) < 0.5, -1.0, 1.0).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    c = _comp(ag, f"topk:{k}", d, tie)
    np.testing.assert_array_equal(_bits(c.compressVector(xt)), _bits(_enc([x], k, tie)[0]), err_msg=tie)
    f = int(ag.select_row_flags(c, 1, d)[0])
    assert f & 16 and not f & 1 and not f & 32, f"{tie}: flags {f}"
