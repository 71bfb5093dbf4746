"""GPU parity of the shift codecs (flc_encode_shift): the compressed algorithms'
client step e = C(a - b); msg = base + e * scale; h' = h + alpha * e, in one call.

Bit-exact against the reference's fixtures (tests/golden/shift.*, made by make_golden_shift.py from
the real codecs and the algorithms' torch expressions) where the step does not depend on a norm,
and against the oracle (oracle.codecs.shift_step, exactly rounded norm) for every codec."""
import numpy as np
import pytest
import torch

from oracle import codecs as oc
from oracle import devrng
from oracle.rng import OracleRandomState
from tests.golden_io import load, shift_fingerprint, shift_inputs

pytestmark = pytest.mark.gpu

SH_META, SH = load("shift")
DITHER = (oc.STD_DITHERING, oc.NAT_DITHERING)


@pytest.fixture(scope="module")
def ag():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from flpytorch_amd import aggregation
    return aggregation


def bits(a):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else a
    return np.asarray(a, dtype=np.float32).view(np.uint32)


def assert_bitexact(got, want):
    g, w = bits(got), bits(want)
    if not np.array_equal(g, w):
        bad = np.nonzero(g != w)[0]
        raise AssertionError(f"{bad.size} of {g.size} differ; first {bad[:5]}: {g[bad[:5]]} vs {w[bad[:5]]}")


def run_case(ag, m, a, b, x3, **kw):
    comp = ag.initCompressor(m["spec"], m["D"])
    comp.generateCompressPattern(np.random.RandomState(m["seed"]), "cuda", 0, {})
    ta, tb, t3 = (torch.from_numpy(v.copy()).cuda() for v in (a, b, x3))
    base = {"b": tb, "x3": t3, None: None}[m["base"]]
    if m["alpha"] is not None:
        msg, h2 = comp.compressShift(ta, tb, scale=m["scale"], base=base, alpha=m["alpha"], shift=tb, **kw)
    else:
        msg, h2 = comp.compressShift(ta, tb, scale=m["scale"], base=base, **kw)
    return comp, msg, h2, (ta, tb, t3)


def oracle_case(m, a, b, x3, pnorm=None):
    o = oc.OracleCompressor(m["spec"], m["D"])
    o.generate(OracleRandomState(m["seed"]))
    base = {"b": b, "x3": x3, None: None}[m["base"]]
    return oc.shift_step(o, a, b, scale=m["scale"], base=base, alpha=m["alpha"],
                         h=b if m["alpha"] is not None else None, pnorm=pnorm), o


@pytest.mark.parametrize("i", range(len(SH_META)), ids=[f"{m['algo']}-{m['spec']}-{m['D']}" for m in SH_META])
def test_shift_golden_and_oracle(ag, i):
    m = SH_META[i]
    a, b, x3 = shift_inputs(m["seed"], m["D"])
    assert shift_fingerprint(a, b, x3) == m["fingerprint"]
    comp, msg, h2, _ = run_case(ag, m, a, b, x3)
    (want_msg, want_h), o = oracle_case(m, a, b, x3)
    assert_bitexact(msg, want_msg)
    if m["alpha"] is not None:
        assert_bitexact(h2, want_h)
    else:
        assert h2 is None
    if o.type not in DITHER:                     # no norm involved: the reference's own bits
        assert_bitexact(msg, SH[f"msg{i}"])
        if m["alpha"] is not None:
            assert_bitexact(h2, SH[f"h{i}"])
    assert comp.last_need_to_send_advance == m["need"]
    assert comp.last_input_advance == m["D"]


SPECS = ["ident", "randk:3%", "topk:2%", "natural", "qsgd:127", "nat.dithering:6:2", "rank_k:2"]


@pytest.mark.parametrize("spec", SPECS)
@pytest.mark.parametrize("d", [1, 7, 4096, 100003])
def test_shift_in_place_and_unaligned(ag, spec, d):
    """EF21 writes g_next over g_prev and DIANA h over h (outputs aliasing inputs); views starting
    one element into a buffer take the scalar path.  Same bits as the out-of-place call."""
    if spec.startswith("rank_k") and d in (1, 7):
        pytest.skip("rank_k needs a matrix view")
    g = np.random.default_rng([d, len(spec)])
    a = g.standard_normal(d + 1).astype(np.float32)
    b = (a + g.standard_normal(d + 1)).astype(np.float32)
    seed = 7 + d
    m = dict(spec=spec, D=d, seed=seed, base="b", scale=0.25, alpha=0.75)
    if spec.startswith("rank_k"):
        comp_tol = 5e-5
    else:
        comp_tol = None

    def fresh():
        c = ag.initCompressor(spec, d)
        c.generateCompressPattern(np.random.RandomState(seed), "cuda", 0, {})
        return c
    ta = torch.from_numpy(a).cuda()
    tb = torch.from_numpy(b).cuda()
    # reference: out of place, aligned
    msg_ref, h_ref = fresh().compressShift(ta[:d].clone(), tb[:d].clone(), scale=m["scale"], base=tb[:d].clone(),
                                           alpha=m["alpha"], shift=tb[:d].clone())
    # in place: msg over b (EF21), h over b in a second call (DIANA) — compare each with the reference
    bb = tb[:d].clone()
    fresh().compressShift(ta[:d], bb, scale=m["scale"], base=bb, out=bb)
    hh = tb[:d].clone()
    fresh().compressShift(ta[:d], hh, alpha=m["alpha"], shift=hh, shift_out=hh, message=False)
    # unaligned views
    ua, ub = ta[1:d + 1], tb[1:d + 1]
    au, bu = ua.clone(), ub.clone()      # same data, aligned copies for the comparison
    msg_u, h_u = fresh().compressShift(ua, ub, scale=m["scale"], base=ub, alpha=m["alpha"], shift=ub)
    msg_a, h_a = fresh().compressShift(au, bu, scale=m["scale"], base=bu, alpha=m["alpha"], shift=bu)
    if comp_tol is None:
        assert_bitexact(bb, msg_ref)
        assert_bitexact(hh, h_ref)
        assert_bitexact(msg_u, msg_a)
        assert_bitexact(h_u, h_a)
        # and the oracle
        o = oc.OracleCompressor(spec, d)
        o.generate(OracleRandomState(seed))
        wm, wh = oc.shift_step(o, a[:d], b[:d], scale=m["scale"], base=b[:d], alpha=m["alpha"], h=b[:d])
        assert_bitexact(msg_ref, wm)
        assert_bitexact(h_ref, wh)
    else:
        for x, y in ((bb, msg_ref), (hh, h_ref), (msg_u, msg_a), (h_u, h_a)):
            assert (x - y).norm().item() <= comp_tol * (1.0 + y.norm().item())


@pytest.mark.parametrize("spec", ["qsgd:127", "natural", "randk:1%"])
def test_shift_device_rng(ag, spec):
    """Device-RNG mode: same draws as flc_encode of the difference (oracle restatement of the RNG)."""
    from flpytorch_amd import _lib
    lib = _lib.load()
    d, seed, client = 50001, 99, 5
    g = np.random.default_rng(11)
    a = g.standard_normal(d).astype(np.float32)
    b = g.standard_normal(d).astype(np.float32)
    h = g.standard_normal(d).astype(np.float32)
    o = oc.OracleCompressor(spec, d)
    if o.type == oc.RANDK:
        idx = np.empty(o.K, dtype=np.int64)
        assert lib.flc_device_randk_indices(seed, client, d, o.K, idx.ctypes.data) == 0
        o.S = idx
    else:
        o.testp = devrng.uniforms(seed, client, d)
    wm, wh = oc.shift_step(o, a, b, scale=1.0, base=None, alpha=0.5, h=h)
    c = ag.initCompressor(spec, d)
    c.device_rng = (seed, client)
    msg, h2 = c.compressShift(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda(), alpha=0.5,
                              shift=torch.from_numpy(h).cuda())
    assert_bitexact(msg, wm)
    assert_bitexact(h2, wh)


def test_shift_argument_errors(ag):
    c = ag.initCompressor("qsgd:4", 16)
    x = torch.ones(16, device="cuda")
    with pytest.raises(ValueError):
        c.compressShift(x, x, message=False)
    with pytest.raises(ValueError):
        c.compressShift(x, x, alpha=0.5)
    with pytest.raises(TypeError):
        c.compressShift(x.double(), x)


@pytest.mark.parametrize("spec", ["qsgd:16", "topk:1%", "randk:5%", "natural"])
def test_algorithm_steps(ag, spec):
    """dianaStep / ef21Step / marinaStep == the algorithms' torch expressions over compressVector."""
    d = 30011
    g = np.random.default_rng(3)
    grad, h, gp, gpx = (torch.from_numpy(g.standard_normal(d).astype(np.float32)).cuda() for _ in range(4))

    def comp():
        c = ag.initCompressor(spec, d)
        c.generateCompressPattern(np.random.RandomState(5), "cuda", 0, {})
        return c
    c0 = comp()
    w = c0.getW() if c0.isUnbiasedCompressor() else 0.0
    alpha = 1.0 / (1.0 + w)
    m, h2 = ag.dianaStep(comp(), grad, h, alpha)
    mr = comp().compressVector(grad - h)
    assert_bitexact(m, mr)
    assert_bitexact(h2, h + alpha * mr)
    mult = 1.0 if c0.isContractionCompressor() else 1.0 / (1.0 + c0.getW())
    assert_bitexact(ag.ef21Step(comp(), grad, gp), gp + comp().compressVector(grad - gp) * mult)
    assert_bitexact(ag.marinaStep(comp(), grad, gpx, gp), gp + comp().compressVector(grad - gpx))


def test_arena_views_feed_the_kernels(ag):
    """A model's gradient arena (flpytorch_amd.arena) is read in place by the codecs: the EF21 step
    on grad_view() equals the step on mutils-style concatenated copies."""
    from flpytorch_amd.arena import FlatArena
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 10)).cuda()
    a = FlatArena(m)
    x = torch.randn(32, 64, device="cuda")
    m(x).square().mean().backward()
    g = a.grad_view()
    cat = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    assert g.data_ptr() == a.gflat.data_ptr() and torch.equal(g, cat)
    gp = torch.randn_like(g)

    def comp():
        c = ag.initCompressor("qsgd:8", a.D)
        c.generateCompressPattern(np.random.RandomState(1), "cuda", 0, {})
        return c
    assert_bitexact(ag.ef21Step(comp(), g, gp), ag.ef21Step(comp(), cat, gp))
