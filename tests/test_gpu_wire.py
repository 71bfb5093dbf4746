"""GPU parity of the wire format (flc_pack / flc_unpack / flc_unpack_reduce):
payload bytes == the oracle's restatement of the layout (oracle/wire.py) packed from the oracle's
encode, unpack(pack(x)) == flc_encode(x) bit for bit, and the server's decode + reduce from the N
payloads == flc_encode_reduce of the rows."""
import numpy as np
import pytest
import torch

from oracle import codecs as oc
from oracle import wire
from oracle.rng import OracleRandomState

pytestmark = pytest.mark.gpu

SPECS = ["ident", "bernulli:0.5", "randk:1%", "topk:1%", "topk:5", "natural", "qsgd:127", "qsgd:4",
         "std.dithering:300", "terngrad", "std.dithering:8:1", "nat.dithering:6:2"]


@pytest.fixture(scope="module")
def ag():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from flpytorch_amd import aggregation
    return aggregation


def bits(a):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else a
    return np.asarray(a).view(np.uint32)


def rows_for(n, d, seed):
    g = np.random.default_rng(seed)
    r = (g.standard_normal((n, d)) * 10.0 ** g.uniform(-2, 2, (n, d))).astype(np.float32)
    r[:, :min(5, d)] = 0.0
    if d > 5:
        r[:, 5] = -0.0
    return r


@pytest.mark.parametrize("spec", SPECS)
@pytest.mark.parametrize("d", [1, 7, 4099, 100003])
def test_pack_matches_oracle_and_round_trips(ag, spec, d):
    x = rows_for(1, d, d)[0]
    comp = ag.initCompressor(spec, d)
    if spec.startswith("topk") and comp.K > d:
        with pytest.raises(ValueError):           # torch.topk(x, K > D) raises in the reference too
            comp.compressPayload(torch.from_numpy(x).cuda())
        return
    comp.generateCompressPattern(np.random.RandomState(11), "cuda", 0, {})
    o = oc.OracleCompressor(spec, d)
    o.generate(OracleRandomState(11))
    out = o.compress(x)
    pn = o.norm(x) if o.type in (oc.STD_DITHERING, oc.NAT_DITHERING) else None
    want = wire.pack(o, out, pn)
    xt = torch.from_numpy(x).cuda()
    pl = comp.compressPayload(xt)
    assert pl.numel() == want.size == comp.payloadBytes(d)
    assert np.array_equal(pl.cpu().numpy(), want)
    back = comp.decompressPayload(pl, d)
    assert np.array_equal(bits(back), bits(out))
    comp2 = ag.initCompressor(spec, d)
    comp2.generateCompressPattern(np.random.RandomState(11), "cuda", 0, {})
    assert np.array_equal(bits(back), bits(comp2.compressVector(xt)))
    assert comp.last_need_to_send_advance == comp2.last_need_to_send_advance


@pytest.mark.parametrize("spec", SPECS)
@pytest.mark.parametrize("n,d", [(5, 4099), (3, 300001)])
def test_unpack_reduce_equals_encode_reduce(ag, spec, n, d):
    rows = rows_for(n, d, n * d)
    w = list(np.random.default_rng(n).uniform(0.5, 2.0, n))
    seed = 2024
    pls, dense = [], []
    rs = np.random.RandomState(seed)
    comps = []
    for i in range(n):
        c = ag.initCompressor(spec, d)
        c.generateCompressPattern(rs, "cuda", 0, {})
        rs.randint(2 ** 31)
        comps.append(c)
    for i in range(n):
        pls.append(comps[i].compressPayload(torch.from_numpy(rows[i]).cuda()))
        dense.append(comps[i].decompressPayload(pls[i], d))
    ld = pls[0].numel()
    mat = torch.stack(pls)
    red = ag.PayloadReducer(comps[0])
    got = red(mat, d=d, weights=w)
    got2 = red(pls, d=d, weights=w)
    # the sequential fold of the decoded rows (oracle arithmetic on the GPU's decodes)
    acc = None
    for i in range(n):
        t = (np.float32(w[i]) * dense[i].cpu().numpy()).astype(np.float32)
        acc = t if acc is None else (acc + t).astype(np.float32)
    tot = w[0]
    for v in w[1:]:
        tot += v                                  # the reducers sum the weights in Python floats
    want = (acc / np.float32(tot)).astype(np.float32)
    assert mat.stride(0) == ld
    if oc.OracleCompressor(spec, d).type in (oc.RANDK, oc.TOPK):
        # chunk-owner fold: -0 sums become +0 (signed zero) — compare values
        np.testing.assert_array_equal(got.cpu().numpy(), want)
    else:
        assert np.array_equal(bits(got), bits(want))
    assert np.array_equal(bits(got), bits(got2))


def test_payload_sizes(ag):
    d = 25_000_000
    assert ag.initCompressor("qsgd:127", d).payloadBytes() == 16 + d            # 1 byte per element
    assert ag.initCompressor("topk:1%", d).payloadBytes() == 16 + 8 * 250000
    assert ag.initCompressor("natural", d).payloadBytes() == 16 + 2 * d


@pytest.mark.parametrize("spec,d", [("rank_k:3", 2465), ("rank_k:8", 65536), ("rank_k:50", 12), ("rank_k:4", 97)])
def test_rank_k_payload(ag, spec, d):
    """Rank-K messages are the K' (A + B) factor values (compressors.py:362): decode == the encode bit
    for bit (one GEMM shape), the server fold from payloads == the fused uplink to fp32 rounding."""
    g = torch.Generator(device="cuda").manual_seed(d)
    rows = torch.randn(4, d, generator=g, device="cuda")
    comp = ag.initCompressor(spec, d)
    k = min(comp.K, comp.A, comp.B)
    assert comp.payloadBytes() == wire.payload_bytes(oc.OracleCompressor(spec, d), d)
    assert comp.payloadBytes() >= 16 + 4 * k * (comp.A + comp.B)
    pls = [comp.compressPayload(rows[i]) for i in range(4)]
    assert comp.last_need_to_send_advance == k * (comp.A + comp.B)
    hdr = pls[0][:16].cpu().numpy().view(np.uint32)
    assert hdr[0] == 6 and hdr[1] == k
    for i in range(4):
        dec = comp.decompressPayload(pls[i], d)
        assert np.array_equal(bits(dec), bits(ag.initCompressor(spec, d).compressVector(rows[i])))
    got = ag.PayloadReducer(comp)(torch.stack(pls), d=d)
    want = ag.UplinkReducer(ag.initCompressor(spec, d))(rows)
    assert (got - want).norm().item() <= 1e-6 * (1.0 + want.norm().item())
    got2 = ag.PayloadReducer(comp)(pls, d=d)
    assert np.array_equal(bits(got), bits(got2))
