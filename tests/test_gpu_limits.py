"""Size edges on the GPU: empty rows and client sets on every entry point, and one large row
(D = 2^28 + 3, 1 GiB) checked through size-independent properties (TopK: exactly K survivors, every
survivor at least as large as every dropped element; RandK: K survivors scaled by D/K; QSGD: every
output a signed multiple of norm/s, the norm exact; the fold: linearity)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ag():
    assert torch.cuda.is_available()
    from flpytorch_amd import aggregation
    return aggregation


@pytest.mark.parametrize("spec", ["ident", "topk:1", "randk:1", "qsgd:4", "natural", "bernulli:0.5", "rank_k:1"])
def test_empty_inputs(ag, spec):
    d = 16
    red = ag.UplinkReducer(ag.initCompressor(spec, d), seed=1)
    out = red(torch.empty(0, d, device="cuda"))
    assert out.shape == (d,) and torch.count_nonzero(out).item() == 0
    assert ag.reduce_rows(torch.ones(d, device="cuda"), []).abs().sum().item() == 0


def test_large_row_properties(ag):
    d = (1 << 28) + 3
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(d, generator=g, device="cuda")
    # TopK 0.1 %
    c = ag.initCompressor("topk:0.1%", d)
    out = c.compressVector(x)
    sel = out != 0
    assert int(sel.sum().item()) == c.K
    assert torch.equal(out[sel], x[sel])
    assert x[sel].abs().min().item() >= x[~sel].abs().max().item()
    del out, sel
    # RandK 0.1 % (device draws): K survivors, each (D/K) x
    c = ag.initCompressor("randk:0.1%", d)
    c.device_rng = (5, 0)
    out = c.compressVector(x)
    sel = out != 0
    assert int(sel.sum().item()) == c.K
    scale = np.float32(d / c.K)
    assert torch.equal(out[sel], x[sel] * float(scale))
    del out, sel
    # QSGD s = 127 (device draws): every value is level * sign * norm with the exact norm
    c = ag.initCompressor("qsgd:127", d)
    c.device_rng = (5, 0)
    pn = torch.empty(1, device="cuda")
    out = c._encode_gpu(x, pnorm_out=pn)
    norm = float(np.float32(np.sqrt(np.sum(x.double().square().cpu().numpy()))))
    assert pn.item() == norm
    lev = (out.abs() / pn).cpu().numpy() * 127.0
    assert np.max(np.abs(lev - np.round(lev))) < 1e-3
    assert torch.equal(torch.sign(out[out != 0]), torch.sign(x[out != 0]))


def test_large_fold_linearity(ag):
    d = (1 << 27) + 1
    g = torch.Generator(device="cuda").manual_seed(12)
    rows = [torch.randn(d, generator=g, device="cuda") for _ in range(3)]
    x = torch.zeros(d, device="cuda")
    a = ag.reduce_rows(x, rows, relative=False)
    b = ag.reduce_rows(x, [r * 2.0 for r in rows], relative=False)      # x 2 is exact in fp32
    assert torch.equal(b, a * 2.0)
