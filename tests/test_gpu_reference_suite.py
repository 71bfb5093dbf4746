"""The reference's own codec tests (fl_pytorch/utils/compressors.py:497-536: test_unbiasedness,
test_topk_compressor, test_rankk_compressor), run against the MI355X codecs — compat mode (the
caller's numpy stream, compressVector per draw, like the reference) and device-RNG mode (the fused
uplink over 1000 clients holding the same x)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

UNBIASED = ["ident", "randk:10%", "bernulli:0.5", "natural", "qsgd:10", "nat.dithering:10:2", "std.dithering:10:2"]


@pytest.fixture(scope="module")
def ag():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from flpytorch_amd import aggregation
    return aggregation


@pytest.mark.parametrize("spec", UNBIASED)
def test_unbiasedness_compat(ag, spec):
    """compressors.py:497-512, as written: 1000 patterns from one RandomState, mean within 10 %."""
    gen = np.random.RandomState(1234)
    d = 10000
    c = ag.initCompressor(spec, d)
    torch.manual_seed(0)
    x = torch.rand(d).cuda()
    x_out = torch.zeros(d, device="cuda")
    for _ in range(1000):
        c.generateCompressPattern(gen, "cuda", -1, None)
        x_out += c.compressVector(x)
    x_out /= 1000
    assert ((x_out - x).norm() / x.norm()).item() < 0.1


@pytest.mark.parametrize("spec", ["randk:10%", "natural", "qsgd:10", "std.dithering:10:2"])
def test_unbiasedness_device_rng(ag, spec):
    """The same bound for the device generator: 1000 clients encode one x under their own keys."""
    d, n = 10000, 1000
    torch.manual_seed(0)
    x = torch.rand(d).cuda()
    rows = x.expand(n, d).contiguous()
    out = ag.UplinkReducer(ag.initCompressor(spec, d), seed=99)(rows)
    assert ((out - x).norm() / x.norm()).item() < 0.1
    # and the draws are really independent across clients: the mean's error shrinks ~ 1/sqrt(n)
    out10 = ag.UplinkReducer(ag.initCompressor(spec, d), seed=99)(rows[:10])
    assert ((out - x).norm() / (out10 - x).norm()).item() < 0.5


def test_topk_compressor(ag):
    """compressors.py:515-523."""
    c = ag.initCompressor("topk:50%", 8)
    x_in = torch.tensor([1, 2, 3, 4, 5, 6, 7, -8], dtype=torch.float32).cuda()
    c.generateCompressPattern(np.random.RandomState(), x_in.device, -1, None)
    x_out = c.compressVector(x_in)
    assert (x_out - torch.tensor([0, 0, 0, 0, 5, 6, 7, -8], dtype=torch.float32, device="cuda")).norm() < 0.1


def test_rankk_compressor(ag):
    """compressors.py:526-536."""
    c = ag.initCompressor("rank_k:100%", 8)
    x_in = torch.tensor([1, 2, 3, 4, 5, 6, 7, -8], dtype=torch.float32).cuda()
    c.generateCompressPattern(np.random.RandomState(), x_in.device, -1, None)
    x_out = c.compressVector(x_in)
    assert (x_out - x_in).norm().item() < 0.0001
