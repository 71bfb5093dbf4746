"""flpytorch_amd.resident (flc_rows_alloc): the resident client-update matrix in one physically
contiguous HBM range.  The memory behaves like any device tensor (the uplink over it gives the same
bits as over a torch allocation), is freed with its tensor, and a request that cannot be served
contiguously falls back to torch's allocator with a warning."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_resident_rows_same_bits_as_torch_allocation():
    from flpytorch_amd import aggregation as ag
    from flpytorch_amd.resident import resident_rows
    n, d = 40, 1_000_003
    rows, kind = resident_rows(n, d)
    assert kind == "contiguous" and rows.shape == (n, d) and rows.is_cuda and rows.dtype == torch.float32
    src = torch.randn(n, d, generator=torch.Generator(device="cuda").manual_seed(3), device="cuda")
    rows.copy_(src)
    for spec in ("qsgd:127", "topk:1%", "randk:1%"):
        red = ag.UplinkReducer(ag.initCompressor(spec, d), seed=11)
        a, b = red(rows), red(src)
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), spec


def test_resident_rows_freed_with_tensor():
    from flpytorch_amd.resident import resident_rows
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    rows, kind = resident_rows(256, 10_000_000)                         # 10.24 GB
    assert kind == "contiguous"
    rows.fill_(1.0)
    assert torch.cuda.mem_get_info()[0] < free0 - 9e9
    del rows
    torch.cuda.synchronize()
    assert torch.cuda.mem_get_info()[0] > free0 - 1e9


def test_resident_rows_fallback_when_too_large():
    from flpytorch_amd import _lib
    lib = _lib.load()
    p = ctypes.c_void_p()
    total = torch.cuda.get_device_properties(0).total_memory
    assert lib.flc_rows_alloc(int(total * 2), 1, ctypes.byref(p)) != 0 and not p.value   # refused, not a crash
    from flpytorch_amd.resident import resident_rows
    with pytest.warns(UserWarning):
        with pytest.raises(torch.cuda.OutOfMemoryError):
            resident_rows(int(total * 2) // (4 * 1_000_000), 1_000_000)     # then torch's allocator refuses too
