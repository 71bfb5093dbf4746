"""flc_combine_partials on a caller-owned RCCL communicator (SURVEY §8b's multi-GPU helper), one
rank on the box's GPU: the collective plumbing, both modes, the division, the workspace contract.
(World sizes > 1 of the same combine logic: tests/test_dist_gloo.py on CPU.)"""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    assert torch.cuda.is_available()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    from flpytorch_amd.sharding import RcclComm
    torch.cuda.set_device(0)
    c = RcclComm()
    yield c
    c.destroy()
    dist.destroy_process_group()


@pytest.mark.parametrize("ordered", [False, True])
@pytest.mark.parametrize("d", [1, 4099, 1 << 20])
def test_combine_single_rank(comm, ordered, d):
    from flpytorch_amd import _lib
    from flpytorch_amd.sharding import combine_partials
    g = torch.Generator(device="cuda").manual_seed(d)
    p = torch.randn(d, generator=g, device="cuda") * 100
    want = (p.cpu().numpy() / np.float32(7.0)).astype(np.float32)      # true fp32 division
    combine_partials(comm, p, 7.0, ordered=ordered)
    torch.cuda.synchronize()
    assert np.array_equal(p.cpu().numpy().view(np.uint32), want.view(np.uint32))
    lib = _lib.load()
    assert lib.flc_combine_workspace_size(comm.ptr, d, 1 if ordered else 0) == (4 * d if ordered else 0)


def test_combine_uplink_end_to_end(comm):
    """encode_reduce with divisor 1.0 then the C-ABI combine == the fused uplink's mean."""
    from flpytorch_amd import aggregation as ag
    from flpytorch_amd.sharding import combine_partials
    n, d = 6, 100003
    rows = torch.randn(n, d, device="cuda")
    red = ag.UplinkReducer(ag.initCompressor("topk:1%", d), seed=5)
    part = red(rows, divisor=1.0)
    combine_partials(comm, part, float(n), ordered=True)
    want = red(rows)
    assert torch.equal(part, want)


def test_combine_rejects_bad_args(comm):
    import ctypes
    from flpytorch_amd import _lib
    lib = _lib.load()
    assert lib.flc_combine_partials(None, None, 10, ctypes.c_float(1.0), 0, None, 0, None) != 0
    p = torch.ones(10, device="cuda")
    assert lib.flc_combine_partials(comm.ptr, ctypes.c_void_p(p.data_ptr()), 10, ctypes.c_float(1.0), 1, None, 0,
                                    None) == 4          # ordered mode without workspace: FLC_ERR_WORKSPACE
