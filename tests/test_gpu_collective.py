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


@pytest.mark.parametrize("nb,d", [(8, 1), (8, 4099), (8, 1 << 20), (3, 1001)])
def test_combine_blocks_single_rank(comm, nb, d):
    """flc_combine_blocks at world size 1 runs the whole multi-rank sequence (slice pack, grouped
    send/recv to itself, block-order fold, all-gather): the result is the sequential fold of the
    block partials / w, bit-exact, and equals sharding.product_fold on the same stack."""
    from flpytorch_amd.sharding import combine_blocks_rccl, product_fold
    g = torch.Generator(device="cuda").manual_seed(nb * 7 + d)
    parts = torch.randn(nb, d, generator=g, device="cuda") * 100
    host = parts.cpu().numpy()
    want = host[0].copy()
    for b in range(1, nb):
        want = want + host[b]
    want = (want / np.float32(37.0)).astype(np.float32)
    got = combine_blocks_rccl(comm, parts, 37.0)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint32), want.view(np.uint32))
    pf = product_fold()(parts, 37.0)
    assert np.array_equal(pf.cpu().numpy().view(np.uint32), want.view(np.uint32))


def test_ordered_uplink_world_one(comm):
    """ShardedUplink(mode='ordered') on the GPU: 8 block partials (HIP encode, divisor 1) folded in
    block order by the HIP fold == the same stated fold computed from per-block fused partials."""
    from flpytorch_amd import aggregation as ag
    from flpytorch_amd.sharding import N_BLOCKS, ShardedUplink, client_block, product_fold, product_partial
    n, d = 21, 50021
    rows = torch.randn(n, d, device="cuda")
    red = ag.UplinkReducer(ag.initCompressor("qsgd:127", d), seed=9)
    up = ShardedUplink(product_partial(red), mode="ordered", fold=product_fold())
    got = up(rows, client0=0, total_weight=float(n), n_clients=n)
    parts = []
    for b in range(N_BLOCKS):
        lo, hi = client_block(n, N_BLOCKS, b)
        parts.append(red(rows[lo:hi], client0=lo, divisor=1.0).cpu().numpy())
    want = parts[0].copy()
    for p in parts[1:]:
        want = want + p
    want = want / np.float32(n)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), want.view(np.uint32))
