"""World-size-2 (and 3) gloo tests of the client sharding + combine path on CPU.

The encoder here is the oracle (the HIP encoder is covered by tests/test_gpu_parity.py); what is
tested is the distributed orchestration: client blocks, client ids per rank (device-RNG keys /
compat stream positions), the partial-sum contract, both combine modes, and that the sharded
result equals the single-process sequential result (bit-exact for 'ordered' when every rank
holds one block; within fp32 reassociation otherwise).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flpytorch_amd.sharding import N_BLOCKS, ShardedUplink, client_block, rank_blocks, rank_clients
from oracle import codecs as oc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_rows(n, d):
    return np.random.default_rng(7).standard_normal((n, d)).astype(np.float32)


def oracle_partial(spec, d):
    def run(rows, client0, out):
        enc = []
        for i in range(rows.shape[0]):
            o = oc.OracleCompressor(spec, d)
            if o.type == oc.TOPK or o.type == oc.IDENTICAL:
                enc.append(o.compress(rows[i].numpy()))
            else:
                raise ValueError("deterministic codecs only in this test")
        acc = enc[0].copy()
        for e in enc[1:]:
            acc = acc + e
        out.copy_(torch.from_numpy(acc))
    return run


def torch_fold(stack, total):
    """The block fold's contract in torch-CPU: sequential fp32 sum in block order, true division."""
    acc = stack[0].clone()
    for b in range(1, stack.shape[0]):
        acc.add_(stack[b])
    return acc.div_(torch.tensor(float(total), dtype=torch.float32))


def _worker(rank, world, port, spec, n, d, mode, replay, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = make_rows(n, d)
    if mode == "ordered":
        lo, hi = rank_clients(n, world, rank)
        up = ShardedUplink(oracle_partial(spec, d), mode=mode, fold=torch_fold)
        if replay:
            out = up(lambda a, b: torch.from_numpy(rows[a:b].copy()), client0=lo, total_weight=float(n), n_clients=n,
                     d=d, device="cpu")
        else:
            out = up(torch.from_numpy(rows[lo:hi].copy()), client0=lo, total_weight=float(n), n_clients=n)
    else:
        lo, hi = client_block(n, world, rank)
        up = ShardedUplink(oracle_partial(spec, d), mode=mode)
        out = up(torch.from_numpy(rows[lo:hi].copy()), client0=lo, total_weight=float(n))
    q.put((rank, out.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, spec, n, d, mode, replay=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, spec, n, d, mode, replay, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("spec", ["topk:5%", "ident"])
def test_sharded_uplink_matches_single_process(world, spec):
    n, d = 7, 4099
    res = _run(world, spec, n, d, "allreduce")
    rows = make_rows(n, d)
    enc = [oc.OracleCompressor(spec, d).compress(rows[i]) for i in range(n)]
    want = oc.reduce_plain(enc)
    for r in range(world):
        np.testing.assert_array_equal(res[r], res[0])            # every rank holds the same result
        np.testing.assert_allclose(res[r], want, rtol=2e-6, atol=1e-7)


def block_fold_want(spec, n, d):
    """(((B_0 + B_1) + ...) + B_7) / n with B_b the client-order sum of block b's encodings."""
    rows = make_rows(n, d)
    enc = [oc.OracleCompressor(spec, d).compress(rows[i]) for i in range(n)]
    parts = []
    for b in range(N_BLOCKS):
        lo, hi = client_block(n, N_BLOCKS, b)
        acc = np.zeros(d, np.float32) if hi == lo else enc[lo].copy()
        for e in enc[lo + 1:hi]:
            acc = acc + e
        parts.append(acc)
    fold = parts[0].copy()
    for p in parts[1:]:
        fold = fold + p
    return fold / np.float32(n)


@pytest.mark.parametrize("spec,n,d", [("topk:5%", 37, 4099), ("ident", 5, 1021), ("ident", 64, 1)])
def test_ordered_mode_is_g_invariant(spec, n, d):
    """the 8 fixed client-block partials folded in block order — G = 1, 2, 4, 8 give
    the same bits on every rank, equal to the stated fold (n = 5: blocks 5..7 empty)."""
    want = block_fold_want(spec, n, d)
    for world in (1, 2, 4, 8):
        res = _run(world, spec, n, d, "ordered")
        for r in range(world):
            assert np.array_equal(res[r].view(np.uint32), want.view(np.uint32)), (world, r)


def test_ordered_mode_replayed_rows():
    """The strong-scaling bench's form: rows(lo, hi) called per block."""
    spec, n, d = "topk:5%", 16, 2053
    want = block_fold_want(spec, n, d)
    res = _run(2, spec, n, d, "ordered", True)
    for r in range(2):
        assert np.array_equal(res[r].view(np.uint32), want.view(np.uint32))


def test_rank_blocks_and_clients():
    assert [list(rank_blocks(4, r)) for r in range(4)] == [[0, 1], [2, 3], [4, 5], [6, 7]]
    with pytest.raises(ValueError):
        rank_blocks(3, 0)
    for n in (0, 5, 37, 4096):
        for world in (1, 2, 4, 8):
            spans = [rank_clients(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    with pytest.raises(ValueError):
        ShardedUplink(lambda *a: None, mode="ordered")


@pytest.mark.parametrize("n,world", [(7, 2), (8, 8), (3, 4), (4096, 8), (1, 1)])
def test_client_blocks_partition(n, world):
    seen = []
    for r in range(world):
        lo, hi = client_block(n, world, r)
        assert 0 <= lo <= hi <= n
        seen.extend(range(lo, hi))
    assert seen == list(range(n))


MIXED_SPECS = ["topk:5%", "ident", "topk:1"]


def _mixed_oracle_partial(d):
    def run(g, rows_g, c0, out):
        acc = None
        for r in rows_g:
            e = oc.OracleCompressor(MIXED_SPECS[g], d).compress(r.numpy())
            acc = e.copy() if acc is None else acc + e
        out.copy_(torch.from_numpy(acc))
    return run


def _mixed_worker(rank, world, port, n, d, q):
    from flpytorch_amd.aggregation.mixed import MixedUplink
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = make_rows(n, d)
    per = n // world
    lo = rank * per
    up = MixedUplink(MIXED_SPECS, d, seed=1, encode_partial=_mixed_oracle_partial(d))
    out = up(torch.from_numpy(rows[lo:lo + per].copy()), client0=lo, group=dist.group.WORLD)
    q.put((rank, out.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_mixed_uplink_two_ranks():
    """C5's combine: per-codec-group partials, each all-reduced asynchronously, summed in group
    order, divided by the global client count — equal on both ranks and to the stated order."""
    world, n, d = 2, 12, 2053
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mixed_worker, args=(r, world, port, n, d, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rows = make_rows(n, d)
    G = len(MIXED_SPECS)
    per = n // world
    parts = []
    for g in range(G):
        rank_sums = []
        for r in range(world):
            acc = None
            for i in range(r * per + g, (r + 1) * per, G):        # global client i uses codec i mod G
                e = oc.OracleCompressor(MIXED_SPECS[g], d).compress(rows[i])
                acc = e.copy() if acc is None else acc + e
            rank_sums.append(acc)
        parts.append(rank_sums[0] + rank_sums[1])
    want = parts[0].copy()
    for p in parts[1:]:
        want = want + p
    want = want / np.float32(n)
    np.testing.assert_array_equal(res[0], res[1])
    np.testing.assert_array_equal(res[0], want)


def test_mixed_uplink_groups():
    from flpytorch_amd.aggregation.mixed import MixedUplink
    up = MixedUplink(["a", "b", "c"], 10, seed=0, encode_partial=lambda *a: None)
    assert up.groups(6, 7) == [([0, 3, 6], 2), ([1, 4], 2), ([2, 5], 2)]
    with pytest.raises(ValueError):
        up.groups(4, 3)
    assert len(set(up.seeds)) == 3


def _mean_bound_check(out, enc, n):
    """SURVEY §8d reduction tolerance: |build - fp64 mean| <= (ceil(log2 N) + 2) 2^-24 mean|.|
    elementwise (mean|.| = the fp64 mean of the encodings' magnitudes at that element)."""
    e64 = np.stack(enc).astype(np.float64)
    mean64 = e64.sum(0) / n
    mabs = np.abs(e64).sum(0) / n
    bound = (int(np.ceil(np.log2(n))) + 2) * 2.0 ** -24 * mabs
    err = np.abs(out.astype(np.float64) - mean64)
    assert np.all(err <= bound), (float((err - bound).max()), int(np.argmax(err - bound)))
    return float((err / np.where(bound > 0, bound, 1.0)).max())


@pytest.mark.parametrize("world,mode", [(2, "allreduce"), (4, "allreduce"), (2, "ordered"), (4, "ordered")])
def test_sharded_mean_within_survey_bound(world, mode):
    """Both combines against the fp64 mean under SURVEY §8d's (ceil(log2 N)+2) 2^-24 bound (not only
    against one process's fp32 result), N = 37 clients over 2 / 4 ranks."""
    spec, n, d = "topk:5%", 37, 4099
    res = _run(world, spec, n, d, mode)
    rows = make_rows(n, d)
    enc = [oc.OracleCompressor(spec, d).compress(rows[i]) for i in range(n)]
    for r in range(world):
        np.testing.assert_array_equal(res[r], res[0])
    used = _mean_bound_check(res[0], enc, n)
    seq = oc.reduce_plain(enc)                                    # the reference's sequential fold
    ulp = int(np.abs(res[0].view(np.int32).astype(np.int64) - seq.view(np.int32).astype(np.int64)).max())
    print(f"world {world} {mode}: max err / bound {used:.3f}, max ulp vs sequential {ulp}")
