"""Multi-process uplink on the box's GPU with the HIP encoder (the CPU gloo tests of
tests/test_dist_gloo.py encode with the oracle and so test orchestration only).

Two ranks share cuda:0 over gloo (RCCL refuses two ranks on one device; the 8-GPU RCCL runs are
the driver's).  Each rank encodes its own clients with flc_encode_reduce (device-RNG draws keyed by
the global client id), and the sharded result is compared bit for bit with what one process
computes from the same HIP partials:
  * "ordered" (G-invariant block combine, sharding.py): identical to the single-process ordered
    uplink;
  * "allreduce" (weak scaling): (P0 + P1) / N in fp32, P_r the rank's exact client-order partial.
Then bench.py's own launcher (`python3 bench.py --gpus 2`, no torchrun) is run end to end.
Reference: thread_pool.py:56-67 (thread per device), algorithms.py:1756-1763 (per-client gathers).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 77


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rows(n, d):
    return torch.from_numpy(np.random.default_rng([n, d]).standard_normal((n, d)).astype(np.float32))


def _worker(rank, world, port, spec, n, d, mode, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from flpytorch_amd import aggregation as ag
        from flpytorch_amd.sharding import ShardedUplink, client_block, product_fold, product_partial, rank_clients
        rows = _rows(n, d).cuda()
        red = ag.UplinkReducer(ag.initCompressor(spec, d), device="cuda", seed=SEED)
        if mode == "ordered":
            lo, hi = rank_clients(n, world, rank)
            up = ShardedUplink(product_partial(red), mode="ordered", fold=product_fold())
            out = up(rows[lo:hi], client0=lo, total_weight=float(n), n_clients=n)
        else:
            lo, hi = client_block(n, world, rank)
            up = ShardedUplink(product_partial(red), mode="allreduce")
            out = up(rows[lo:hi], client0=lo, total_weight=float(n))
        torch.cuda.synchronize()
        q.put((rank, out.cpu().numpy().copy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, spec, n, d, mode):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, spec, n, d, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=100) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


def _bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("spec", ["qsgd:127", "topk:1%", "randk:1%"])
@pytest.mark.parametrize("mode", ["ordered", "allreduce"])
def test_two_ranks_hip_encoder(spec, mode):
    from flpytorch_amd import aggregation as ag
    from flpytorch_amd.sharding import ShardedUplink, client_block, product_fold, product_partial
    n, d = 16, 300_007
    res = _run(2, spec, n, d, mode)
    assert np.array_equal(_bits(res[0]), _bits(res[1])), "ranks disagree"
    rows = _rows(n, d).cuda()
    red = ag.UplinkReducer(ag.initCompressor(spec, d), device="cuda", seed=SEED)
    if mode == "ordered":
        up = ShardedUplink(product_partial(red), mode="ordered", fold=product_fold())
        want = up(rows, client0=0, total_weight=float(n), n_clients=n)
    else:
        parts = []
        for r in range(2):
            lo, hi = client_block(n, 2, r)
            parts.append(red(rows[lo:hi], client0=lo, divisor=1.0).clone())
        want = (parts[0] + parts[1]).div_(torch.tensor(float(n), dtype=torch.float32, device="cuda"))
    got = res[0]
    w = want.cpu().numpy()
    bad = np.flatnonzero(_bits(got) != _bits(w))
    assert bad.size == 0, f"{bad.size} of {d} differ, first {bad[:5]}: {got[bad[:5]]} vs {w[bad[:5]]}"
    if spec.startswith("topk"):
        # the HIP-encoded 2-rank mean against the fp64 mean of the oracle's encodings,
        # |build - mean64| <= (ceil(log2 N) + 2) 2^-24 mean|.| elementwise (TopK: deterministic
        # encodings, so the oracle's are the clients' own)
        from oracle import codecs as oc
        rows_h = _rows(n, d).numpy()
        e64 = np.stack([oc.OracleCompressor(spec, d).compress(rows_h[i]) for i in range(n)]).astype(np.float64)
        bound = (int(np.ceil(np.log2(n))) + 2) * 2.0 ** -24 * np.abs(e64).sum(0) / n
        err = np.abs(got.astype(np.float64) - e64.sum(0) / n)
        assert np.all(err <= bound), (float((err - bound).max()), int(np.argmax(err - bound)))


def _bench(args, timeout=200):
    env = dict(os.environ, FLC_BENCH_SHARE_GPU="1", FLC_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_bench_self_launch_two_ranks():
    """`python3 bench.py --gpus 2` without torchrun: the parent starts both ranks (gloo, both on
    cuda:0 for this rehearsal) and exactly one JSON line comes back, from rank 0, with n_gpus 2."""
    line = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--clients", "64", "--dim", "1000000",
                   "--no-cpu-baseline"])
    assert line["n_gpus"] == 2 and line["config"]["clients_total"] == 128
    assert line["scaling"] == "weak" and line["value"] > 0
    # the multi_gpu block: what the process group really was
    mg = line["multi_gpu"]
    assert mg["pg_world_size"] == 2 and mg["backend"] == "gloo" and [r["rank"] for r in mg["ranks"]] == [0, 1]
    assert all(r["device"] == 0 for r in mg["ranks"])          # the rehearsal shares cuda:0
    assert mg["allreduce_bytes"] == 4 * 1_000_000 and mg["allreduce_ms"] > 0


@pytest.mark.timeout(300)
def test_bench_self_launch_strong_c4():
    """--scaling strong --workload c4 through the same launcher (fixed N in 8 blocks, G-invariant)."""
    line = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--workload", "c4", "--scaling", "strong",
                   "--clients", "64", "--dim", "300000", "--no-cpu-baseline"])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["config"]["clients_total"] == 64
