"""bench.py's own rank launcher (`python3 bench.py --gpus G` without torchrun), on CPU.

launch_ranks() starts G children with torch.distributed.run's environment contract and propagates
their exit status; a failed rank must take the others down instead of leaving them waiting in a
collective.  The GPU end-to-end run is tests/test_gpu_dist.py::test_bench_self_launch_*.
"""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_ranks_get_the_rendezvous_environment(tmp_path):
    out = tmp_path / "env"
    code = ("import os, json; k = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT'];"
            f"open(r'{out}' + os.environ['RANK'], 'w').write(json.dumps({{x: os.environ[x] for x in k}}))")
    assert bench.launch_ranks(3, [sys.executable, "-c", code]) == 0
    envs = [json.loads((tmp_path / f"env{r}").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] and [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"} and {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_failed_rank_ends_the_job():
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(120)"
    t0 = time.monotonic()
    assert bench.launch_ranks(2, [sys.executable, "-c", code], grace_s=5.0) == 3
    assert time.monotonic() - t0 < 30


def test_killed_rank_reports_its_signal():
    code = "import os, signal; r = int(os.environ['RANK']); os.kill(os.getpid(), signal.SIGKILL) if r == 0 else None"
    assert bench.launch_ranks(2, [sys.executable, "-c", code]) == 128 + 9


def test_ranks_rendezvous_over_gloo():
    code = ("import torch, torch.distributed as dist; dist.init_process_group('gloo');"
            "t = torch.ones(4) * (dist.get_rank() + 1); dist.all_reduce(t);"
            "assert t.tolist() == [3.0] * 4, t; dist.destroy_process_group()")
    assert bench.launch_ranks(2, [sys.executable, "-c", code]) == 0


@pytest.mark.timeout(180)
def test_bench_without_gpu_fails_loudly_not_hangs():
    """The real entry point through the launcher on a host without a GPU: every rank fails at its
    first device call, the parent returns non-zero and prints no result line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["FLC_BENCH_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=170)
    if p.returncode == 0:
        pytest.skip("a GPU is visible here")
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


def test_dist_info_fields_over_gloo(tmp_path):
    """bench.dist_info (the multi_gpu block of a G > 1 bench line) on two gloo
    ranks with CPU tensors: the group's world size and backend, one entry per rank, the exchange's
    bytes and timing — the same function the GPU line calls over RCCL."""
    out = tmp_path / "info.json"
    code = ("import json, sys, torch, torch.distributed as dist; sys.path.insert(0, r'%s'); import bench;"
            "dist.init_process_group('gloo');"
            "i = bench.dist_info(dist, torch.device('cpu'), 1000, reps=2);"
            "(open(r'%s', 'w').write(json.dumps(i)) if dist.get_rank() == 0 else None);"
            "dist.destroy_process_group()") % (ROOT, out)
    assert bench.launch_ranks(2, [sys.executable, "-c", code]) == 0
    info = json.loads(out.read_text())
    assert info["pg_world_size"] == 2 and info["backend"] == "gloo" and info["rccl_version"] is None
    assert [r["rank"] for r in info["ranks"]] == [0, 1]
    assert info["allreduce_bytes"] == 4000 and info["allreduce_ms"] > 0 and info["allreduce_busbw_GBps"] > 0
    assert info["distinct_devices"] == 1          # CPU tensors: no device to tell the ranks apart


_STRONG_CODE = (
    "import json, sys, torch, torch.distributed as dist; sys.path.insert(0, r'%s'); import bench;"
    "dist.init_process_group('gloo');"
    "d = 1000; rows = torch.from_numpy(__import__('numpy').random.default_rng(3).standard_normal((4, d)).astype('float32'));"
    # a toy encode whose partial depends on the client ids (as the device-RNG draws do)
    "enc = lambda r, c0, out: out.copy_(sum(r[i] * float(1 + (c0 + i) %% 7) for i in range(r.shape[0])));"
    "fold = lambda st, tot: (lambda a: [a.add_(st[b]) for b in range(1, st.shape[0])] and a.div_(torch.tensor(float(tot))))(st[0].clone());"
    "b = bench.strong_block(enc, fold, rows, 32, d, torch.device('cpu'), steps=2, warmup=1, group=dist.group.WORLD);"
    "(open(r'%s', 'w').write(json.dumps(b)) if dist.get_rank() == 0 else None);"
    "dist.destroy_process_group()")


@pytest.mark.parametrize("world", [2, 4])
def test_strong_block_digest_is_g_invariant(tmp_path, world):
    """bench.strong_block (the strong_c4 block of every default line) over gloo
    with CPU tensors: 32 clients in 8 fixed blocks of 4 resident rows replayed per block with the
    block's client ids, the ordered combine — the result digest at G = world equals G = 1's, and
    the block reports G, the clients per rank, the step time and the whole-job rate."""
    outs = {}
    for g in (1, world):
        out = tmp_path / f"strong{g}.json"
        assert bench.launch_ranks(g, [sys.executable, "-c", _STRONG_CODE % (ROOT, out)]) == 0
        outs[g] = json.loads(out.read_text())
    assert outs[1]["result_sha256"] == outs[world]["result_sha256"]
    assert outs[1]["n_gpus"] == 1 and outs[world]["n_gpus"] == world
    assert outs[1]["clients_per_gpu"] == 32 and outs[world]["clients_per_gpu"] == 32 // world
    for b in outs.values():
        assert b["ms_per_step"] > 0 and b["value_GBps"] > 0 and b["clients_total"] == 32
