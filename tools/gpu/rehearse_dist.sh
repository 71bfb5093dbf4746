#!/bin/bash
# Rehearsal of bench.py's multi-rank paths on the one-GPU box: 2 ranks share cuda:0 over gloo
# (RCCL refuses two ranks on one GPU).  Weak scaling (all-reduce) and fixed-N (ordered blocks).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FLC_BENCH_SHARE_GPU=1 FLC_BENCH_BACKEND=gloo
out=gpurun_out/rehearse; mkdir -p $out
R="timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511"
$R bench.py --gpus 2 --steps 3 --warmup 1 --clients 64 --no-cpu-baseline > $out/weak.log 2>&1 || exit $?
$R bench.py --gpus 2 --steps 3 --warmup 1 --workload c4 --clients 64 --scaling strong --no-cpu-baseline > $out/strong.log 2>&1 || exit $?
$R bench.py --gpus 2 --steps 2 --warmup 1 --workload c5 --clients 96 --no-cpu-baseline > $out/c5.log 2>&1 || exit $?
exit 0
