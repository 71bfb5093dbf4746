#!/bin/bash
# round-1 evidence pass: default bench (with cpu_baseline), rocprof stats, PMC traffic, e2e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/collect_pmc.py --workload c3 > gpurun_out/pmc_c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/collect_pmc.py --workload c4 > gpurun_out/pmc_c4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_c3 -o run --output-format csv -- \
   python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/stats_c3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_c4 -o run --output-format csv -- \
   python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/stats_c4.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --e2e --workload c3 --n 64 --steps 3 --warmup 1 > gpurun_out/e2e_c3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --e2e --workload c4 --n 64 --steps 3 --warmup 1 > gpurun_out/e2e_c4.log 2>&1 || exit $?
exit 0
