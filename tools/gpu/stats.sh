#!/bin/bash
# kernel-trace stats of one workload: ./gpu_stats.sh <wl>
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
wl=${1:-c3}
rm -rf gpurun_out/prof_$wl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$wl -o run --output-format csv -- \
    python bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$wl.log 2>&1
