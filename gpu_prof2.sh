#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
   python bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || exit $?
for v in 2x2 2x4 4x2; do
  FLC_EW_TILE=$v timeout -k 10 200 python bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/tile_$v.log 2>&1 || exit $?
done
exit 0
