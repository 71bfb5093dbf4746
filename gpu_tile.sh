#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 2x2 2x4 1x8 1x4 4x2; do
  FLC_EW_TILE=$v timeout -k 10 200 python bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/tile_$v.log 2>&1 || exit $?
done
exit 0
