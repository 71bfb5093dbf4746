#!/bin/bash
# fold kernels' UTCL1 (address translation) counters, C4 and C3, one step each
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/pmct; mkdir -p $o
for wl in c4 c3; do
  timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum \
     -d $o/$wl -o run --output-format csv -- python3 bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline > $o/$wl.log 2>&1 || exit 1
done
exit 0
