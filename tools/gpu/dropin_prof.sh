#!/bin/bash
# kernel durations of the drop-in (one compressVector per client) lines under rocprofv3
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/dropin_prof; mkdir -p $out
for wl in c3 c4; do
  n=8; [ $wl = c4 ] && n=4
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats_$wl -o run --output-format csv -- \
     python bench.py --dropin --workload $wl --n $n --steps 10 --warmup 2 > $out/dropin_$wl.log 2>&1 || exit $?
  grep '^{' $out/dropin_$wl.log | tail -1 | cut -c1-300
done
