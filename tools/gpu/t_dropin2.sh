#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/td2; mkdir -p $out
for wl in c4 c2; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/st_$wl -o run --output-format csv -- python bench.py --dropin --workload $wl --steps 3 --warmup 1 > $out/dropin_$wl.log 2>&1 || exit 1
tail -1 $out/dropin_$wl.log
done
