#!/bin/bash
# k_ds_filter cost breakdown (FLC_DS_PROBE modes; results of modes 1-3 are not valid outputs)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/sweep; mkdir -p $out; rm -f $out/probe.log
for p in 0 6 4 0 6 4; do
  FLC_DS_PROBE=$p timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$p $(tail -1 $out/run.log)" >> $out/probe.log
done
exit 0
