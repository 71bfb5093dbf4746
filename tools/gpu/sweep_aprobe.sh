#!/bin/bash
# k_ds_accum cost breakdown (FLC_DS_APROBE modes; outputs of modes 1-3 are not valid)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/sweep; mkdir -p $out; rm -f $out/aprobe.log
for p in 0 7 4 0 7; do
  FLC_DS_APROBE=$p timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$p $(tail -1 $out/run.log)" >> $out/aprobe.log
done
exit 0
