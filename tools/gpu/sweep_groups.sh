#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/sweep; mkdir -p $out; rm -f $out/groups.log
for g in 1 4 2 8 1; do
  FLC_DS_GROUPS=$g timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$g $(tail -1 $out/run.log)" >> $out/groups.log
done
exit 0
