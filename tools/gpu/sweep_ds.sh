#!/bin/bash
# sparse-QSGD kernel variants on one box (C4 bench): FLC_DS_GCAP / FLC_DS_GRID
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/sweep; mkdir -p $out; rm -f $out/sweep.log
for cfg in "512 over" "256 over" "1024 over" "512 over" "256 over"; do
  set -- $cfg
  FLC_DS_GCAP=$1 FLC_DS_GRID=$2 timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$1/$2 $(tail -1 $out/run.log)" >> $out/sweep.log
done
exit 0
