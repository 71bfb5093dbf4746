#!/bin/bash
# C4: fold of row group g beside the filter of group g+1 with the filter grid capped (tuning build)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FLC_LIB_VARIANT=tuning
out=gpurun_out/sweep_gp; mkdir -p $out; rm -f $out/res.log
for cfg in "1 100" "2 100" "2 85" "2 70" "4 100" "4 85" "4 70" "8 85" "1 100"; do
  set -- $cfg
  FLC_DS_GRIDPCT=$2 timeout -k 10 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --row-groups $1 > $out/run.log 2>&1 || exit $?
  echo "$cfg $(python -c "import json;d=json.loads(open('$out/run.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['kernel_ms_per_step'], d['roofline']['other_kernels_avg_ms'])")" >> $out/res.log
done
exit 0
