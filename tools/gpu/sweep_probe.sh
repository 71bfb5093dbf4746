#!/bin/bash
# k_ds_filter cost breakdown (FLC_DS_PROBE modes; outputs of modes 2-4 are not valid):
#   0 normal, 2 norm only (no candidate test / compaction), 3 no f64 norm (xor), 4 no copy-out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/sweep; mkdir -p $out; rm -f $out/probe.log
for p in ${PROBES:-0 2 3 4 0 2 3 4}; do
  FLC_DS_PROBE=$p timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$p $(tail -1 $out/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_ms_per_step"], r["achieved"])')" >> $out/probe.log
done
exit 0
