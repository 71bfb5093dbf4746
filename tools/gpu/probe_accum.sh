#!/bin/bash
# k_chunk_accum cost breakdown at C3 (FLC_ACCUM_PROBE: 1 no tile adds, 2 no list loads; outputs invalid)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/pacc; mkdir -p $out; rm -f $out/p.log
for v in 0 1 2 0 1 2; do
  FLC_ACCUM_PROBE=$v timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$v $(tail -1 $out/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["other_kernels_avg_ms"]["k_chunk_accum"])')" >> $out/p.log
done
exit 0
