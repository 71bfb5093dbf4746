#!/bin/bash
# same-box A/B of library variants on the C4 shard: VARIANTS="head c d" (libflcodec_<tag>.so), each
# run twice interleaved; one line per run: tag ms_per_step filter_ms other kernels
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/ab; mkdir -p $out; rm -f $out/ab.log
for rep in 1 2; do
  for v in ${VARIANTS:-head c}; do
    FLC_LIB_VARIANT=$v timeout -k 10 300 python bench.py --workload ${WL:-c4} --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
    echo "$v $(tail -1 $out/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_ms_per_step"], r.get("other_kernels_avg_ms"))')" >> $out/ab.log
  done
done
exit 0
