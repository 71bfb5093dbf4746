#!/bin/bash
# chunk-accum column split on short rows: randk / topk parity under the forced modes, C2 lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/abc2; mkdir -p $out; rm -f $out/ab.log
for v in 4 2; do
  FLC_ACCUM_PARTS=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wire.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "randk or topk or unpack" > $out/tests_$v.log 2>&1 || exit $?
done
for v in 1 0 1 0 1 0; do
  FLC_ACCUM_PARTS=$v timeout -k 10 300 python bench.py --workload c2 --steps 50 --warmup 5 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$v $(tail -1 $out/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["other_kernels_avg_ms"])')" >> $out/ab.log
done
for v in 1 0; do
  FLC_ACCUM_PARTS=$v timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "c3 $v $(tail -1 $out/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["other_kernels_avg_ms"])')" >> $out/ab.log
done
exit 0
