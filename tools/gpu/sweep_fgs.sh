#!/bin/bash
# filter item size / staging capacity variants: parity tests under FGS=4, then C4 bench lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/fgs; mkdir -p $out; rm -f $out/sweep.log
FLC_DS_FGS=4 FLC_DS_GCAP=1024 timeout -k 10 300 python -u -m pytest tests/test_gpu_dither_sparse.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit $?
for cfg in "2 512" "4 1024" "4 512" "2 1024" "2 512" "4 1024" "4 512" "2 1024"; do
  set -- $cfg
  FLC_DS_FGS=$1 FLC_DS_GCAP=$2 timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$cfg $(tail -1 $out/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_ms_per_step"], r["achieved"], r["other_kernels_avg_ms"])')" >> $out/sweep.log
done
exit 0
