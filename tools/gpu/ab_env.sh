#!/bin/bash
# A/B of an env knob on one box: tests under B, then alternating bench lines.
#   usage: ab_env.sh <VAR> <A> <B> <workload> [test-regex]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
var=$1; a=$2; b=$3; wl=$4; rx=$5
out=gpurun_out/ab_$var; mkdir -p $out; rm -f $out/ab.log
if [ -n "$rx" ]; then
  env $var=$b timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$rx" > $out/tests.log 2>&1 || exit $?
fi
for v in $a $b $a $b $a $b; do
  env $var=$v timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$v $(tail -1 $out/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_ms_per_step"], r["other_kernels_avg_ms"])')" >> $out/ab.log
done
exit 0
