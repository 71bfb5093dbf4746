#!/bin/bash
# GPU tests (all) + bench lines for the listed workloads.  usage: quick2.sh <tag> "<wl> ..." [tests-regex]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-q}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread ${3:+-k "$3"} > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for wl in ${2:-c3 c4}; do
  timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/bench_$wl.log 2>&1 || { tail -20 $out/bench_$wl.log; exit 1; }
  tail -1 $out/bench_$wl.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["config"]["workload"], d["ms_per_step"], d["value"], r["kernel_ms_per_step"], r["frac"], r.get("other_kernels_avg_ms"))'
done
exit 0
