#!/bin/bash
# C3 run-to-run check on one box: default bench twice, with per-step times, and a rocprof stats run
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/c3var; mkdir -p $out
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --step-times > $out/b$k.log 2> $out/b$k.err || exit $?
done
timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --step-times > $out/b60.log 2> $out/b60.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/stats.log 2>&1 || exit $?
exit 0
