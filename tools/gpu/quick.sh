#!/bin/bash
# quick loop: GPU tests (all) + c3/c4 bench lines.   usage: tools/gpu/quick.sh [tag] [tests-regex]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-q}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread ${2:+-k "$2"} > $out/tests.log 2>&1 || exit $?
for wl in c4 c3; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/bench_$wl.log 2>&1 || exit $?
done
exit 0
