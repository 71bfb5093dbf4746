#!/bin/bash
# Round evidence pass on one GPU box: parity tests, smoke, default bench (with cpu_baseline),
# rocprof kernel stats for c3 / c4, PMC HBM traffic for c3.   usage: tools/gpu/evidence.sh [tag]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-ev}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -rf > $out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit $?
for wl in c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats_$wl -o run --output-format csv -- \
     python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline > $out/stats_$wl.log 2>&1 || exit $?
done
timeout -k 10 300 python tools/collect_pmc.py --workload c3 > $out/pmc_c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/collect_pmc.py --workload c4 > $out/pmc_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 > $out/bench_c4.log 2>&1 || exit $?
exit 0
