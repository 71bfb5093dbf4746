#!/bin/bash
# Round evidence pass on one GPU box: parity tests, smoke, default bench (with cpu_baseline), the
# other workloads' bench lines, wire / end-to-end lines, rocprof kernel stats for c3 / c4 / c5, PMC
# HBM traffic for c3 / c4.   usage: tools/gpu/evidence.sh [tag]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-ev}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -rf > $out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit $?
for wl in c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats_$wl -o run --output-format csv -- \
     python bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline > $out/stats_$wl.log 2>&1 || exit $?
done
timeout -k 10 300 python tools/collect_pmc.py --workload c3 > $out/pmc_c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/collect_pmc.py --workload c4 > $out/pmc_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 > $out/bench_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > $out/bench_c2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload c5 --steps 5 --warmup 2 > $out/bench_c5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload reduce --no-cpu-baseline > $out/bench_reduce.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 --wire --steps 10 > $out/wire_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 --e2e --wire --steps 5 --warmup 2 > $out/e2e_wire_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c3 --e2e --steps 5 --warmup 2 > $out/e2e_c3.log 2>&1 || exit $?
exit 0
