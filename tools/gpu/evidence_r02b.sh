#!/bin/bash
# Round-2 (second half) evidence pass on one GPU box: tests, smoke, PMC traffic, rocprof stats,
# bench lines.  Output under gpurun_out/ev3; copy what is judged into profiles/archive/r02b.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/ev3
mkdir -p $out
B="timeout -k 10 400 python bench.py"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -rf > $out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for wl in c3 c4 c2; do
  timeout -k 10 400 python tools/collect_pmc.py --workload $wl > $out/pmc_$wl.log 2>&1 || exit $?
done
for wl in c2 c3 c4 c5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/stats_$wl -o run --output-format csv -- \
     python bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline > $out/stats_$wl.log 2>&1 || exit $?
done
$B > $out/bench_default.log 2>&1 || exit $?
$B --workload c4 > $out/bench_c4.log 2>&1 || exit $?
$B --workload c2 > $out/bench_c2.log 2>&1 || exit $?
$B --workload c5 --steps 5 --warmup 2 > $out/bench_c5.log 2>&1 || exit $?
$B --workload reduce --no-cpu-baseline > $out/bench_reduce.log 2>&1 || exit $?
$B --workload c4 --scaling strong --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_c4_strong.log 2>&1 || exit $?
$B --workload c3 --e2e --steps 5 --warmup 2 > $out/e2e_c3.log 2>&1 || exit $?
exit 0
