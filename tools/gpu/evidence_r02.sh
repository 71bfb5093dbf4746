#!/bin/bash
# Round-2 evidence pass on one GPU box (see tools/gpu/evidence.sh for round 1)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/ev2
mkdir -p $out
B="timeout -k 10 400 python bench.py"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -rf > $out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for wl in c2 c5; do
  timeout -k 10 400 python tools/collect_pmc.py --workload $wl > $out/pmc_$wl.log 2>&1 || exit $?
done
timeout -k 10 400 python tools/collect_pmc.py --workload c5 --kernel k_randk_fold --tag c5_randk > $out/pmc_c5_randk.log 2>&1 || exit $?
$B > $out/bench_default.log 2>&1 || exit $?
for wl in c2 c3 c4 c5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/stats_$wl -o run --output-format csv -- \
     python bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline > $out/stats_$wl.log 2>&1 || exit $?
done
$B --workload c4 > $out/bench_c4.log 2>&1 || exit $?
$B --workload c2 > $out/bench_c2.log 2>&1 || exit $?
$B --workload c5 --steps 5 --warmup 2 > $out/bench_c5.log 2>&1 || exit $?
$B --workload reduce --no-cpu-baseline > $out/bench_reduce.log 2>&1 || exit $?
$B --workload c2 --compat --no-cpu-baseline > $out/bench_c2_compat.log 2>&1 || exit $?
$B --workload c4 --compat --n 256 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_c4_compat.log 2>&1 || exit $?
$B --workload c4 --scaling strong --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_c4_strong.log 2>&1 || exit $?
$B --workload c3 --scaling strong --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_c3_strong.log 2>&1 || exit $?
$B --workload c4 --wire --steps 10 > $out/wire_c4.log 2>&1 || exit $?
$B --workload c4 --e2e --wire --steps 5 --warmup 2 > $out/e2e_wire_c4.log 2>&1 || exit $?
$B --workload c3 --e2e --steps 5 --warmup 2 > $out/e2e_c3.log 2>&1 || exit $?
for wl in c3 c4 c2; do
  $B --dropin --workload $wl --steps 5 --warmup 2 > $out/dropin_$wl.log 2>&1 || exit $?
done
exit 0
