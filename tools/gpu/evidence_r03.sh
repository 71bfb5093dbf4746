#!/bin/bash
# Round-3 evidence pass on one GPU box: tests, smoke, PMC traffic of the dominant kernels, each bench
# line printed under rocprofv3 --kernel-trace --stats of the same command, the other bench lines.
# Output under gpurun_out/ev_r03; copy what is judged into profiles/r03/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${EV_OUT:-ev_r03}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -rf > $out/gpu_tests.log 2>&1 || exit $?
echo "tests: $(tail -1 $out/gpu_tests.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for wl in c3 c4 c2; do
  timeout -k 10 400 python tools/collect_pmc.py --workload $wl > $out/pmc_$wl.log 2>&1 || exit $?
done
echo "pmc done"
# bench lines under rocprofv3 stats of the same command (the line's in-process kernel time and
# rocprof's average for the dominant kernel come from one run)
for wl in c3 c4 c2 c5; do
  st=20; wu=3; [ $wl = c5 ] && { st=5; wu=2; }
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/stats_$wl -o run --output-format csv -- \
     python bench.py --workload $wl --steps $st --warmup $wu > $out/bench_$wl.log 2>&1 || exit $?
  echo "$wl: $(tail -1 $out/bench_$wl.log | cut -c1-200)"
done
B="timeout -k 10 400 python bench.py"
$B > $out/bench_default.log 2>&1 || exit $?
$B --workload c4 --no-cpu-baseline > $out/bench_c4_plain.log 2>&1 || exit $?
$B --workload reduce --no-cpu-baseline > $out/bench_reduce.log 2>&1 || exit $?
$B --workload c4 --compat --n 256 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_c4_compat.log 2>&1 || exit $?
$B --workload c4 --scaling strong --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_c4_strong.log 2>&1 || exit $?
$B --dropin --workload c3 --n 8 --steps 10 --warmup 2 > $out/dropin_c3.log 2>&1 || exit $?
$B --dropin --workload c4 --n 4 --steps 5 --warmup 1 > $out/dropin_c4.log 2>&1 || exit $?
$B --workload c3 --e2e --steps 5 --warmup 2 > $out/e2e_c3.log 2>&1 || exit $?
# same-allocation A/B of this build against the previous one, if that build is present
if [ -f flpytorch_amd/libflcodec_head.so ]; then   # (optional: a previous build for a same-allocation check)
  timeout -k 10 400 python tools/ab_inproc.py --workload c3 --variants head,prod --rounds 3 > $out/inproc_c3.log 2>&1 || exit $?
  timeout -k 10 400 python tools/ab_inproc.py --workload c4 --variants head,prod --rounds 3 > $out/inproc_c4.log 2>&1 || exit $?
fi
exit 0
