#!/bin/bash
# Round-5 evidence pass on one GPU box: the GPU suite, smoke, PMC traffic of the dominant kernels
# (c2, c3, c4 and the c4 compat line), each main bench line under rocprofv3 --kernel-trace --stats of
# the same command, the other lines, and bench.py's own 2-rank launcher (gloo, both ranks on cuda:0).
# Output under gpurun_out/${EV_OUT:-ev_r05}; tools/collect_final.sh copies what is judged to profiles/r05/final/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${EV_OUT:-ev_r05}
mkdir -p $out
# EV_SKIP_TESTS=1: the suite already ran on this build in an earlier call (its log is copied in)
if [ -z "$EV_SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -rf > $out/gpu_tests.log 2>&1 || exit $?
echo "tests: $(tail -1 $out/gpu_tests.log)"
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for wl in c3 c4 c2; do
  timeout -k 10 400 python tools/collect_pmc.py --workload $wl > $out/pmc_$wl.log 2>&1 || exit $?
done
timeout -k 10 500 python tools/collect_pmc.py --workload c4 --compat --n 256 --steps 1 > $out/pmc_c4_compat.log 2>&1 || exit $?
timeout -k 10 400 python tools/collect_pmc.py --dropin --workload c3 --n 8 --steps 5 > $out/pmc_dropin_c3.log 2>&1 || exit $?
timeout -k 10 400 python tools/collect_pmc.py --dropin --workload c4 --n 4 --steps 5 > $out/pmc_dropin_c4.log 2>&1 || exit $?
echo "pmc done"
for wl in c3 c4 c2 c5; do
  st=20; wu=3; [ $wl = c5 ] && { st=5; wu=2; }
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/stats_$wl -o run --output-format csv -- \
     python bench.py --workload $wl --steps $st --warmup $wu > $out/bench_$wl.log 2>&1 || exit $?
  echo "$wl: $(tail -1 $out/bench_$wl.log | cut -c1-200)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/stats_dropin_c3 -o run --output-format csv -- \
   python bench.py --dropin --workload c3 --n 8 --steps 10 --warmup 2 > $out/dropin_c3_prof.log 2>&1 || exit $?
B="timeout -k 10 400 python bench.py"
$B > $out/bench_default.log 2>&1 || exit $?
$B --workload c4 --no-cpu-baseline > $out/bench_c4_plain.log 2>&1 || exit $?
$B --workload reduce --no-cpu-baseline > $out/bench_reduce.log 2>&1 || exit $?
$B --workload c4 --compat --n 256 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_c4_compat.log 2>&1 || exit $?
$B --workload c4 --scaling strong --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_c4_strong.log 2>&1 || exit $?
$B --dropin --workload c3 --n 8 --steps 10 --warmup 2 > $out/dropin_c3.log 2>&1 || exit $?
$B --dropin --workload c4 --n 4 --steps 5 --warmup 1 > $out/dropin_c4.log 2>&1 || exit $?
$B --workload c3 --e2e --steps 5 --warmup 2 > $out/e2e_c3.log 2>&1 || exit $?
FLC_BENCH_SHARE_GPU=1 FLC_BENCH_BACKEND=gloo $B --gpus 2 --steps 3 --warmup 1 --clients 256 --no-cpu-baseline > $out/bench_2rank_rehearsal.log 2>&1 || exit $?
exit 0
