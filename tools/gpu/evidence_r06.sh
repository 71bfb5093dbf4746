#!/bin/bash
# Round-6 evidence pass on one GPU box: the GPU suite, smoke, PMC traffic of the dominant kernels
# (c2, c3, c4, c5, the c4 compat line, both drop-in kernels; every pass records its rows, D and
# launches per step), each main bench line under rocprofv3 --kernel-trace --stats of the same
# command, the other lines (the default line carries strong_c4: C4 at fixed N=4096), the drop-in
# QSGD with the reference's torch-order norm, and bench.py's own 2-rank launcher (gloo, both ranks
# on cuda:0) whose strong_c4 digest must equal the 1-GPU line's.
# Output under gpurun_out/${EV_OUT:-ev_r06}; tools/collect_final.sh copies it to profiles/r06/<dst>.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${EV_OUT:-ev_r06}
mkdir -p $out
if [ -z "$EV_SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -rf > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
echo "tests: $(tail -1 $out/gpu_tests.log)"
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
if [ -z "$EV_SKIP_PMC" ]; then
for wl in c3 c4 c2; do
  timeout -k 10 400 python tools/collect_pmc.py --workload $wl > $out/pmc_$wl.log 2>&1 || exit $?
done
timeout -k 10 600 python tools/collect_pmc.py --workload c5 --steps 1 > $out/pmc_c5.log 2>&1 || exit $?
timeout -k 10 600 python tools/collect_pmc.py --workload c5 --steps 1 --kernel k_randk_fold --tag c5_randk > $out/pmc_c5_randk.log 2>&1 || exit $?
timeout -k 10 500 python tools/collect_pmc.py --workload c4 --compat --n 256 --steps 1 > $out/pmc_c4_compat.log 2>&1 || exit $?
timeout -k 10 400 python tools/collect_pmc.py --dropin --workload c3 --n 8 --steps 5 > $out/pmc_dropin_c3.log 2>&1 || exit $?
timeout -k 10 400 python tools/collect_pmc.py --dropin --workload c4 --n 4 --steps 5 > $out/pmc_dropin_c4.log 2>&1 || exit $?
echo "pmc done"
fi
[ -n "$EV_STOP_AFTER_PMC" ] && exit 0
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
$B --dropin --workload c4 --n 4 --steps 3 --warmup 1 --norm-mode torch_cpu > $out/dropin_c4_torchnorm.log 2>&1 || exit $?
$B --workload c3 --e2e --steps 5 --warmup 2 > $out/e2e_c3.log 2>&1 || exit $?
FLC_BENCH_SHARE_GPU=1 FLC_BENCH_BACKEND=gloo $B --gpus 2 --steps 3 --warmup 1 --clients 256 --no-cpu-baseline > $out/bench_2rank_rehearsal.log 2>&1 || exit $?
python3 - $out <<'PY'
import json, sys
o = sys.argv[1]
last = lambda f: json.loads([l for l in open(f"{o}/{f}") if l.startswith("{")][-1])
a, b = last("bench_default.log").get("strong_c4"), last("bench_2rank_rehearsal.log").get("strong_c4")
print("strong_c4 G=1", a and a["ms_per_step"], a and a["result_sha256"][:16], "| G=2 rehearsal", b and b["ms_per_step"],
      b and b["result_sha256"][:16], "| digests equal:", bool(a and b and a["result_sha256"] == b["result_sha256"]))
PY
exit 0
