#!/bin/bash
# Round-2 final evidence pass on one GPU box.  Every bench line runs under
# `rocprofv3 --kernel-trace --stats` (the stats are of the same command as the line); PMC
# traffic in separate passes.  Output under gpurun_out/ev4; copy what is judged into profiles/r02b.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${EV_OUT:-ev4}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -rf > $out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for wl in c3 c4 c2; do
  timeout -k 10 400 python tools/collect_pmc.py --workload $wl > $out/pmc_$wl.log 2>&1 || exit $?
done
P="timeout -k 10 500 rocprofv3 --kernel-trace --stats -o run --output-format csv"
$P -d $out/st_default -- python bench.py > $out/bench_default.log 2>&1 || exit $?
$P -d $out/st_c4 -- python bench.py --workload c4 > $out/bench_c4.log 2>&1 || exit $?
$P -d $out/st_c2 -- python bench.py --workload c2 > $out/bench_c2.log 2>&1 || exit $?
$P -d $out/st_c5 -- python bench.py --workload c5 --steps 5 --warmup 2 > $out/bench_c5.log 2>&1 || exit $?
$P -d $out/st_reduce -- python bench.py --workload reduce --no-cpu-baseline > $out/bench_reduce.log 2>&1 || exit $?
$P -d $out/st_c4_strong -- python bench.py --workload c4 --scaling strong --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_c4_strong.log 2>&1 || exit $?
$P -d $out/st_dropin_c3 -- python bench.py --dropin --workload c3 --steps 5 --warmup 2 > $out/dropin_c3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c3 --e2e --steps 5 --warmup 2 > $out/e2e_c3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 --e2e --wire --steps 5 --warmup 2 > $out/e2e_wire_c4.log 2>&1 || exit $?
exit 0
