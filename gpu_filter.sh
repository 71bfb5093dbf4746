#!/bin/bash
# filter A/B (ring 8 vs 16) + GPU parity tests + benches
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -rf -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/status.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 2 4; do
  FLC_FILTER_GS=$r timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3_r$r.log 2>&1 || exit $?
done
for wl in c4 reduce; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$wl.log 2>&1 || exit $?
done
exit 0
