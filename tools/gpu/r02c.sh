#!/bin/bash
# RandK device-mode rework: counts kernel first (no data-dependent addressing), then the fold tests,
# the whole GPU suite, c2 / c5 bench lines + rocprof stats for c5
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r02c; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_randk_device.py -x -v -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k counts_kernel > $out/tests_counts.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_randk_device.py -x -v -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $out/tests_randk.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $out/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > $out/bench_c2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_c5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > $out/bench_c3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats_c5 -o run --output-format csv -- \
     python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $out/stats_c5.log 2>&1 || exit $?
exit 0
