#!/bin/bash
# C2 device RandK breakdown: randk tests, bench c2, rocprof stats of c2
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r02d; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_randk_device.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $out/tests_randk.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > $out/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats_c2 -o run --output-format csv -- \
     python bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline > $out/stats_c2.log 2>&1 || exit $?
exit 0
