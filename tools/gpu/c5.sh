#!/bin/bash
# C2 / C5 pass: randk + mixed parity tests, bench c2 and c5, rocprof kernel stats of c5.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-c5}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mixed.py tests/test_gpu_shift.py -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k "randk or mixed or shift" > $out/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > $out/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_c5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats_c5 -o run --output-format csv -- \
    python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $out/stats_c5.log 2>&1 || exit $?
exit 0
