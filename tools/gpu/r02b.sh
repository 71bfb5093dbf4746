#!/bin/bash
# round-2 check: new collective tests, bench modes (strong scaling, compat, torch-CPU baseline),
# sparse-gather calibration probe (+ FETCH_SIZE pass)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r02b; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_collective.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $out/tests.log 2>&1 || exit $?
timeout -k 10 200 python tools/probe_gather.py > $out/probe_gather.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $out/pg_fetch -o run --output-format csv -- python tools/probe_gather.py --reps 1 > $out/probe_gather_pmc.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 --scaling strong --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_c4_strong.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c2 --compat --no-cpu-baseline > $out/bench_c2_compat.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > $out/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 --compat --n 256 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_c4_compat.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit $?
exit 0
