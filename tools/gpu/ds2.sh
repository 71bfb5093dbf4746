#!/bin/bash
# sparse QSGD (sure / ambiguous classification) check: its parity tests, then C4 bench + kernel stats
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/ds2; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dither_sparse.py \
   > $out/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/c4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- \
   python bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > $out/stats.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload reduce --steps 10 --warmup 2 --no-cpu-baseline > $out/reduce.log 2>&1 || exit $?
exit 0
