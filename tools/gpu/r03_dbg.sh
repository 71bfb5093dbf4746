#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03dbg; mkdir -p $out
T="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 300 python -u tools/debug_marina.py > $out/debug_marina.log 2>&1; echo "debug rc=$?"; tail -12 $out/debug_marina.log
timeout -k 10 900 $T -x tests/test_gpu_parity.py tests/test_gpu_rows_ref.py tests/test_gpu_dither_sparse.py > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $out/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --dropin --workload c3 --n 8 --steps 10 --warmup 2 > $out/dropin_c3.log 2>&1 || exit $?
tail -1 $out/dropin_c3.log | cut -c1-900
timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > $out/c3.log 2>&1 || exit $?
tail -1 $out/c3.log | cut -c1-1500
exit 0
