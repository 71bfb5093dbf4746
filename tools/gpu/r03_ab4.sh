#!/bin/bash
# round 3: MARINA same-box parity (harness tests), branch-free candidate staging (QSGD filter
# PROBE 5) tests + same-box A/B against the branching staging
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03ab4; mkdir -p $out
T="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $T -x tests/test_gpu_harness.py > $out/tests_harness.log 2>&1; echo "harness tests rc=$? $(tail -1 $out/tests_harness.log)"
grep -E "^(FAILED|ERROR)" $out/tests_harness.log | head -5
FLC_LIB_VARIANT=tuning FLC_DS_PROBE=5 timeout -k 10 600 $T -x tests/test_gpu_dither_sparse.py > $out/tests_p5.log 2>&1; echo "probe5 tests rc=$? $(tail -1 $out/tests_p5.log)"
VARIANTS="tuning@FLC_DS_PROBE=0 tuning@FLC_DS_PROBE=5 tuning@FLC_DS_PROBE=0 tuning@FLC_DS_PROBE=5" WLS="c4" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab_c4.log
cat $out/ab_c4.log
exit 0
