#!/bin/bash
# round 3: MARINA replay debug; TopK half-chunk fold (split lists) + resolve rewrite tests; A/B of
# the LDS-atomic QSGD fold (c4) and of the split fold (c3)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03ab3; mkdir -p $out
T="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 300 python -u tools/debug_marina.py > $out/debug_marina.log 2>&1; echo "debug rc=$?"; tail -12 $out/debug_marina.log
timeout -k 10 900 $T -x tests/test_gpu_parity.py tests/test_gpu_rows_ref.py tests/test_gpu_wire.py tests/test_gpu_randk_device.py \
   tests/test_gpu_shift.py tests/test_gpu_dither_sparse.py tests/test_gpu_configs.py > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $out/tests.log | head -20; exit 1; }
FLC_LIB_VARIANT=tuning FLC_DS_LDSADD=1 timeout -k 10 600 $T -x tests/test_gpu_dither_sparse.py > $out/tests_ldsadd.log 2>&1; echo "ldsadd tests rc=$? $(tail -1 $out/tests_ldsadd.log)"
VARIANTS="exp tuning@FLC_DS_LDSADD=1" WLS="c4" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab_c4.log
VARIANTS="exp tuning@FLC_SPLIT_FOLD=0" WLS="c3" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab_c3.log
cat $out/ab_c4.log $out/ab_c3.log
exit 0
