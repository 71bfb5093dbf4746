#!/bin/bash
# round 3: the sparse-QSGD back half — resolve rewrite (product) and the LDS-atomic fold (tuning)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03ab2; mkdir -p $out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_dither_sparse.py tests/test_gpu_configs.py tests/test_gpu_rows_ref.py tests/test_gpu_harness.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
FLC_LIB_VARIANT=tuning FLC_DS_LDSADD=1 timeout -k 10 600 $T tests/test_gpu_dither_sparse.py > $out/tests_ldsadd.log 2>&1; echo "ldsadd tests rc=$? $(tail -1 $out/tests_ldsadd.log)"
VARIANTS="exp tuning@FLC_DS_LDSADD=1 tuning@FLC_DS_LDSADD=0" WLS="c4" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab.log
cat $out/ab.log
exit 0
