#!/bin/bash
# round 3: GPU tests of the half-major QSGD lists + the row-size reference pins, then the C4 A/B
# of group-hash / grid variants (same box, interleaved)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03ab1; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dither_sparse.py tests/test_gpu_configs.py tests/test_gpu_rows_ref.py \
   tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
VARIANTS="new base g1 g2 tuning@FLC_DS_GRID=res" WLS="c4" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab.log
cat $out/ab.log
exit 0
