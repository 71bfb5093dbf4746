#!/bin/bash
# round 4: a smaller last row group (its tail is the exposed one): C3 (TopK, 4 groups) and C4 (2 groups)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04o}; mkdir -p $out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
FLC_LIB_VARIANT=tl30 timeout -k 10 300 $T tests/test_gpu_parity.py -k "tail_groups or c3_variant" > $out/tests_tl30.log 2>&1 || exit $?
FLC_LIB_VARIANT=dl30 timeout -k 10 300 $T tests/test_gpu_dither_sparse.py -k "row_groups or shapes" > $out/tests_dl30.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 5 --prof-modes off"
timeout -k 10 400 $A --workload c3 --variants prod,tl50,tl30 > $out/ab_c3.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c4 --variants prod,dl50,dl30 > $out/ab_c4.txt 2>&1 || exit $?
exit 0
