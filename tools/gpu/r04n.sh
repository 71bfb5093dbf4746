#!/bin/bash
# round 4: C3 row-group folds: side selects 512 (prod) vs 256 threads, one-wave fold ring 4 (prod) vs 8
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04n}; mkdir -p $out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
FLC_LIB_VARIANT=gs256 timeout -k 10 300 $T tests/test_gpu_parity.py -k "tail_groups or c3_variant" > $out/tests_gs256.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 5 --prof-modes off"
timeout -k 10 400 $A --workload c3 --variants prod,gs256,gap8 > $out/ab_c3.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c3 --variants gap8,gs256,prod > $out/ab_c3_b.txt 2>&1 || exit $?
exit 0
