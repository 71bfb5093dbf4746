#!/bin/bash
# round 4: tests of the new TopK/dist cases on the product build, the sparse-QSGD tests on the
# per-lane staging variant (abvar/libflcodec_pl.so), then same-allocation A/Bs (tools/ab_inproc.py).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04b}; mkdir -p $out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "c3_variant or 4chunk or few_rows" > $out/tests_topk.log 2>&1 || exit $?
FLC_LIB_VARIANT=pl timeout -k 10 300 $T tests/test_gpu_dither_sparse.py tests/test_gpu_rows_ref.py -k "sparse or qsgd" > $out/tests_pl.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 4"
timeout -k 10 400 $A --workload c4 --variants prod,pl,mld > $out/ab_c4.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c3 --variants prod,base,ap16 > $out/ab_c3.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c4 --variants prod,dsap32 --rounds 3 > $out/ab_c4_ap32.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c3 --variants prod,ap32 --rounds 3 > $out/ab_c3_ap32.txt 2>&1 || exit $?
timeout -k 10 300 $T tests/test_gpu_dist.py > $out/tests_dist.log 2>&1 || exit $?
exit 0
