#!/bin/bash
# round 4: classification of 1..4 candidate batches per iteration (FLC_DS_CU), and the pipelined
# filter (v2), same allocation; sparse-QSGD tests on the product build first
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04h}; mkdir -p $out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_dither_sparse.py tests/test_gpu_rows_ref.py tests/test_gpu_configs.py -k "sparse or qsgd or c4" > $out/tests_ds.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 4 --prof-modes off"
timeout -k 10 400 $A --workload c4 --variants prod,cu1,cu2 > $out/ab_c4_a.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c4 --variants prod,cu3,v2 > $out/ab_c4_b.txt 2>&1 || exit $?
exit 0
