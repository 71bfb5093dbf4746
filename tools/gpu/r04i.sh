#!/bin/bash
# round 4: the pipelined-classification filter at staging 384 (5 blocks / CU) and 512 (4 / CU) vs
# the product (k_ds_filter, 2 batches per classification iteration); two processes (placements)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04i}; mkdir -p $out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
FLC_LIB_VARIANT=v2c384 timeout -k 10 400 $T tests/test_gpu_dither_sparse.py tests/test_gpu_rows_ref.py tests/test_gpu_configs.py -k "sparse or qsgd or c4" > $out/tests_v2.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 4"
timeout -k 10 400 $A --workload c4 --variants prod,v2c384,v2c512 > $out/ab_c4_a.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c4 --variants prod,v2c384,v2c512 > $out/ab_c4_b.txt 2>&1 || exit $?
exit 0
