#!/bin/bash
# round 4: sparse-QSGD tests on the product build (resolve with up-front window gathers), then
# same-allocation C4 A/Bs: prod vs the previous commit vs masked fold loads; filter probes.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04c}; mkdir -p $out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_dither_sparse.py tests/test_gpu_rows_ref.py tests/test_gpu_configs.py -k "sparse or qsgd or c4" > $out/tests_ds.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 4"
timeout -k 10 400 $A --workload c4 --variants prod,base,mld > $out/ab_c4.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c4 --variants prod,p6,p3 --rounds 3 > $out/ab_c4_probe.txt 2>&1 || exit $?
exit 0
