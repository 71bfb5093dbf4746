#!/bin/bash
# sparse-dithering bring-up: its tests, the existing GPU suite, C4 bench (sparse vs dense)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/ds; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dither_sparse.py -x -v -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $out/tests_ds.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $out/tests_all.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/bench_c4.log 2>&1 || exit $?
FLC_DITHER_PATH=dense timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_c4_dense.log 2>&1 || exit $?
exit 0
