#!/bin/bash
# k_ds_accum level-1 fast walk (prod) vs head (FLC_DS_L1FAST=0)
# the QSGD sparse-path suites, then the same-allocation C4 A/B and a trace of the new build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/l1f; mkdir -p $o
t() { local tm=$1 nm=$2; shift 2; timeout -k 10 $tm python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $o/$nm.log 2>&1 || { tail -30 $o/$nm.log; exit 1; }; tail -1 $o/$nm.log; }
t 400 tests_ds tests/test_gpu_dither_sparse.py tests/test_gpu_mixed.py
t 400 tests_cfg tests/test_gpu_configs.py tests/test_gpu_rows_ref.py
timeout -k 10 600 python3 tools/ab_inproc.py --workload c4 --variants prod,head --rounds 4 --steps 5 --prof-modes off > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
tail -4 $o/ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$o/c4 -o tr --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 4 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$o/c4.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/timeline.py $o/c4 k_ds_sample 2 > $o/c4_tl.txt
