#!/bin/bash
# TopK exposed last-group fold: one-wave workgroups with the full ring (prod, k_chunk_accum1x) vs
# 4-wave blocks (head, FLC_TK_LAST1=0); TopK suites first, then the same-allocation C3 A/B + trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/last1; mkdir -p $o
t() { local tm=$1 nm=$2; shift 2; timeout -k 10 $tm python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $o/$nm.log 2>&1 || { tail -30 $o/$nm.log; exit 1; }; tail -1 $o/$nm.log; }
t 600 tests_tk tests/test_gpu_parity.py tests/test_gpu_rows_ref.py tests/test_gpu_configs.py tests/test_gpu_mixed.py tests/test_gpu_harness.py
timeout -k 10 600 python3 tools/ab_inproc.py --workload c3 --variants prod,head --rounds 5 --steps 5 --prof-modes off > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
tail -2 $o/ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$o/c3 -o tr --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c3 --steps 4 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$o/c3.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/timeline.py $o/c3 k_topk_sample 2 > $o/c3_tl.txt
