#!/bin/bash
# folds' carried tile loaded with all loads in flight (prod) vs the per-64-column loop (head,
# FLC_TILE_V4=0): fold suites, then same-allocation C4 and C3 A/Bs and traces
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/tv4; mkdir -p $o
t() { local tm=$1 nm=$2; shift 2; timeout -k 10 $tm python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $o/$nm.log 2>&1 || { tail -30 $o/$nm.log; exit 1; }; tail -1 $o/$nm.log; }
t 700 tests tests/test_gpu_dither_sparse.py tests/test_gpu_parity.py tests/test_gpu_rows_ref.py tests/test_gpu_configs.py tests/test_gpu_mixed.py tests/test_gpu_harness.py
for wl in c4 c3; do
  timeout -k 10 600 python3 tools/ab_inproc.py --workload $wl --variants prod,head --rounds 4 --steps 5 --prof-modes off > $o/ab_$wl.log 2>&1 || { tail -20 $o/ab_$wl.log; exit 1; }
  tail -2 $o/ab_$wl.log
done
cd /tmp && export TMPDIR=/tmp
for wl in c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$o/$wl -o tr --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 4 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$o/$wl.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT && python3 tools/timeline.py $o/c4 k_ds_sample 2 > $o/c4_tl.txt && python3 tools/timeline.py $o/c3 k_topk_sample 2 > $o/c3_tl.txt
