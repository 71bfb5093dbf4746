#!/bin/bash
# Round 6: large scratch (C3 / C4 candidate lists) in contiguous HBM too? (FLC_WS_CONTIG A/B, pairs)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_ws; mkdir -p $o
timeout -k 10 200 python -u -m pytest tests/test_gpu_threads.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
B="timeout -k 10 400 python bench.py --no-cpu-baseline"
for rep in 1 2; do for w in 0 1; do
  FLC_WS_CONTIG=$w $B --workload c4 > $o/c4_ws${w}_$rep.log 2>&1 || exit 1
  FLC_WS_CONTIG=$w $B --no-strong-c4 > $o/c3_ws${w}_$rep.log 2>&1 || exit 1
done; done
for f in $o/c4_*.log $o/c3_*.log; do tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f'.split('/')[-1], d['ms_per_step'], r['kernel_ms_per_step'], r['other_kernels_avg_ms'], r['read_ceiling_GBps'])"; done
