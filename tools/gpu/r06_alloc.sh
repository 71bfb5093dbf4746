#!/bin/bash
# Round 6: the resident rows in contiguous HBM — its tests and the C3 / C4 lines with both allocations
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_alloc; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
B="timeout -k 10 400 python bench.py --no-cpu-baseline"
for a in contiguous default; do
  $B --workload c4 --alloc $a > $o/c4_$a.log 2>&1 || exit 1
  $B --alloc $a --no-strong-c4 > $o/c3_$a.log 2>&1 || exit 1
done
for f in $o/c4_*.log $o/c3_*.log; do tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f'.split('/')[-1], d['ms_per_step'], d['value'], r['frac'], r['read_ceiling_GBps'], d['config']['rows_alloc'])"; done
