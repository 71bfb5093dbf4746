#!/bin/bash
# Round 6: kernel durations (rocprofv3 kernel trace) of k_lone_resident cut short at each point
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_exit2; mkdir -p $o
for v in s2 ex1 ex2 ex3; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/$v -o run --output-format csv -- python tools/ab_lone.py --variants $v --n 32 --rounds 2 > $o/$v.log 2>&1 || exit 1
  f=$(find $o/$v -name '*kernel_stats.csv' | head -1)
  echo "$v $(grep k_lone_resident $f | cut -d, -f1-8)"
done
