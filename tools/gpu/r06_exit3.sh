#!/bin/bash
# Round 6: kernel durations (rocprofv3 kernel trace) of k_lone_resident cut short after each phase:
# ex4 + window histograms, ex5 + flush and arrival, ex6 + merger and release, ex7 all but the
# non-ranking workgroups' dense stores; cur the whole call
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_exit4; mkdir -p $o
for v in cur ex4 ex5 ex6 ex7; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/$v -o run --output-format csv -- python tools/ab_lone.py --variants $v --n 32 --rounds 2 > $o/$v.log 2>&1 || exit 1
  f=$(find $o/$v -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'k_lone_resident' in r['Name']: print('$v', r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['MinNs'])/1e3,2))"
done
