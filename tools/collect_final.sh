#!/bin/bash
# copy an evidence pass (tools/gpu/evidence_r06.sh, gpurun_out/<ev>) into profiles/${ROUND:-r06}/<dst>
# usage: tools/collect_final.sh <ev> <dst> "<build note>"
set -e
src=gpurun_out/$1; dst=profiles/${ROUND:-r06}/$2; mkdir -p $dst
for f in $src/bench_*.log $src/dropin_*.log $src/e2e_*.log; do
  b=$(basename $f .log); grep '^{' $f | tail -1 > $dst/$b.jsonl
done
for wl in c2 c3 c4 c5; do cp $(find $src/stats_$wl -name '*kernel_stats.csv' | head -1) $dst/${wl}_kernel_stats.csv; done
for wl in c2 c3 c4 c5 c5_randk c4_compat dropin_c3 dropin_c4; do [ -f $src/pmc_$wl.log ] || continue; grep '^{' $src/pmc_$wl.log | tail -1 > $dst/pmc_$wl.json; cp $dst/pmc_$wl.json profiles/pmc_$wl.json; done
f=$(find $src/stats_dropin_c3 -name '*kernel_stats.csv' 2>/dev/null | head -1); [ -n "$f" ] && cp $f $dst/dropin_c3_kernel_stats.csv
tail -1 $src/gpu_tests.log > $dst/gpu_tests_summary.txt
cp $src/smoke.log $dst/smoke.log
for wl in c3 c4; do [ -f $src/inproc_$wl.log ] && cp $src/inproc_$wl.log $dst/inproc_vs_previous_$wl.txt; done
echo "$3" > $dst/BUILD.txt
