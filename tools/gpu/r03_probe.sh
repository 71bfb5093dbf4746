#!/bin/bash
# Round 3, first box: read-ceiling probe (register ring vs LDS-DMA forms) beside the C4 / C3 lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03p; mkdir -p $out
timeout -k 10 240 tools/probe_read 512 25000000 4 2 > $out/probe_read.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/bench_c4_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > $out/bench_c3.log 2>&1 || exit $?
exit 0
