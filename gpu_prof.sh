#!/bin/bash
# profiling pass: kernel-trace stats for c3/c4/c2 + PMC byte counters for c3 (separate passes)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c4 c2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$wl -o run --output-format csv -- \
      python bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$wl.log 2>&1 || exit $?
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/pmc_c3_$ctr -o run --output-format csv -- \
      python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_c3_$ctr.log 2>&1 || exit $?
done
exit 0
