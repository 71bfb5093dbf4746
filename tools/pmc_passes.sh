#!/bin/bash
# Collect rocprofv3 PMC counters for one bench workload, one pass per counter group.
#   tools/pmc_passes.sh <tag> <bench args...> -- <group1> [<group2> ...]   (group = "CTR1,CTR2")
# Output: gpurun_out/pmc_<tag>_<i>/run_counter_collection.csv per group.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
args=()
while [ "$1" != "--" ]; do args+=("$1"); shift; done
shift
i=0
for grp in "$@"; do
  timeout -k 10 300 rocprofv3 --pmc ${grp//,/ } -d gpurun_out/pmc_${tag}_$i -o run --output-format csv -- \
     python bench.py "${args[@]}" --no-cpu-baseline > gpurun_out/pmc_${tag}_$i.log 2>&1 || exit $?
  i=$((i+1))
done
exit 0
