#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -rf -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/status.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
   python bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1
echo "bench rc=$?" >> gpurun_out/status.txt
exit 0
