#!/bin/bash
# first GPU pass: smoke, parity tests, short bench, rocprof stats
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocminfo | grep -m2 -E "gfx950|Marketing" > gpurun_out/device.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/status.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/status.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/status.txt
exit 0
