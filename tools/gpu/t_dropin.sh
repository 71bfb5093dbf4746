#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/td; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python bench.py --dropin --workload c3 --steps 5 --warmup 2 > $out/dropin_c3.log 2>&1 || { tail -20 $out/dropin_c3.log; exit 1; }
tail -1 $out/dropin_c3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/st -o run --output-format csv -- python bench.py --dropin --workload c3 --steps 3 --warmup 1 > $out/dropin_prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > $out/c3.log 2>&1 || exit 1
tail -1 $out/c3.log
