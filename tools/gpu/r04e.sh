#!/bin/bash
# round 4: full GPU suite on the product build (k_ds_filter2, one-wave chunk fold), then
# same-allocation A/Bs against the same tree with each change off, and the TopK filter probes
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04e}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 4"
timeout -k 10 400 $A --workload c4 --variants prod,v1 > $out/ab_c4.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c3 --variants prod,ca4 > $out/ab_c3.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c3 --variants prod,tk1,tk2 --rounds 3 --no-bitcheck > $out/ab_c3_probe.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c3 --variants prod,tk3 --rounds 3 --no-bitcheck > $out/ab_c3_probe3.txt 2>&1 || exit $?
exit 0
