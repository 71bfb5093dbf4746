#!/bin/bash
# round 3: tail-overlap A/B (tuning build: FLC_DS_TAILOV / FLC_TK_TAILOV row groups) after its tests
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03ab7; mkdir -p $out
T="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"
FLC_LIB_VARIANT=tuning FLC_DS_TAILOV=4 FLC_TK_TAILOV=4 timeout -k 10 600 $T -x tests/test_gpu_dither_sparse.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "topk or dither or c4 or qsgd or sparse" > $out/tests_tailov.log 2>&1; rc=$?
echo "tailov tests rc=$rc $(tail -1 $out/tests_tailov.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests_tailov.log | head; exit 1; }
VARIANTS="tuning@FLC_DS_TAILOV=1 tuning@FLC_DS_TAILOV=2 tuning@FLC_DS_TAILOV=4 tuning@FLC_DS_TAILOV=8" WLS="c4" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab_c4.log
VARIANTS="tuning@FLC_TK_TAILOV=1 tuning@FLC_TK_TAILOV=2 tuning@FLC_TK_TAILOV=4 tuning@FLC_TK_TAILOV=8" WLS="c3" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab_c3.log
cat $out/ab_c4.log $out/ab_c3.log
exit 0
