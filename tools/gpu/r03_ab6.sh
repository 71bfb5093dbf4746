#!/bin/bash
# round 3: the lone-row TopK sample with its two rank searches merged (drop-in c3 line); compat QSGD through the single-pass sparse path (tests + C4 compat line), then the
# tail-overlap A/B (tuning build: FLC_DS_TAILOV / FLC_TK_TAILOV)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03ab6; mkdir -p $out
T="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T -x tests/test_gpu_dither_sparse.py > $out/tests_ds.log 2>&1; rc=$?
echo "sparse dithering tests rc=$rc $(tail -1 $out/tests_ds.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests_ds.log | head -20; exit 1; }
timeout -k 10 900 $T -x -m gpu tests > $out/tests_all.log 2>&1; rc=$?
echo "gpu suite rc=$rc $(tail -1 $out/tests_all.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests_all.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --dropin --workload c3 --n 8 --steps 10 --warmup 2 > $out/dropin_c3.log 2>&1 || exit $?
echo "dropin c3 $(tail -1 $out/dropin_c3.log)"
timeout -k 10 300 python bench.py --workload c4 --compat --steps 5 --warmup 1 --no-cpu-baseline > $out/c4_compat.log 2>&1; rc=$?
echo "c4 compat rc=$rc"; tail -1 $out/c4_compat.log; [ $rc -eq 0 ] || exit 1
FLC_LIB_VARIANT=tuning FLC_DS_TAILOV=4 FLC_TK_TAILOV=4 timeout -k 10 600 $T -x tests/test_gpu_dither_sparse.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "topk or dither or c4 or qsgd or sparse" > $out/tests_tailov.log 2>&1; rc=$?
echo "tailov tests rc=$rc $(tail -1 $out/tests_tailov.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $out/tests_tailov.log | head; exit 1; }
VARIANTS="tuning@FLC_DS_TAILOV=1 tuning@FLC_DS_TAILOV=2 tuning@FLC_DS_TAILOV=4 tuning@FLC_DS_TAILOV=8" WLS="c4" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab_c4.log
VARIANTS="tuning@FLC_TK_TAILOV=1 tuning@FLC_TK_TAILOV=2 tuning@FLC_TK_TAILOV=4 tuning@FLC_TK_TAILOV=8" WLS="c3" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab_c3.log
cat $out/ab_c4.log $out/ab_c3.log
exit 0
