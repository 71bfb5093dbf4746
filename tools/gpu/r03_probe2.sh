#!/bin/bash
# round 3: (1) TopK / QSGD GPU tests on the product (few-row candidate select, sharded lists);
# (2) where the C4 filter's time goes (tuning build probes; outputs not valid: 0 full, 2 no
# candidate staging, 3 loads + norm only, 4 group hash without multiplies; g1 = 24-bit-multiply
# group hash); (3) the drop-in compressVector: product vs the one-workgroup select / chunk assign
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03p2; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rows_ref.py tests/test_gpu_shift.py \
   tests/test_gpu_wire.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for v in "" tuning@FLC_CS_SINGLE=1 tuning@FLC_ASSIGN_FOLD=1; do
  vv=${v%%@*}; ev=""; [ "$v" != "$vv" ] && ev=${v#*@}
  env $ev FLC_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --dropin --workload c3 --n 8 --steps 10 --warmup 2 > $out/dropin_c3.log 2>&1 || exit $?
  echo "dropin c3 [$v] $(tail -1 $out/dropin_c3.log)"
done
timeout -k 10 300 python bench.py --dropin --workload c4 --n 4 --steps 5 --warmup 1 > $out/dropin_c4.log 2>&1 || exit $?
echo "dropin c4 $(tail -1 $out/dropin_c4.log)"
VARIANTS="tuning@FLC_DS_PROBE=0 tuning@FLC_DS_PROBE=2 tuning@FLC_DS_PROBE=3 tuning@FLC_DS_PROBE=4 g1" WLS="c4" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab.log
cat $out/ab.log
exit 0
