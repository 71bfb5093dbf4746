#!/bin/bash
# lone QSGD row: k_lone_dither with its first trip loaded before the norm fold (prod) vs head
# (FLC_LONE_PRE=0) vs pipe (FLC_LONE_PIPE=1); dithering parity first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/lone_pre; mkdir -p $o
t() { local tm=$1 nm=$2; shift 2; timeout -k 10 $tm python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $o/$nm.log 2>&1 || { tail -30 $o/$nm.log; exit 1; }; tail -1 $o/$nm.log; }
t 300 tests_ds tests/test_gpu_dither_sparse.py -k "lone"
t 400 tests_par tests/test_gpu_parity.py -k "compress or dither or qsgd or golden"
t 300 tests_rows tests/test_gpu_rows_ref.py
for rep in 1 2; do
for v in prod head pipe; do
  if [ $v = prod ]; then unset FLC_LIB_VARIANT; else export FLC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python3 tools/dropin_probe.py --spec qsgd:127 --d 25000000 --compat > $o/c_$v.json || exit 1
  timeout -k 10 120 python3 tools/dropin_probe.py --spec qsgd:127 --d 25000000 > $o/d_$v.json || exit 1
  echo "$rep $v compat $(cat $o/c_$v.json)"; echo "$rep $v dev $(cat $o/d_$v.json)"
done
done
