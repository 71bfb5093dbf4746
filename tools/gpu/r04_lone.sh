#!/bin/bash
# lone rows: parity of the dithering / codec suites, then the drop-in probe new vs old
# (abvar/libflcodec_old.so: -DFLC_LONE_DITHER=0) and a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/lone; mkdir -p $o
t() { local tm=$1 nm=$2; shift 2; timeout -k 10 $tm python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $o/$nm.log 2>&1 || { tail -30 $o/$nm.log; exit 1; }; tail -1 $o/$nm.log; }
t 300 tests_ds tests/test_gpu_dither_sparse.py -k "lone"
t 400 tests_par tests/test_gpu_parity.py -k "compress or dither or qsgd or golden"
t 300 tests_rows tests/test_gpu_rows_ref.py tests/test_gpu_shift.py tests/test_gpu_wire.py
for v in new old new old; do
  if [ $v = old ]; then export FLC_LIB_VARIANT=old; else unset FLC_LIB_VARIANT; fi
  timeout -k 10 120 python3 tools/dropin_probe.py --spec qsgd:127 --d 25000000 --compat > $o/probe_qsgdc_$v.json || exit 1
  timeout -k 10 120 python3 tools/dropin_probe.py --spec qsgd:127 --d 25000000 > $o/probe_qsgd_$v.json || exit 1
  echo "$v $(cat $o/probe_qsgdc_$v.json)"; echo "$v $(cat $o/probe_qsgd_$v.json)"
done
unset FLC_LIB_VARIANT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$o/profq -o tr -- python3 $GRAFT_REPO_ROOT/tools/dropin_probe.py --reps 40 --spec qsgd:127 --d 25000000 --compat > $GRAFT_REPO_ROOT/$o/profq.log 2>&1
