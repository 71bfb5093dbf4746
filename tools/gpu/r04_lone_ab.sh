#!/bin/bash
# lone QSGD compressVector variants (abvar builds), compat uniforms, D = 25 M
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/lone_ab; mkdir -p $o
for rep in 1 2; do
for v in prod keep keepnt outnt u8; do
  if [ $v = prod ]; then unset FLC_LIB_VARIANT; else export FLC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python3 tools/dropin_probe.py --spec qsgd:127 --d 25000000 --compat > $o/c_$v.json || exit 1
  echo "$rep $v $(cat $o/c_$v.json)"
done
done
