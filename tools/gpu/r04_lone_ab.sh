#!/bin/bash
# lone-row compressVector A/B (abvar builds): QSGD compat at D = 25 M over the k_lone_dither grid
# variants, TopK 1 % at D = 10 M prod vs head (the histogram scan)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/lone_ab; mkdir -p $o
for rep in 1 2; do
for v in prod c1 c2 c3 c4; do
  if [ $v = prod ]; then unset FLC_LIB_VARIANT; else export FLC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python3 tools/dropin_probe.py --spec qsgd:127 --d 25000000 --compat > $o/c_$v.json || exit 1
  echo "$rep $v $(cat $o/c_$v.json)"
done
for v in; do
  if [ $v = prod ]; then unset FLC_LIB_VARIANT; else export FLC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python3 tools/dropin_probe.py > $o/t_$v.json || exit 1
  echo "$rep topk $v $(cat $o/t_$v.json)"
done
done
