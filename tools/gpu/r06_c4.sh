#!/bin/bash
# Round 6, C4 levers, each a same-allocation A/B against the product build:
# row groups 1 / 2 / 3 with the round-5 fold, then the filter's rows per item block (the pages a CU
# walks at once: the translation lever) and the tail overlap of a single group, on the tuning build.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_c4; mkdir -p $o
A="timeout -k 10 300 python tools/ab_inproc.py --workload c4 --rounds 5 --steps 5 --prof-modes off"
$A --variants prod,prod:rg1,prod:rg3 > $o/rg.jsonl 2>&1 || exit 1
grep median $o/rg.jsonl
for rb in 4 64; do
  FLC_DS_RB=$rb $A --variants prod,tuning > $o/rb$rb.jsonl 2>&1 || exit 1
  echo "rb=$rb"; grep median $o/rb$rb.jsonl
done
FLC_DS_TAILOV=2 $A --variants prod,tuning:rg1 > $o/tailov2.jsonl 2>&1 || exit 1
echo "tailov2"; grep median $o/tailov2.jsonl
