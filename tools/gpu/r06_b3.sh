#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_b3; mkdir -p $o
timeout -k 10 300 python tools/ab_lone.py --variants r05,prod,nocnt --rounds 12 > $o/ab1.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/ab_lone.py --variants prod,r05,nocnt --rounds 12 > $o/ab2.jsonl 2>&1 || exit 1
grep median $o/ab*.jsonl
