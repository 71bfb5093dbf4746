#!/bin/bash
# Round 6: k_lone_resident knobs, same process: group replicas 4 (cur) / 2 / 8, abort-word poll
# every 4th, no s_sleep between polls
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_knobs; mkdir -p $o
PYTHONPATH=. timeout -k 10 400 python tools/ab_lone.py --variants cur,ng8,pa4 --n 32 --rounds 6 > $o/ab.jsonl 2>&1 || exit 1
grep -E "median|DIFFER" $o/ab.jsonl
