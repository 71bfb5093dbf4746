#!/bin/bash
# Round 6: lone A/B (poll interval, exit count), new GPU tests, the default bench line with its strong_c4 block
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_b1; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_norm_torch.py tests/test_gpu_tie.py -x -q -p no:cacheprovider \
   --timeout 120 --timeout-method thread -rf > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python tools/ab_lone.py --variants prod,p16,nocnt --rounds 8 > $o/ab1.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/ab_lone.py --variants r05,prod --rounds 8 > $o/ab2.jsonl 2>&1 || exit 1
grep median $o/ab*.jsonl
timeout -k 10 400 python bench.py --no-cpu-baseline > $o/bench_default.log 2>&1 || { tail -20 $o/bench_default.log; exit 1; }
tail -1 $o/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], json.dumps(d.get('strong_c4')))"
