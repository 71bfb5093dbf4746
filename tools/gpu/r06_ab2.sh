cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_lone2
timeout -k 10 300 python tools/ab_lone.py --variants prod,p16,nocnt --rounds 8 > gpurun_out/r06_lone2/ab1.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/ab_lone.py --variants r05,prod --rounds 8 > gpurun_out/r06_lone2/ab2.jsonl 2>&1 || exit 1
grep median gpurun_out/r06_lone2/ab*.jsonl
