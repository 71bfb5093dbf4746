#!/bin/bash
# single-row compressVector latency (the drop-in path) + C3 / C4 lines + the affected parity tests
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/cv; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shift.py tests/test_gpu_dither_sparse.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit $?
cat > $out/cv.py <<'PY'
import sys, time, numpy as np, torch
sys.path.insert(0, ".")
from flpytorch_amd import aggregation as ag
d = 10_000_000
x = torch.randn(d, device="cuda")
for spec in ["topk:1%", "qsgd:127", "natural", "randk:1%"]:
    c = ag.initCompressor(spec, d)
    c.generateCompressPattern(np.random.RandomState(1), "cuda", 0, {})
    for _ in range(5):
        c.compressVector(x)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(50):
        c.compressVector(x)
    e.record(); torch.cuda.synchronize()
    print(spec, "%.1f us/call" % (s.elapsed_time(e) * 1e3 / 50))
PY
timeout -k 10 120 python $out/cv.py > $out/cv.log 2>&1 || exit $?
for wl in c3 c4; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/bench_$wl.log 2>&1 || exit $?
done
exit 0
