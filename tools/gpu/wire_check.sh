#!/bin/bash
# wire-format parity after a change to the pack path + the pack cost at D = 25 M
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/wc; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_shift.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit $?
cat > $out/pk.py <<'PY'
import sys, numpy as np, torch
sys.path.insert(0, ".")
from flpytorch_amd import aggregation as ag
d = 25_000_000
x = torch.randn(d, device="cuda")
for spec in ["qsgd:127", "natural", "topk:1%", "ident"]:
    c = ag.initCompressor(spec, d)
    c.device_rng = (3, 0)
    out = torch.empty(c.payloadBytes(d), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        c.compressPayload(x, out=out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(20):
        c.compressPayload(x, out=out)
    e.record(); torch.cuda.synchronize()
    print(spec, "pack %.1f us" % (s.elapsed_time(e) * 1e3 / 20))
PY
timeout -k 10 120 python $out/pk.py > $out/pk.log 2>&1 || exit $?
exit 0
