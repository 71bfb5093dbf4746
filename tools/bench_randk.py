"""Timing probe (not product code): device RandK counts kernel and fused uplink at C2 / C5 shapes."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
from flpytorch_amd import _lib  # noqa: E402
from flpytorch_amd import aggregation as ag  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


lib = _lib.load()
SHAPES = [(256, 1_000_000, 10_000, "c2"), (683, 100_000_000, 1_000_000, "c5-randk"),
          (64, 10_000_000, 100_000, "mid")]
if len(sys.argv) > 1 and sys.argv[1] == "counts":
    SHAPES = [(1, 1_000_000, 10_000, "c2x1"), (16, 1_000_000, 10_000, "c2x16"), (1, 100_000_000, 1_000_000, "c5x1"),
              (64, 100_000_000, 1_000_000, "c5x64"), (1, 1_000_000, 100, "c2-k100"), (1, 4096 * 256, 256 * 41, "L8")]
for n, d, k, label in SHAPES:
    C = (d + 4095) // 4096
    out = torch.zeros((C, n), dtype=torch.int32, device="cuda")
    wsb = lib.flc_device_randk_counts_workspace_size(n, d)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")

    def counts():
        assert lib.flc_device_randk_counts(7, 0, n, d, k, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                           wsb, _lib.stream_ptr()) == 0
    res = {"shape": label, "n": n, "d": d, "k": k, "counts_ms": round(timed(counts), 4)}
    if len(sys.argv) > 1:
        print(json.dumps(res), flush=True)
        continue
    if d * n * 4 < 40e9:
        rows = torch.randn(n, d, device="cuda")
        red = ag.UplinkReducer(ag.initCompressor(f"randk:{k}", d), seed=7)
        res["uplink_ms"] = round(timed(lambda: red(rows)), 4)
        del rows
    else:
        pool = torch.randn(16, d, device="cuda")
        rl = [pool[i % 16] for i in range(n)]
        red = ag.UplinkReducer(ag.initCompressor(f"randk:{k}", d), seed=7)
        res["uplink_ms_pool16"] = round(timed(lambda: red(rl), reps=3), 4)
        del pool
    print(json.dumps(res), flush=True)
