"""Is the C4 / C3 step time bimodal per allocation or per process?  One process, several fresh
allocations of the [N, D] rows (with a shifting dummy allocation in front), each timed over a few
steps with HIP events; a plain torch streaming read of the same rows beside it."""
import json
import sys

import torch

sys.path.insert(0, ".")
from flpytorch_amd import aggregation as ag  # noqa: E402

spec = sys.argv[1] if len(sys.argv) > 1 else "qsgd:127"
n, d = (512, 25_000_000) if spec.startswith("qsgd") else (1024, 10_000_000)
red = ag.UplinkReducer(ag.initCompressor(spec, d), seed=7)
res = []
for trial in range(6):
    pad = torch.empty(int((trial * 37 % 11) * 2**27), dtype=torch.uint8, device="cuda")   # 0..1.3 GB shift
    rows = torch.empty((n, d), device="cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    rows.normal_(generator=g)
    out = red(rows)
    torch.cuda.synchronize()
    ts = []
    for k in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = red(rows, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = rows.sum(dim=0)
    e0.record()
    for k in range(3):
        s = torch.sum(rows, dim=0, out=s)
    e1.record()
    torch.cuda.synchronize()
    res.append({"trial": trial, "pad_MB": pad.numel() >> 20, "rows_ptr_mod_2MB": rows.data_ptr() % (1 << 21),
                "rows_ptr_GB": round(rows.data_ptr() / 2**30, 2), "uplink_ms": [round(t, 3) for t in ts],
                "torch_sum_ms": round(e0.elapsed_time(e1) / 3, 3)})
    print(json.dumps(res[-1]), flush=True)
    del rows, pad
    torch.cuda.empty_cache()
