"""Probe: a few lone compressVector calls (D = 10 M, K = 1 %) on the current library variant
(FLC_LIB_VARIANT), for device-side printf probes of k_lone_resident.  usage: python tools/probe_lone.py [d] [calls]"""
import sys

import torch

import flpytorch_amd.aggregation as ag

d = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 4
x = torch.randn(d, device="cuda")
c = ag.initCompressor("topk:1%", d)
for _ in range(calls):
    c.compressVector(x)
    torch.cuda.synchronize()
print("flags", int(ag.select_row_flags(c, 1, d)[0]))
