"""Probe: the per-workgroup timeline of back-to-back lone compressVector calls (D = 10 M, K = 1 %,
32 client rows in turn, like bench.py --dropin), printed by the FLC_RS_PRINT build every 16th call
(variant: FLC_LIB_VARIANT=rsprint).  usage: python tools/probe_lone_tl.py [d] [rounds]"""
import sys

import torch

import flpytorch_amd.aggregation as ag

d = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
n = 32
rows = torch.randn(n, d, generator=torch.Generator(device="cuda").manual_seed(9), device="cuda")
comps = [ag.initCompressor("topk:1%", d) for _ in range(n)]
for _ in range(rounds):
    for i in range(n):
        comps[i].compressVector(rows[i])
torch.cuda.synchronize()
print("flags", int(ag.select_row_flags(comps[0], 1, d)[0]))
