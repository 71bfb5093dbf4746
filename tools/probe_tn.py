"""Probe: one torch-order norm of a Gaussian row (flc_norm2_torch_cpu_ws) on the current library
variant (FLC_LIB_VARIANT), for the walk's device printf (FLC_TN_PRINT builds).  usage: python tools/probe_tn.py [d]"""
import sys

import torch

import flpytorch_amd.aggregation as ag

d = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
x = torch.randn(d, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
c = ag.initCompressor("qsgd:127", d)
print("norm", float(c.torchNorm(x)))
torch.cuda.synchronize()
