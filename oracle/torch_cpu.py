"""ORACLE — TEST / BENCH INFRASTRUCTURE ONLY (never imported by flpytorch_amd/).

Op-for-op torch-CPU restatement of the reference's uplink, used by ``bench.py``'s
``cpu_baseline`` leg to time what the reference itself costs on the GPU box's host cores (the
reference's Python cannot travel there; SURVEY §8d "Reference CPU path timing").  It issues the
same torch / numpy calls the reference issues, in the same order, on CPU tensors:

* ``generate``  — generateCompressPattern, compressors.py:196-216: the experiment's numpy
  ``RandomState`` draws (``choice(D, K, replace=False)`` -> int64 tensor for RandK, ``rand(D)``
  float64 uniforms for the dithering family; nothing for TopK / ident).
* ``compress``  — compressVector, compressors.py:218-299, 330-335: RandK zeros + index scatter of
  ``(D/K) * x[S]``; TopK ``torch.topk(|x|, K)`` + scatter; standard dithering / QSGD the norm, then
  the reference's per-level mask loop (s passes over D), the zero rule and ``out * sign * pnorm``.
* ``fold``      — serverGradient core, algorithms.py:1753-1768: ``gi = x - x_i; gs += wi * gi``
  in Buffer order, ``gs / w_total``.

The outputs agree with ``oracle/codecs.py`` (tests/test_host.py checks a small case); what this
module is for is the *cost*: ``time_uplink`` times the three phases separately, per client.
"""
import math
import time

import numpy as np
import torch


class TorchCpuCodec:
    """One client's compressor, restated with the reference's own torch calls (randk / topk /
    std dithering family / ident)."""

    def __init__(self, spec, d):
        parts = spec.lower().split(":")
        self.name, self.d = parts[0], d
        if self.name in ("randk", "topk"):
            a = parts[1]
            self.k = math.ceil(float(a[:-1]) / 100.0 * d) if a.endswith("%") else math.ceil(float(a))
        elif self.name in ("qsgd", "std_dithering"):
            self.s = int(parts[1])
            self.p = 2.0 if self.name == "qsgd" else float(parts[2]) if len(parts) > 2 else float("inf")
            # compressors.py:87
            self.levels = torch.arange(0.0, 1.0 + 1.0 / self.s * 0.5, 1.0 / self.s)
        elif self.name != "ident":
            raise ValueError(f"torch_cpu baseline: {spec} not restated")

    def generate(self, rndgen):
        if self.name == "randk":
            self.S = torch.from_numpy(rndgen.choice(self.d, self.k, replace=False)).to(torch.long)
        elif self.name in ("qsgd", "std_dithering"):
            self.testp = torch.from_numpy(rndgen.rand(self.d))

    def compress(self, x):
        if self.name == "ident":
            return x
        if self.name == "randk":
            out = torch.zeros_like(x)
            out[self.S] = (self.d / self.k) * x[self.S]
            return out
        if self.name == "topk":
            _, ind = torch.topk(x.abs(), self.k)
            out = torch.zeros_like(x)
            out[ind] = x[ind]
            return out
        out = torch.zeros_like(x)
        pnorm = torch.norm(x, p=self.p)
        sign = torch.sign(x)
        y = torch.abs(x) / pnorm
        lv = self.levels
        for s in range(len(lv) - 1):
            c1 = y >= lv[s]
            c2 = y <= lv[s + 1]
            p = (y - lv[s + 1]) / (lv[s] - lv[s + 1])
            c3 = self.testp < p
            out[c1 & c2 & c3] = lv[s]
            out[c1 & c2 & (~c3)] = lv[s + 1]
        out[x == 0.0] = 0.0
        return out * sign * pnorm


def fold(x, client_models, weights=None):
    """serverGradient's core on CPU tensors, in Buffer order (algorithms.py:1753-1768)."""
    weights = weights or [1.0] * len(client_models)
    wi = weights[0]
    gs = wi * (x - client_models[0])
    w_total = wi
    for xi, wi in zip(client_models[1:], weights[1:]):
        w_total += wi
        gs += wi * (x - xi)
    return gs / w_total


def time_uplink(specs, d, budget_s, seed=123, min_clients=2, max_clients=64):
    """Time the reference's CPU uplink on this host: per client the pattern draws, the compress
    and (as the server's Buffer fold does) one accumulation step; clients are added until
    ``budget_s`` of measured work or ``max_clients``.  Returns per-phase seconds and the count.
    Client models are x - gamma * C(g_i) with gamma = 1 and x = 0, the form serverGradient folds."""
    rs = np.random.RandomState(seed)
    gen = torch.Generator().manual_seed(seed)
    x = torch.zeros(d)
    t_pat = t_comp = t_fold = 0.0
    n = 0
    gs = None
    w_total = 0.0
    while n < max_clients and (n < min_clients or t_pat + t_comp + t_fold < budget_s):
        g = torch.randn(d, generator=gen)
        c = TorchCpuCodec(specs[n % len(specs)], d)
        t0 = time.perf_counter()
        c.generate(rs)
        rs.randint(2 ** 31)                       # clientState's seed draw (algorithms.py:2055)
        t1 = time.perf_counter()
        e = c.compress(g)
        t2 = time.perf_counter()
        xi = x - e                                # the local step x_i = x - gamma C(g_i) (not timed
        t3 = time.perf_counter()                  # as part of the server: client-side)
        gi = x - xi
        if gs is None:
            gs = 1.0 * gi
        else:
            gs += 1.0 * gi
        w_total += 1.0
        t4 = time.perf_counter()
        t_pat += t1 - t0
        t_comp += t2 - t1
        t_fold += t4 - t3
        n += 1
    t5 = time.perf_counter()
    gs = gs / w_total
    t_fold += time.perf_counter() - t5
    return {"clients": n, "pattern_s": t_pat, "compress_s": t_comp, "fold_s": t_fold}
