#!/usr/bin/env python3
"""Generate tests/golden/weighted.{npz,json}: the reference's serverGradient fold with client
weights other than 1.0, run on the REAL reference (development container only; imported read-only
from /root/reference with the throwaway stubs of make_golden.py).

The algorithms' clientState overwrites every weight with 1.0 (algorithms.py:2045-2052), so no
run.py capture exercises w_i != 1; the serverGradient bodies themselves fold
``gs = w0 (x - x0); gs += wi (x - xi); gs / w_total`` with Python-float weights
(algorithms.py:1753-1768 DCGD, 1810-1832 FedAvg).  These cases pin that arithmetic (Python-float
weight times an fp32 tensor, the Python-float total as the divisor) for the product's weighted fold.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/fl_pytorch"
sys.path.insert(0, HERE)
from make_golden import _write_stubs  # noqa: E402

CASES = [
    # (N, D, weights, kind)
    (1, 1, [0.5], "normal"),
    (3, 1027, [0.5, 2.0, 1.25], "normal"),
    (4, 4099, [1.0, -0.75, 0.0, 3.3333333333333335], "normal"),
    (7, 10007, [0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7], "heavy"),
    (5, 16384, [1e-3, 1e3, 2.5, 0.125, 7.0], "heavy"),
    (2, 333, [-1.0, -2.0], "zeros"),
]


def make(seed, N, D, kind):
    g = np.random.default_rng(seed)
    x = g.standard_normal(D).astype(np.float32)
    rows = g.standard_normal((N, D)).astype(np.float32)
    if kind == "heavy":
        rows *= (10.0 ** g.uniform(-3, 3, (N, D))).astype(np.float32)
    if kind == "zeros":
        rows[:, ::3] = x[::3]            # x - x_i = +0 on every third column
        rows[0, 1::3] = -0.0
    return x, rows


def main():
    tmp = tempfile.mkdtemp(prefix="flstubs_")
    _write_stubs(tmp)
    for p in (tmp, os.path.join(REF, "utils"), REF):
        sys.path.insert(0, p)
    sys.dont_write_bytecode = True
    import torch
    from utils import algorithms, buffer, compressors   # the reference modules, imported read-only
    torch.set_num_threads(1)
    master = compressors.Compressor()
    master.makeIdenticalCompressor()
    meta, arrays = [], {}
    for ci, (N, D, w, kind) in enumerate(CASES):
        x, rows = make(100 + ci, N, D, kind)
        for algo, cls in (("dcgd", algorithms.DCGD), ("fedavg", algorithms.FedAvg)):
            buf = buffer.Buffer(N)
            for i in range(N):
                buf.pushBack({"model": torch.from_numpy(rows[i].copy()), "client_state": {"weight": w[i]}})
            H = {"fl_dtype": torch.float32, "compressor_master": master}
            gs = cls.serverGradient(buf, N, None, torch.from_numpy(x.copy()), H)
            arrays[f"c{ci}_{algo}_gs"] = gs.numpy().copy()
            meta.append({"case": ci, "algorithm": algo, "N": N, "D": D, "weights": w, "kind": kind})
        arrays[f"c{ci}_x"] = x
        arrays[f"c{ci}_rows"] = rows
    np.savez_compressed(os.path.join(HERE, "weighted.npz"), **arrays)
    with open(os.path.join(HERE, "weighted.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("weighted:", len(meta), "cases")


if __name__ == "__main__":
    main()
