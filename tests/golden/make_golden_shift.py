#!/usr/bin/env python3
"""Generate tests/golden/shift.{npz,json}: the compressed algorithms' client step, run on the REAL
reference codecs with the algorithms' own torch expressions.

Test infrastructure only (development container; the reference is read-only at /root/reference and
its compressors.py imports only torch / math / numpy).  Per case: a seeded
``np.random.RandomState`` draws the pattern (``generateCompressPattern``, compressors.py:196-216),
then the step is evaluated exactly as the algorithm writes it:
    DIANA   m = C(g - h);  h' = h + alpha * m,  alpha = 1 / (1 + w)     algorithms.py:1349-1350, 1383-1391
    EF21    g_next = g_prev + C(g - g_prev) * mult,
            mult = 1 / (1 + w) unless C is a contraction               algorithms.py:1506-1517
    MARINA  g_next = g_prev + C(g - g_prev_x)                          algorithms.py:537
The reference's torch norm of g - b is recorded (dithering), so the oracle can be compared bit for
bit given that norm, as for compressVector.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference/fl_pytorch/utils")
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import compressors  # noqa: E402  (the reference module, imported, never copied)
from tests.golden_io import shift_fingerprint as fingerprint, shift_inputs as inputs  # noqa: E402

SPECS = ["ident", "bernulli:0.5", "randk:10%", "topk:5%", "natural", "qsgd:127", "qsgd:4", "std.dithering:8:2",
         "terngrad", "nat.dithering:6:2"]
ALGOS = ["diana", "ef21", "marina"]


def main():
    torch.set_num_threads(1)
    meta, arrays = [], {}
    i = 0
    for D in (1027, 4099):
        for si, spec in enumerate(SPECS):
            for algo in ALGOS:
                seed = 1000 * D + 10 * si + ALGOS.index(algo)
                a, b, x3 = inputs(seed, D)
                rs = np.random.RandomState(seed)
                c = compressors.initCompressor(spec, D)
                c.generateCompressPattern(rs, "cpu", 0, {})
                ta, tb, t3 = torch.from_numpy(a), torch.from_numpy(b), torch.from_numpy(x3)
                w = c.getW() if c.isUnbiasedCompressor() else None
                p = getattr(c, "p", None)
                pn = float(torch.norm(ta - tb, p)) if p is not None else 0.0
                if algo == "diana":
                    alpha = 1.0 / (1.0 + w) if w is not None else 0.5
                    m = c.compressVector(ta - tb)
                    h2 = tb + alpha * m
                    rec = dict(scale=1.0, alpha=alpha, base=None)
                    outs = dict(msg=m, h=h2)
                elif algo == "ef21":
                    mult = 1.0
                    if not c.isContractionCompressor():
                        mult = 1.0 / (1.0 + c.getW())
                    gn = tb + c.compressVector(ta - tb) * mult
                    rec = dict(scale=mult, alpha=None, base="b")
                    outs = dict(msg=gn)
                else:
                    gn = t3 + c.compressVector(ta - tb)
                    rec = dict(scale=1.0, alpha=None, base="x3")
                    outs = dict(msg=gn)
                meta.append(dict(spec=spec, D=D, algo=algo, seed=seed, pnorm=pn,
                                 need=float(c.last_need_to_send_advance), **rec))
                # inputs are regenerated from the seed by the tests (inputs(seed, D) below); the
                # fixture keeps a fingerprint so a changed generator fails loudly
                meta[-1]["fingerprint"] = fingerprint(a, b, x3)
                for k, v in outs.items():
                    arrays[f"{k}{i}"] = v.numpy().astype(np.float32)
                i += 1
    np.savez_compressed(os.path.join(HERE, "shift.npz"), **arrays)
    with open(os.path.join(HERE, "shift.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{len(meta)} shift cases written")


if __name__ == "__main__":
    main()
