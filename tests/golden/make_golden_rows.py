#!/usr/bin/env python3
"""Generate tests/golden/rows.{npz,json}: the REAL reference's codecs at the config row sizes.

Test infrastructure only, run in the development container where the reference is mounted
read-only (compressors.py imports only torch, math and numpy and is imported
directly from /root/reference/fl_pytorch/utils).  The other fixtures stop at D = 65 536; these pin
the reference itself at BASELINE.json's row sizes:

* ``topk:1%`` at D = 10 M (C3's row): ``torch.topk(|x|, K)`` (compressors.py:330-335) — the
  index set is stored (sorted, int32), with a digest of the dense output;
* ``qsgd:127`` at D = 25 M (C4's row): ``torch.norm(x, 2)`` (compressors.py:272: torch's CPU fp32
  reduction, NOT exactly rounded) and the per-level mask loop against the numpy-stream uniforms
  ``rand(D)`` (compressors.py:208-212, 284-296) — stored: the reference's norm (fp32 bits), the
  exactly rounded norm of the same row, the nonzero count, the per-level histogram, a digest of the
  whole output and 4096 sampled (index, output) pairs.

Inputs are seed-regenerable on the GPU box without the reference: rows from
``np.random.default_rng(seed).standard_normal(D, dtype=float32)`` (times ``10**U(-3, 3)`` for the
heavy distribution of SURVEY §8d), uniforms from ``np.random.RandomState(seed)`` through the
reference's own ``generateCompressPattern``; digests of both are stored so a test can tell a
regeneration mismatch from a codec mismatch.  torch's intra-op threads are recorded (the CPU
norm's reduction order may depend on them).
"""
import hashlib
import json
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference/fl_pytorch/utils")
import compressors  # noqa: E402  (the reference module, imported, never copied)

CASES = [
    # (name, spec, D, row seed, distribution, pattern seed)
    ("topk_c3", "topk:1%", 10_000_000, 31, "normal", None),
    ("topk_c3_heavy", "topk:1%", 10_000_000, 32, "heavy", None),
    ("qsgd_c4", "qsgd:127", 25_000_000, 41, "normal", 4242),
    ("qsgd_c4_heavy", "qsgd:127", 25_000_000, 42, "heavy", 4343),
]


def row(seed, d, dist):
    """The synthetic row (also restated in tests/test_gpu_rows_ref.py)."""
    g = np.random.default_rng(seed)
    x = g.standard_normal(d, dtype=np.float32)
    if dist == "heavy":
        x *= np.power(np.float32(10.0), g.uniform(-3.0, 3.0, d).astype(np.float32))
    return x


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:32]


def exact_norm(x):
    """RN(sqrt(sum x^2)) from float64 squares (exact to well under an fp32 ulp at these D)."""
    v = x.astype(np.float64)
    return np.float32(math.sqrt(float(np.dot(v, v))))


def main():
    meta, arrays = [], {}
    for name, spec, D, seed, dist, pseed in CASES:
        x = row(seed, D, dist)
        c = compressors.initCompressor(spec, D)
        m = {"name": name, "spec": spec, "D": D, "seed": seed, "dist": dist, "pattern_seed": pseed,
             "x_sha": sha(x), "torch_threads": torch.get_num_threads(), "torch": torch.__version__, "K": int(getattr(c, "K", 0))}
        if pseed is not None:
            rs = np.random.RandomState(pseed)
            c.generateCompressPattern(rs, "cpu", 0, None)
            m["testp_sha"] = sha(c.testp.numpy())
        y = c.compressVector(torch.from_numpy(x.copy())).numpy()
        m["out_sha"] = sha(y)
        m["need"] = float(c.last_need_to_send_advance)
        nz = np.flatnonzero(y)
        m["nnz"] = int(nz.size)
        if spec.startswith("topk"):
            arrays[f"{name}_ind"] = nz.astype(np.int32)
            assert nz.size == c.K
        else:
            pn = np.float32(torch.norm(torch.from_numpy(x), 2).item())
            ex = exact_norm(x)
            m["pnorm_bits"] = int(pn.view(np.uint32))
            m["exact_norm_bits"] = int(ex.view(np.uint32))
            m["pnorm_ulps_from_exact"] = int(pn.view(np.int32)) - int(ex.view(np.int32))
            lev = np.rint(np.abs(y[nz]).astype(np.float64) / float(pn) * c.s).astype(np.int64)
            m["level_hist"] = np.bincount(lev, minlength=c.s + 1).tolist()
            m["l1_over_l2"] = float(np.abs(x).astype(np.float64).sum() / float(ex))
            samp = np.random.default_rng(seed + 1)
            idx = np.concatenate([samp.choice(nz, 2048, replace=False), samp.choice(D, 2048, replace=False)])
            idx = np.unique(idx)
            arrays[f"{name}_idx"] = idx.astype(np.int32)
            arrays[f"{name}_val"] = y[idx]
        meta.append(m)
        print(name, {k: v for k, v in m.items() if k != "level_hist"}, flush=True)
    np.savez_compressed(os.path.join(HERE, "rows.npz"), **arrays)
    with open(os.path.join(HERE, "rows.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{len(meta)} row-size cases written")


if __name__ == "__main__":
    main()
