#!/usr/bin/env python3
"""Generate tests/golden/rank_k.{npz,json} from the REAL reference's Rank-K compressor.

Test infrastructure only, run in the development container where the reference is mounted
read-only (compressors.py imports only torch, math and numpy, so it is imported
directly from /root/reference/fl_pytorch/utils).  For each case it records the input, the
reference ``compressVector`` output (compressors.py:336-364: torch.linalg.svd of the A x B view,
U_K diag(S_K) Vt_K, fp32 on the CPU), the wire count ``last_need_to_send_advance`` and the
constants A, B, K, alpha (makeRankKCompressor, compressors.py:151-172).

A truncated SVD is unique only up to the singular-vector signs and the basis of a repeated
singular value; the reconstruction U_K S_K Vt_K is unique when S_K > S_{K+1}.  The cases use
inputs whose spectra have that gap (or K >= rank), so the fixtures pin the output to fp32
rounding of the LAPACK path, and the tests compare with a stated tolerance.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference/fl_pytorch/utils")
import compressors  # noqa: E402  (the reference module, imported, never copied)


def low_rank(rs, A, B, r, noise):
    u = rs.randn(A, r) * np.linspace(3.0, 1.0, r)
    v = rs.randn(r, B)
    return ((u @ v) + noise * rs.randn(A, B)).astype(np.float32).reshape(-1)


def cases():
    rs = np.random.RandomState(20240607)
    out = []
    out.append(("rank_k:100%", 8, np.array([1, 2, 3, 4, 5, 6, 7, -8], dtype=np.float32)))
    out.append(("rank_k:1", 2465, rs.randn(2465).astype(np.float32)))
    out.append(("rank_k:3", 2465, low_rank(rs, 85, 29, 3, 1e-3)))
    out.append(("rank_k:5", 4096, low_rank(rs, 64, 64, 3, 1e-2)))
    out.append(("rank_k:1", 1000, np.outer(rs.randn(40), rs.randn(25)).astype(np.float32).reshape(-1)))
    out.append(("rank_k:4", 97, rs.randn(97).astype(np.float32)))           # prime: A = 97, B = 1
    out.append(("rank_k:10", 10000, low_rank(rs, 100, 100, 12, 1e-2)))
    out.append(("rank_k:2", 30000, low_rank(rs, 150, 200, 2, 1e-3)))
    out.append(("rank_k:50", 12, rs.randn(12).astype(np.float32)))          # K > min(A, B)
    out.append(("rank_k:8", 65536, low_rank(rs, 256, 256, 8, 1e-3)))
    return out


def main():
    torch.set_num_threads(1)
    meta, arrays = [], {}
    for i, (spec, D, x) in enumerate(cases()):
        c = compressors.initCompressor(spec, D)
        y = c.compressVector(torch.from_numpy(x.copy()))
        meta.append({"spec": spec, "D": D, "A": c.A, "B": c.B, "K": c.K, "alpha": c.alpha,
                     "need": int(c.last_need_to_send_advance)})
        arrays[f"x{i}"] = x
        arrays[f"y{i}"] = y.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "rank_k.npz"), **arrays)
    with open(os.path.join(HERE, "rank_k.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{len(meta)} rank_k cases written")


if __name__ == "__main__":
    main()
