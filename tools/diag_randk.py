"""Diagnostic (not a test): where does the device RandK fold differ from the oracle?"""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import codecs as oc
from oracle import devrng
from flpytorch_amd import aggregation as ag

for n, d, spec in [(3, 100_003, "randk:1%"), (1, 8192, "randk:1%"), (2, 4096, "randk:1"), (1, 4096, "randk:10")]:
    seed, client0 = 20241015, 11
    rows = np.random.default_rng([n, d]).standard_normal((n, d)).astype(np.float32)
    enc, sets = [], []
    for i in range(n):
        o = oc.OracleCompressor(spec, d)
        o.S = devrng.randk_indices(seed, client0 + i, d, o.K)
        sets.append(set(o.S.tolist()))
        enc.append(o.compress(rows[i]))
    want = oc.reduce_plain(enc)
    got = ag.UplinkReducer(ag.initCompressor(spec, d), seed=seed)(torch.from_numpy(rows).cuda(), client0=client0).cpu().numpy()
    bad = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
    print(spec, n, d, "mismatches", bad.size, "of", d, "nonzero want", np.count_nonzero(want), "nonzero got", np.count_nonzero(got))
    for j in bad[:12]:
        print("  j", j, "chunk", j // 4096, "got", got[j], "want", want[j], "rows keeping", [i for i in range(n) if j in sets[i]],
              "x", [float(rows[i, j]) for i in range(n)])
    gotnz = set(np.nonzero(got)[0].tolist())
    wantnz = set(np.nonzero(want)[0].tolist())
    print("  got-not-want", sorted(gotnz - wantnz)[:10], "want-not-got", sorted(wantnz - gotnz)[:10])
