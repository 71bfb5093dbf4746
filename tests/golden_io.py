"""Loaders for the committed golden fixtures (tests/golden/, made by make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    data = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return meta, data


def shift_inputs(seed, D):
    """Inputs of the shift fixtures (make_golden_shift.py): g, b and a third vector (MARINA's g_prev)."""
    g = np.random.default_rng(seed)
    a = g.standard_normal(D).astype(np.float32)
    b = (a + 0.3 * g.standard_normal(D)).astype(np.float32)
    b[:5] = a[:5]                                     # exact zeros in the difference
    x3 = g.standard_normal(D).astype(np.float32)
    return a, b, x3


def shift_fingerprint(*xs):
    return [float(np.sum(x.astype(np.float64))) for x in xs]
