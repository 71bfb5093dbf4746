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
