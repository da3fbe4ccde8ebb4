"""Helpers to read tests/golden/*.npz (fixtures generated from the reference by
oracle/gen_golden.py; data only)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def state_of(rec):
    """p0.<key> entries -> state dict of torch tensors."""
    return {k[3:]: torch.from_numpy(v) for k, v in rec.items() if k.startswith("p0.")}


def relerr(a, b, floor=1e-3):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), floor))
