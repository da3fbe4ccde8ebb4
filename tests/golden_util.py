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


def _rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def _rand(seed, shape, lo=-1.0, hi=1.0):
    return _rng(seed).uniform(lo, hi, size=shape).astype(np.float32)


# ---- UNetResNet tail fixtures (oracle/gen_golden.py gen_vae): everything that
# can be regenerated from a seed is regenerated, not stored ----------------------
VAE_TAIL = ("mu_head", "logvar_head", "z_initial", "decoder_blocks", "final_conv")


def vae_feature(shape, seed, i):
    """Seeded stand-in encoder feature i (non-negative, like post-ReLU maps)."""
    return _rand(seed * 10 + i, shape, 0.0, 1.0)


def vae_feature_shapes(B, S):
    return [(B, 64, S // 2, S // 2), (B, 64, S // 4, S // 4), (B, 128, S // 8, S // 8),
            (B, 256, S // 16, S // 16), (B, 512, S // 32, S // 32)]


def vae_eps(B, seed):
    return _rand(seed + 7, (B, 32), -2.0, 2.0)


def vae_target(B, S, seed):
    return (_rand(seed + 8, (B, 1, S, S), 0.0, 1.0) < 0.05).astype(np.float32)


def seed_vae_tail(model, seed):
    """Seeded init of every non-encoder submodule of a UNetResNet (the
    reference's or vaeunet_amd's: same submodule names)."""
    from vaeunet_amd.init import seeded_init_
    for i, name in enumerate(VAE_TAIL):
        seeded_init_(getattr(model, name), seed + i)
