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


# ---- inference fixtures (oracle/gen_golden.py gen_inference) -----------------
def pyramid_encoder(seed):
    """TEST DOUBLE for the encoder: a deterministic, input-dependent feature
    pyramid [64, 64, 128, 256, 512] at strides 2..32 (relu of an affine map of
    the average-pooled input channels).  Restates nothing of timm."""
    import torch.nn as nn
    import torch.nn.functional as F

    chans = [64, 64, 128, 256, 512]

    class _FI:
        def channels(self):
            return list(chans)

    class PyramidEncoder(nn.Module):
        def __init__(self):
            super().__init__()
            for i, c in enumerate(chans):
                self.register_buffer(f"a{i}", torch.from_numpy(_rand(seed * 100 + 2 * i, (c,), 0.5, 1.5)))
                self.register_buffer(f"b{i}", torch.from_numpy(_rand(seed * 100 + 2 * i + 1, (c,), -0.3, 0.3)))
            self.feature_info = _FI()

        def forward(self, x):
            feats = []
            for i, c in enumerate(chans):
                p = F.avg_pool2d(x, 2 ** (i + 1))
                idx = torch.arange(c, device=x.device) % x.shape[1]
                a, b = getattr(self, f"a{i}"), getattr(self, f"b{i}")
                feats.append(torch.relu(p[:, idx] * a[None, :, None, None] + b[None, :, None, None]))
            return feats

    return PyramidEncoder()


def seed_bn_stats(model, seed):
    """Non-trivial BatchNorm running statistics (eval-mode fixtures)."""
    rng = _rng(seed)
    with torch.no_grad():
        for k, b in model.named_buffers():
            if k.startswith("encoder."):
                continue
            if k.endswith("running_mean"):
                b.copy_(torch.from_numpy(rng.uniform(-0.2, 0.2, size=tuple(b.shape)).astype(np.float32)))
            elif k.endswith("running_var"):
                b.copy_(torch.from_numpy(rng.uniform(0.5, 1.5, size=tuple(b.shape)).astype(np.float32)))


INFER_SEED = 400
INFER_GEN = dict(B=2, S=64, samples=3, temperature=0.7)
INFER_FULL = dict(H=96, W=64)
INFER_PATCH = dict(H=100, W=84, patch=64, batch=4)


def infer_inputs():
    """Seeded inputs of the inference fixtures."""
    g = INFER_GEN
    return {
        "gen_images": _rand(INFER_SEED + 1, (g["B"], 3, g["S"], g["S"]), 0.0, 1.0),
        "gen_eps": _rand(INFER_SEED + 2, (g["samples"], g["B"], 32), -2.0, 2.0),
        "full_img": _rand(INFER_SEED + 3, (1, 3, INFER_FULL["H"], INFER_FULL["W"]), 0.0, 1.0),
        "full_z": _rand(INFER_SEED + 4, (1, 32, 1, 1), -1.5, 1.5),
        "patch_img": _rand(INFER_SEED + 5, (1, 3, INFER_PATCH["H"], INFER_PATCH["W"]), 0.0, 1.0),
        "patch_z": _rand(INFER_SEED + 6, (1, 32, 1, 1), -1.5, 1.5),
        "segs": _rand(INFER_SEED + 7, (5, 1, 12, 10), 0.0, 1.0),
    }
