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


# fp32 adjudication factor: the HIP fp32 path may differ from fp64 by at most
# FP32_ERR_FACTOR x the fp32 oracle's own largest margin error (different
# summation orders: implicit-GEMM K order, fp64-combined BN statistics vs
# torch's CPU reductions), and a flipped pixel's fp64 margin must lie inside
# that envelope.
FP32_ERR_FACTOR = 4.0


def class_margin(lg):
    """Signed class margin: logit(1) - logit(0) for 2 classes, the logit for 1."""
    return (lg[:, 1] - lg[:, 0]) if lg.shape[1] == 2 else lg[:, 0]


def adjudicate_flips(tag, m_gpu, m32, m64):
    """Class-map flips of an fp32 HIP run against the fp32 oracle, judged by
    fp64: the HIP margin error vs fp64 must stay within FP32_ERR_FACTOR x the
    fp32 oracle's own largest margin error, and so must the fp64 |margin| of
    every flipped pixel.  Returns the flip count vs the fp32 oracle."""
    e_ref = float((m32 - m64).abs().max())
    e_gpu = float((m_gpu - m64).abs().max())
    s_gpu, s32, s64 = m_gpu > 0, m32 > 0, m64 > 0
    flips_ref = s_gpu != s32                 # what bench.py's parity block counts
    flips_gpu64 = s_gpu != s64
    flips_ref64 = s32 != s64
    bound = FP32_ERR_FACTOR * e_ref
    m64_at_flips = m64.abs()[flips_ref | flips_gpu64]
    worst = float(m64_at_flips.max()) if m64_at_flips.numel() else 0.0
    print(f"{tag}: fp32 margin error vs fp64: HIP {e_gpu:.3e}, oracle {e_ref:.3e}; flips HIP-vs-fp32-oracle "
          f"{int(flips_ref.sum())}, HIP-vs-fp64 {int(flips_gpu64.sum())}, oracle-fp32-vs-fp64 "
          f"{int(flips_ref64.sum())}; largest fp64 |margin| at a flip {worst:.3e} (bound {bound:.3e})")
    assert e_gpu <= bound, (e_gpu, e_ref)
    assert worst <= bound, (worst, bound)
    return int(flips_ref.sum())
