"""Inference sampling path of the VAE-U-Net, MI355X-first.

Drop-ins for the reference's uncertainty workload, same names, arguments and
results:

* ``utils/vae_utils.py``: ``sample_from_latent`` (5-10), ``encode_images``
  (13-25), ``generate_predictions`` (28-76), ``calculate_latent_stats``
  (79-103);
* ``visualize_vae.py``: ``predict_full_image`` (61-87),
  ``predict_with_patches`` (243-415), ``calculate_uncertainty_metrics``
  (90-117), and ``segmentation_distribution`` = the sampling loop of
  ``get_segmentation_distribution_from_image`` (578-652) on an image tensor
  (the dataset lookup is out of scope).

What differs from the reference is HOW it runs:

* the encoder runs ONCE per image (per patch batch), and the N latent samples
  go through the decoder as ONE batched pass of N x B images (the reference
  loops N times over encoder + decoder); in eval mode the encoder features
  do not depend on z, so the results are the same;
* everything stays on the device: patch extraction (``vu_input_pack`` on a
  window), the per-patch resize (``vu_upsample_fwd``), sigmoid, the
  feathered blending (``vu_patch_blend``, patch order preserved: the same fp32
  accumulation order as the reference's CPU accumulation), the final
  division and the uncertainty maps are HIP kernels; the reference moves every
  patch prediction to the host.

Randomness: every sampling entry point takes an optional ``eps`` (the
standard-normal draws, [num_samples, B, latent_dim]) so a run can be
reproduced exactly; without it the draws come from torch's RNG like the
reference's ``torch.randn_like``.
"""
import math

import torch

from . import engine as E
from . import kernels as K
from . import vae_engine as V
from ._lib import F32

CL = torch.channels_last


# ---------------------------------------------------------------------------
# building blocks
# ---------------------------------------------------------------------------
def _mode(model, device):
    model.eval()
    return E.current_mode(device)


def _features(model, M, x):
    """Encoder features in NHWC storage of the mode (fused ResNet34 encoder, or
    any module returning the five feature maps)."""
    from .unet_resnet import ResNet34Features
    if isinstance(model.encoder, ResNet34Features):
        cp = (x.shape[1] + 7) // 8 * 8
        feats, _ = V.encoder_fwd(M, model.encoder, E.to_act(M, x, cp), cp)
        return feats
    return [E.to_act(M, f) for f in model.encoder(x)]


def _heads(model, M, f4):
    """mu_head / logvar_head (unet_resnet.py:140-147): conv1x1 + global average
    pool, computed as the per-sample channel mean followed by an [L x C] map."""
    N = f4.shape[0]
    pooled = V.sample_sum(M, f4, 1.0 / (f4.shape[2] * f4.shape[3]))
    out = []
    for head in (model.mu_head[0], model.logvar_head[0]):
        o = torch.empty((N, model.latent_dim), dtype=torch.float32, device=f4.device)
        K.call("vu_linear_small_fwd", K.ptr(pooled), N, f4.shape[1], K.ptr(head.weight), K.ptr(head.bias),
               model.latent_dim, K.ptr(o), K.stream())
        out.append(o)
    return out[0], out[1]


def _repeat(M, t, n):
    """[B, C, H, W] NHWC -> [n*B, C, H, W] (copy k at rows k*B..k*B+B-1)."""
    if n == 1:
        return t
    B, C_, H, W = t.shape
    out = K.empty_act(n * B, C_, H, W, t.dtype, t.device)
    for k in range(n):
        K.copy(t, out[k * B:(k + 1) * B])
    return out


def _decode(model, M, feats, z, skip_always=False):
    """z_initial / DecoderBlocks / final_conv (unet_resnet.py:224-237) for a
    latent vector z [B', L] over features of batch B'; returns the final_conv
    output [B', n_classes, h, w] (fp32 NHWC, decoder resolution)."""
    N = z.shape[0]
    H4, W4 = feats[-1].shape[2], feats[-1].shape[3]
    zps = [None] * len(model.decoder_blocks)
    if V.latent_vectors_ok(M, model, N):
        # z_initial and every z_proj on the [N, L] vectors, maps written once
        cons, zps = V.latent_consumers(M, model, feats, N, skip_always)
        V.latent_fwd(M, z.float().contiguous(), cons)
        V.zbias_tables(M, [c.zsc for c in cons if c.zsc is not None])
        h = cons[0].out if model.use_bottleneck else feats[-1]
    elif model.use_bottleneck:
        h, _ = V.cbr1x1_fwd(M, model.z_initial, V.latent_map(M, z, N, H4, W4))
    else:
        h = feats[-1]
    for i, blk in enumerate(model.decoder_blocks):
        use = i < len(feats) - 1 and (skip_always or model.use_skip)
        h, _ = V.decoder_fwd(M, blk, h, feats[-(i + 2)] if use else None, z, zp_vec=zps[i])
    out, _ = E.outconv_fwd(M, model.final_conv, h)
    return out


def _latents(mu, logvar, n, temperature, eps, sample):
    """z for n draws, sample-major [n*B, L]: mu + eps*temperature*exp(0.5*logvar)."""
    B, L = mu.shape
    if not sample:
        return mu.repeat(n, 1) if n > 1 else mu
    if eps is None:
        eps = torch.randn((n, B, L), device=mu.device)
    eps = eps.to(device=mu.device, dtype=torch.float32).reshape(n * B, L)
    if temperature != 1.0:
        eps = eps * float(temperature)
    eps = eps.contiguous()
    # keep every operand referenced until the launch is enqueued (a temporary
    # freed early goes straight back to the caching allocator)
    mu_r = mu.repeat(n, 1) if n > 1 else mu
    lv_r = logvar.repeat(n, 1) if n > 1 else logvar
    z = torch.empty((n * B, L), dtype=torch.float32, device=mu.device)
    K.call("vu_reparam_fwd", K.ptr(mu_r), K.ptr(lv_r), K.ptr(eps), n * B * L, K.ptr(z), K.stream())
    return z


def _resize(x, Ho, Wo):
    """bilinear, align_corners=True, fp32 NHWC -> fp32 NHWC (Ho, Wo)."""
    N, C_, H, W = x.shape
    if (H, W) == (Ho, Wo):
        return x
    y = K.empty_act(N, C_, Ho, Wo, torch.float32, x.device)
    K.upsample_fwd(x, y, Ho, Wo, 0, 0, F32)
    return y


def _sigmoid(x):
    y = torch.empty_like(x)
    K.call("vu_sigmoid", K.ptr(x), x.numel(), K.ptr(y), K.stream())
    return y


def _nchw1(x):
    """[B, 1, H, W] NHWC fp32 -> a standard contiguous tensor (no copy for C == 1)."""
    return x.contiguous() if x.shape[1] == 1 else x.contiguous()


# ---------------------------------------------------------------------------
# utils/vae_utils.py
# ---------------------------------------------------------------------------
def sample_from_latent(mu, logvar, temperature=1.0, eps=None):
    """vae_utils.py:5-10: mu + randn * exp(0.5*logvar) * temperature."""
    return _latents(mu.float().contiguous(), logvar.float().contiguous(), 1, temperature,
                    None if eps is None else eps.reshape(1, *mu.shape), True)


@torch.no_grad()
def encode_images(model, images):
    """vae_utils.py:13-25: eval mode, (mu, logvar) of the images."""
    M = _mode(model, images.device)
    return _heads(model, M, _features(model, M, images)[-1])


@torch.no_grad()
def generate_predictions(model, images, temperature=1.0, num_samples=3, eps=None):
    """vae_utils.py:28-76: the mean over ``num_samples`` latent draws of the
    final_conv output (decoder resolution, before any resize).  Sampling is
    skipped only for latent_injection == 'none' (as the reference)."""
    M = _mode(model, images.device)
    feats = _features(model, M, images)
    mu, logvar = _heads(model, M, feats[-1])
    sample = getattr(model, "latent_injection", "all") != "none"
    z = _latents(mu, logvar, num_samples, temperature, eps, sample)
    rep = [_repeat(M, f, num_samples) for f in feats]
    pred = _decode(model, M, rep, z)
    if num_samples == 1:
        return pred
    B = images.shape[0]
    out = torch.empty((B,) + tuple(pred.shape[1:]), dtype=torch.float32, device=pred.device,
                      memory_format=CL)
    K.call("vu_mean_groups", K.ptr(pred), num_samples, out.numel(), K.ptr(out), K.stream())
    return out


def calculate_latent_stats(mu, logvar):
    """vae_utils.py:79-103 (host-side logging statistics of [B, L] tensors)."""
    mean_mu = mu.mean(dim=0)
    var = torch.exp(logvar)
    mean_var = var.mean(dim=0)
    active = ((mean_mu.abs() > 0.1) | (mean_var < 0.9) | (mean_var > 1.1)).sum().item()
    kl_per_dim = 0.5 * (mean_mu.pow(2) + mean_var - logvar.mean(dim=0) - 1)
    return {"active_dims": active, "total_dims": mu.shape[1], "activity_ratio": active / mu.shape[1],
            "total_kl": kl_per_dim.sum().item(), "mean_mu_abs": mean_mu.abs().mean().item(),
            "mean_var": mean_var.mean().item()}


# ---------------------------------------------------------------------------
# visualize_vae.py
# ---------------------------------------------------------------------------
def _z_vector(z, n):
    """z [B|1, L, 1, 1] or [B|1, L] (spatially constant) -> [n, L] fp32."""
    zv = z.reshape(z.shape[0], -1).float().contiguous()
    if zv.shape[0] == n:
        return zv
    if zv.shape[0] != 1:
        raise ValueError("z batch must be 1 or match the image batch")
    return zv.expand(n, -1).contiguous()


@torch.no_grad()
def predict_full_image(model, img, z):
    """visualize_vae.py:61-87: sigmoid(resize(final_conv(decoder(encoder(img), z)))).
    z: [B|1, L, 1, 1] (or a list/stack of draws: [S*B, L, 1, 1] decodes every
    draw in one batched pass and returns [S*B, C, H, W])."""
    M = _mode(model, img.device)
    feats = _features(model, M, img)
    B = img.shape[0]
    S = max(1, z.shape[0] // B) if z.shape[0] != 1 else 1
    zv = _z_vector(z, S * B)
    rep = [_repeat(M, f, S) for f in feats]
    out = _decode(model, M, rep, zv, skip_always=True)
    out = _resize(out, img.shape[2], img.shape[3])
    return _sigmoid(_nchw1(out))


def _patch_grid(H, W, patch_size, overlap):
    stride = patch_size - overlap
    nh = math.ceil((H - overlap) / stride)
    nw = math.ceil((W - overlap) / stride)
    info = []
    for i in range(nh):
        for j in range(nw):
            sh, sw = i * stride, j * stride
            if i == nh - 1:
                eh = H
                sh = max(0, eh - patch_size)
            else:
                eh = min(sh + patch_size, H)
            if j == nw - 1:
                ew = W
                sw = max(0, ew - patch_size)
            else:
                ew = min(sw + patch_size, W)
            info.append((sh, eh, sw, ew))
    return nh, nw, info


def _crop(img, sh, eh, sw, ew, cp, d):
    """img[:, :, sh:eh, sw:ew] -> NHWC storage (Cp channels) by one pack launch."""
    N, C_ = img.shape[0], img.shape[1]
    x = img.float() if img.dtype != torch.float32 else img
    st = x.stride()
    out = K.empty_act(N, cp, eh - sh, ew - sw, torch.bfloat16 if d else torch.float32, x.device)
    base = x.data_ptr() + (sh * st[2] + sw * st[3]) * x.element_size()
    K.call("vu_input_pack", base, st[0], st[1], st[2], st[3], N, C_, eh - sh, ew - sw, cp, K.ptr(out), d,
           K.stream())
    return out


@torch.no_grad()
def predict_with_patches(model, img, z, patch_size=512, overlap=None, batch_size=4, samples=None):
    """visualize_vae.py:243-415 for a B = 1 image: overlapping patches
    (stride = patch - overlap, the last row/column flush with the border),
    ``batch_size`` patches per encoder/decoder pass, sigmoid, resize to the
    patch, ramp-tapered weights, weighted average.  ``z`` [1, L, 1, 1]; with
    ``samples`` = S draws stacked in z ([S, L, 1, 1]) every patch batch is
    encoded once and decoded for all S draws in one pass: returns [S, 1, H, W]."""
    from .unet_resnet import ResNet34Features
    M = _mode(model, img.device)
    B, C_, H, W = img.shape
    if B != 1:
        raise ValueError("predict_with_patches handles one image (B == 1), as the reference")
    if overlap is None:
        overlap = max(min(int(patch_size * 0.2), 128), 32)
    S = samples or 1
    zall = _z_vector(z, S)                                 # [S, L]
    nh, nw, info = _patch_grid(H, W, patch_size, overlap)
    dev = img.device
    out = torch.zeros((S, 1, H, W), dtype=torch.float32, device=dev)
    wsum = torch.zeros_like(out)
    ramp = torch.linspace(0, 1, overlap).to(dev) if overlap > 0 else torch.zeros(1, device=dev)
    fused = isinstance(model.encoder, ResNet34Features)
    cp = (C_ + 7) // 8 * 8 if fused else C_
    for b0 in range(0, len(info), batch_size):
        coords = info[b0:b0 + batch_size]
        nb = len(coords)
        ph = max(c[1] - c[0] for c in coords)
        pw = max(c[3] - c[2] for c in coords)
        if any((c[1] - c[0], c[3] - c[2]) != (ph, pw) for c in coords):
            raise NotImplementedError("patches of different sizes in one batch")
        crops = [_crop(img, *c, cp, M.d) for c in coords]
        if nb == 1:
            stack = crops[0]
        else:
            stack = K.empty_act(nb, cp, ph, pw, crops[0].dtype, dev)
            for k, t in enumerate(crops):
                K.copy(t, stack[k:k + 1])
        if fused:
            feats, _ = V.encoder_fwd(M, model.encoder, stack, cp)
        else:
            xin = stack[:, :C_].float().contiguous()
            feats = [E.to_act(M, f) for f in model.encoder(xin)]
        rep = [_repeat(M, f, S) for f in feats]
        zb = zall.repeat_interleave(nb, 0) if nb > 1 else zall  # [S*nb, L], sample-major
        pred = _sigmoid(_decode(model, M, rep, zb, skip_always=True))  # [S*nb, 1, h, w]
        pred = _resize(pred, ph, pw).contiguous()
        for k, (sh, eh, sw, ew) in enumerate(coords):
            gi = b0 + k
            i, j = divmod(gi, nw)
            for s in range(S):
                K.call("vu_patch_blend", K.ptr(pred[s * nb + k]), ph * pw, 1, ph, pw, K.ptr(out[s]),
                       K.ptr(wsum[s]), H, W, sh, sw, K.ptr(ramp), overlap, int(i > 0), int(i < nh - 1),
                       int(j > 0), int(j < nw - 1), K.stream())
    K.call("vu_blend_finish", K.ptr(out), K.ptr(wsum), out.numel(), K.stream())
    return out if samples else out[0:1]


@torch.no_grad()
def segmentation_distribution(model, img, num_samples=32, patch_size=None, overlap=None, temperature=1.0,
                              batch_size=4, eps=None, sample_batch=8):
    """The sampling loop of get_segmentation_distribution_from_image
    (visualize_vae.py:601-652) on an image tensor [1, C, H, W]: returns
    (segmentations [num_samples, 1, H, W], mu, logvar).  Draws are decoded
    ``sample_batch`` at a time in one batched pass (the encoder once per
    image / patch batch)."""
    mu, logvar = encode_images(model, img)
    sample = getattr(model, "latent_injection", "all") not in ["none"]
    if eps is None and sample:
        eps = torch.randn((num_samples,) + tuple(mu.shape), device=img.device)
    H, W = img.shape[2], img.shape[3]
    segs = torch.empty((num_samples, 1, H, W), dtype=torch.float32, device=img.device)
    for s0 in range(0, num_samples, sample_batch):
        n = min(sample_batch, num_samples - s0)
        z = _latents(mu, logvar, n, temperature, eps[s0:s0 + n] if sample else None, sample)
        z4 = z.view(n, -1, 1, 1)
        if patch_size is not None and patch_size > 0:
            ov = overlap if overlap is not None else max(min(int(patch_size * 0.2), 128), 32)
            segs[s0:s0 + n] = predict_with_patches(model, img, z4, patch_size, ov, batch_size, samples=n)
        else:
            segs[s0:s0 + n] = predict_full_image(model, img, z4).view(n, 1, H, W)
    return segs, mu, logvar


@torch.no_grad()
def calculate_uncertainty_metrics(segmentations):
    """visualize_vae.py:90-117 over dim 0 of [S, B, 1, H, W] (or [S, 1, H, W]):
    mean, std (unbiased), entropy, mutual_info, coeff_var, channel squeezed."""
    seg = segmentations.float().contiguous()
    S = seg.shape[0]
    n = seg[0].numel()
    maps = [torch.empty(seg.shape[1:], dtype=torch.float32, device=seg.device) for _ in range(5)]
    K.call("vu_uncertainty", K.ptr(seg), S, n, *[K.ptr(m) for m in maps], K.stream())
    return {k: m.squeeze(1) for k, m in zip(("mean", "std", "entropy", "mutual_info", "coeff_var"), maps)}
