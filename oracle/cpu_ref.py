"""CPU oracle — TEST INFRASTRUCTURE ONLY.

A clean-room, functional fp32 restatement of the reference's hot path, used by
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg as the checker and the timed CPU baseline.  Nothing in ``vaeunet_amd``
imports it; the product path has no CPU fallback.

Every function takes a flat ``params`` dict keyed exactly like the
reference's state_dict (prefix + key) and plain torch CPU tensors.  Pinned
against tests/golden/*.npz (generated from the reference itself by
oracle/gen_golden.py) in tests/test_oracle.py.

Reference semantics restated (file:line):
  BatchNorm2d train mode ......... torch.nn.BatchNorm2d (unet_parts.py:41,44,12,16,20)
  DoubleConv ...................... unet/unet_parts.py:32-49
  Down ............................ unet/unet_parts.py:51-63
  Up (+F.pad, attention, cat) ..... unet/unet_parts.py:65-95
  AttentionGate ................... unet/unet_parts.py:7-30
  OutConv ......................... unet/unet_parts.py:97-103
  UNet ............................ unet/unet_model.py:6-36
  DecoderBlock .................... unet/unet_resnet.py:31-101
  UNetResNet (VAE) ................ unet/unet_resnet.py:103-279 (encoder: timm
                                    resnet34 features_only, restated; PARITY
                                    UNPINNED — timm absent)
  dice_loss / CombinedLoss ........ utils/loss.py:6-28, 44-63
  KLAnnealer / kl_with_free_bits .. utils/loss.py:114-145, 148-170
  dice_score ...................... utils/metrics.py:8-35
  train step ...................... train.py:381-411 (AdamW train.py:334)
  patch-cache window statistics ... utils/data_loading.py:287-300, 370-397
"""
import math

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------
# primitives
# ----------------------------------------------------------------------------
# Conditioning probe (tests only): when set to a dict, every train-mode
# BatchNorm records (xhat, output) under its prefix and keeps the output's
# gradient, so a test can form the per-channel sums of |terms| of the affine
# gradients (sum |dz| for the bias, sum |dz * xhat| for the weight) -- the
# conditioning of those reductions (tests/test_gpu_config_parity.py).
PROBE = None


def probe_bn_conditioning():
    """{prefix + 'weight' / 'bias': per-channel sum of |terms|} of the probed
    BatchNorms after backward (fp64 run)."""
    out = {}
    for pre, v in PROBE.items():
        if pre.startswith("gate:"):
            continue
        xh, y = v
        dz = y.grad
        out[pre + "bias"] = dz.abs().sum(dim=(0, 2, 3)).detach().double()
        out[pre + "weight"] = (dz * xh.detach()).abs().sum(dim=(0, 2, 3)).double()
    return out


def batch_norm_train(x, p, pre, bufs, momentum=0.1, eps=1e-5):
    """Batch statistics over (N,H,W); biased var for normalisation, unbiased
    for the running estimate (in-place on ``bufs``)."""
    mean = x.mean(dim=(0, 2, 3))
    var = x.var(dim=(0, 2, 3), unbiased=False)
    n = x.numel() // x.shape[1]
    if bufs is not None:
        with torch.no_grad():
            rm, rv = bufs[pre + "running_mean"], bufs[pre + "running_var"]
            rm.mul_(1 - momentum).add_(momentum * mean.detach())
            rv.mul_(1 - momentum).add_(momentum * var.detach() * n / max(n - 1, 1))
            bufs[pre + "num_batches_tracked"] += 1
    xh = (x - mean[None, :, None, None]) / torch.sqrt(var[None, :, None, None] + eps)
    y = xh * p[pre + "weight"][None, :, None, None] + p[pre + "bias"][None, :, None, None]
    if PROBE is not None and y.requires_grad:
        y.retain_grad()
        PROBE[pre] = (xh, y)
    return y


def batch_norm_eval(x, p, pre, bufs, eps=1e-5):
    rm, rv = bufs[pre + "running_mean"], bufs[pre + "running_var"]
    xh = (x - rm[None, :, None, None]) / torch.sqrt(rv[None, :, None, None] + eps)
    return xh * p[pre + "weight"][None, :, None, None] + p[pre + "bias"][None, :, None, None]


def bn(x, p, pre, bufs, train):
    return batch_norm_train(x, p, pre, bufs) if train else batch_norm_eval(x, p, pre, bufs)


def conv(x, p, pre, pad=0, stride=1, bias=True):
    return F.conv2d(x, p[pre + "weight"], p.get(pre + "bias") if bias else None,
                    stride=stride, padding=pad)


def bilinear_ac(x, size):
    """bilinear, align_corners=True: src = dst*(in-1)/(out-1)."""
    return F.interpolate(x, size=size, mode="bilinear", align_corners=True)


# ----------------------------------------------------------------------------
# U-Net blocks
# ----------------------------------------------------------------------------
def double_conv(x, p, pre, bufs, train):
    y = torch.relu(bn(conv(x, p, pre + "0.", 1, bias=False), p, pre + "1.", bufs, train))
    return torch.relu(bn(conv(y, p, pre + "3.", 1, bias=False), p, pre + "4.", bufs, train))


def down(x, p, pre, bufs, train):
    return double_conv(F.max_pool2d(x, 2), p, pre + "maxpool_conv.1.double_conv.", bufs, train)


def attention_gate(g, x, p, pre, bufs, train):
    g1 = bn(conv(g, p, pre + "W_g.0."), p, pre + "W_g.1.", bufs, train)
    x1 = bn(conv(x, p, pre + "W_x.0."), p, pre + "W_x.1.", bufs, train)
    s = torch.relu(g1 + x1)
    q = conv(s, p, pre + "psi.0.")
    z = bn(q, p, pre + "psi.1.", bufs, train)
    psi = torch.sigmoid(z)
    out = x * psi
    if PROBE is not None and out.requires_grad:   # test probe: the gate's intermediates
        for t in (z, psi, out):
            t.retain_grad()
        PROBE["gate:" + pre] = (q, z, psi, out)
    return out


def up(x1, x2, p, pre, bufs, train, bilinear):
    if bilinear:
        x1 = bilinear_ac(x1, (2 * x1.shape[2], 2 * x1.shape[3]))
    else:
        x1 = F.conv_transpose2d(x1, p[pre + "up.weight"], p[pre + "up.bias"], stride=2)
    dy, dx = x2.shape[2] - x1.shape[2], x2.shape[3] - x1.shape[3]
    x1 = F.pad(x1, [dx // 2, dx - dx // 2, dy // 2, dy - dy // 2])
    x2 = attention_gate(x1, x2, p, pre + "attention.", bufs, train)
    return double_conv(torch.cat([x2, x1], dim=1), p, pre + "conv.double_conv.", bufs, train)


def out_conv(x, p, pre):
    return conv(x, p, pre + "conv.")


def unet_forward(x, p, bufs, train=True, bilinear=False):
    x1 = double_conv(x, p, "inc.double_conv.", bufs, train)
    x2 = down(x1, p, "down1.", bufs, train)
    x3 = down(x2, p, "down2.", bufs, train)
    x4 = down(x3, p, "down3.", bufs, train)
    x5 = down(x4, p, "down4.", bufs, train)
    y = up(x5, x4, p, "up1.", bufs, train, bilinear)
    y = up(y, x3, p, "up2.", bufs, train, bilinear)
    y = up(y, x2, p, "up3.", bufs, train, bilinear)
    y = up(y, x1, p, "up4.", bufs, train, bilinear)
    return out_conv(y, p, "outc.")


# ----------------------------------------------------------------------------
# VAE-U-Net (unet_resnet.py) — decoder pinned via DecoderBlock goldens,
# encoder = restated timm resnet34 features_only (parity unpinned)
# ----------------------------------------------------------------------------
def decoder_block(x, skip, z, p, pre, bufs, train, use_attention=True, use_skip=True,
                  use_latent=True):
    size = skip.shape[2:] if skip is not None else (x.shape[2] * 2, x.shape[3] * 2)
    x = bilinear_ac(x, size)
    parts = [x]
    if skip is not None and use_skip:
        if use_attention:
            skip = attention_gate(x, skip, p, pre + "attention.", bufs, train)
        parts.append(skip)
    if use_latent:
        zp = bilinear_ac(z, size)
        zp = torch.relu(bn(conv(zp, p, pre + "z_proj.0."), p, pre + "z_proj.1.", bufs, train))
        parts.append(zp)
    x = torch.cat(parts, dim=1)
    x = torch.relu(bn(conv(x, p, pre + "conv1.0.", 1, bias=False), p, pre + "conv1.1.", bufs, train))
    return torch.relu(bn(conv(x, p, pre + "conv2.0.", 1, bias=False), p, pre + "conv2.1.", bufs, train))


def basic_block(x, p, pre, bufs, train, stride):
    y = torch.relu(bn(conv(x, p, pre + "conv1.", 1, stride, bias=False), p, pre + "bn1.", bufs, train))
    y = bn(conv(y, p, pre + "conv2.", 1, 1, bias=False), p, pre + "bn2.", bufs, train)
    if pre + "downsample.0.weight" in p:
        sc = bn(conv(x, p, pre + "downsample.0.", 0, stride, bias=False), p, pre + "downsample.1.", bufs, train)
    else:
        sc = x
    return torch.relu(y + sc)


def resnet34_features(x, p, pre, bufs, train):
    f0 = torch.relu(bn(conv(x, p, pre + "conv1.", 3, 2, bias=False), p, pre + "bn1.", bufs, train))
    y = F.max_pool2d(f0, 3, 2, 1)
    feats = [f0]
    for li, (nb, st) in enumerate([(3, 1), (4, 2), (6, 2), (3, 2)]):
        for b in range(nb):
            y = basic_block(y, p, f"{pre}layer{li + 1}.{b}.", bufs, train, st if b == 0 else 1)
        feats.append(y)
    return feats


def unet_resnet_forward(x, p, bufs, eps=None, train=True, latent_injection="all"):
    feats = resnet34_features(x, p, "encoder.", bufs, train)
    return unet_resnet_tail(feats, x.shape[2:], p, bufs, eps, train, latent_injection)


def unet_resnet_tail(feats, size, p, bufs, eps=None, train=True, latent_injection="all"):
    """unet_resnet.py:203-240 given the encoder features (pinned by the
    vae_*_256 goldens, generated with a fixed-feature encoder double)."""
    xe = feats[-1]
    mu = conv(xe, p, "mu_head.0.").mean(dim=(2, 3))
    logvar = conv(xe, p, "logvar_head.0.").mean(dim=(2, 3))
    if latent_injection not in ("none", "inject_no_bottleneck"):
        std = torch.exp(0.5 * logvar)
        z = mu + (eps if eps is not None else torch.randn_like(std)) * std
    else:
        z = mu
    zs = bilinear_ac(z[:, :, None, None], xe.shape[2:])
    use_bottleneck = latent_injection not in ("none", "inject_no_bottleneck")
    if use_bottleneck:
        h = torch.relu(bn(conv(zs, p, "z_initial.0."), p, "z_initial.1.", bufs, train))
    else:
        h = xe
    inj = {"all": [1, 1, 1, 1], "inject_no_bottleneck": [1, 1, 1, 1], "first": [1, 0, 0, 0],
           "last": [0, 0, 0, 1], "bottleneck": [0, 0, 0, 0], "none": [0, 0, 0, 0]}[latent_injection]
    for i in range(4):
        h = decoder_block(h, feats[-(i + 2)], zs, p, f"decoder_blocks.{i}.", bufs, train,
                          use_latent=bool(inj[i]))
    out = conv(h, p, "final_conv.")
    return bilinear_ac(out, size), mu, logvar


# ----------------------------------------------------------------------------
# objective (utils/loss.py) and metric (utils/metrics.py)
# ----------------------------------------------------------------------------
def dice_loss(inputs, targets, smooth=1.0):
    s = torch.sigmoid(inputs)
    s = torch.where(torch.isnan(s), torch.zeros_like(s), s)
    s, t = s.reshape(-1), targets.reshape(-1)
    inter = (s * t).sum()
    dice = (2.0 * inter + smooth) / (torch.clamp(s.sum(), min=smooth / 2) +
                                    torch.clamp(t.sum(), min=smooth / 2) + smooth)
    return 1.0 - dice


def bce_with_logits_mean(x, t):
    return (torch.clamp(x, min=0) - x * t + torch.log1p(torch.exp(-x.abs()))).mean()


def combined_loss(x, t, w_bce=0.5, w_dice=0.5):
    return w_bce * bce_with_logits_mean(x, t) + w_dice * dice_loss(x, t)


def kl_with_free_bits(mu, logvar, free_bits=1e-4):
    mu = torch.nan_to_num(mu, nan=0.0)
    logvar = torch.nan_to_num(logvar, nan=0.0)
    kl = 0.5 * (mu * mu + torch.exp(logvar) - logvar - 1)
    kl = torch.clamp(kl, -100.0, 100.0)
    if free_bits > 0:
        kl = torch.maximum(kl, torch.full_like(kl, free_bits))
    return torch.nan_to_num(kl.sum(dim=1).mean(), nan=1e-8)


def kl_weight(epoch, kl_start=0.0, kl_end=1.0, warmup_epochs=10):
    prog = min(epoch / warmup_epochs, 1.0)
    return kl_start + prog * (kl_end - kl_start)


def dice_score(x, t, eps=1e-6):
    a = (x > 0.5).float().reshape(-1)
    b = (t > 0.5).float().reshape(-1)
    den = a.sum() + b.sum()
    if float(den) == 0:
        return torch.tensor(1.0)
    return (2.0 * (a * b).sum() + eps) / (den + eps)


# ----------------------------------------------------------------------------
# AdamW (torch.optim.AdamW defaults: betas (0.9, 0.999), eps 1e-8) + clip
# ----------------------------------------------------------------------------
class AdamW:
    def __init__(self, params, lr=1e-4, weight_decay=1e-5, betas=(0.9, 0.999), eps=1e-8):
        self.params = list(params)
        self.lr, self.wd, self.b1, self.b2, self.eps = lr, weight_decay, betas[0], betas[1], eps
        self.m = [torch.zeros_like(q) for q in self.params]
        self.v = [torch.zeros_like(q) for q in self.params]
        self.t = 0

    @torch.no_grad()
    def step(self):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2 = 1 - self.b2 ** self.t
        for q, m, v in zip(self.params, self.m, self.v):
            if q.grad is None:
                continue
            g = q.grad
            q.mul_(1 - self.lr * self.wd)
            m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
            q.addcdiv_(m, denom, value=-self.lr / bc1)


def clip_grad_norm(params, max_norm=1.0):
    grads = [q.grad for q in params if q.grad is not None]
    total = torch.sqrt(sum((g.double() ** 2).sum() for g in grads)).float()
    coef = max_norm / (total + 1e-6)
    if coef < 1:
        for g in grads:
            g.mul_(coef)
    return total


# ----------------------------------------------------------------------------
# whole train step (train.py:381-411 with grad-accum 1), CPU fp32
# ----------------------------------------------------------------------------
class UNetRef:
    """Parameter container mirroring the reference UNet's state_dict."""

    def __init__(self, state, bilinear=False):
        self.p = {k: v.clone().float().requires_grad_(True) for k, v in state.items()
                  if "running" not in k and "num_batches" not in k}
        self.bufs = {k: v.clone() for k, v in state.items()
                     if "running" in k or "num_batches" in k}
        self.bilinear = bilinear

    def forward(self, x, train=True):
        return unet_forward(x, self.p, self.bufs, train, self.bilinear)


def train_step(model, opt, x, target, clip=1.0):
    logits = model.forward(x, True)
    loss = combined_loss(logits, target)
    for q in model.p.values():
        q.grad = None
    loss.backward()
    total = clip_grad_norm(list(model.p.values()), clip)
    opt.step()
    return logits.detach(), loss.detach(), total


class UNetResNetRef:
    """Parameter container mirroring the reference UNetResNet's state_dict
    (unet_resnet.py:103-279); `eps` fixes reparameterize's draw (:191-194)."""

    def __init__(self, state, latent_injection="all"):
        self.p = {k: v.clone().float().requires_grad_(True) for k, v in state.items()
                  if "running" not in k and "num_batches" not in k}
        self.bufs = {k: v.clone() for k, v in state.items()
                     if "running" in k or "num_batches" in k}
        self.latent_injection = latent_injection

    def forward(self, x, eps=None, train=True):
        return unet_resnet_forward(x, self.p, self.bufs, eps, train, self.latent_injection)


def vae_train_step(model, opt, x, target, eps, beta=1e-3, free_bits=1e-3, clip=1.0):
    """train.py:381-411 for the resnet path: CombinedLoss + beta * KL with free
    bits (utils/loss.py:148-170), clip, AdamW."""
    logits, mu, logvar = model.forward(x, eps, True)
    loss = combined_loss(logits, target) + beta * kl_with_free_bits(mu, logvar, free_bits)
    for q in model.p.values():
        q.grad = None
    loss.backward()
    total = clip_grad_norm(list(model.p.values()), clip)
    opt.step()
    return (logits.detach(), mu.detach(), logvar.detach()), loss.detach(), total


# ----------------------------------------------------------------------------
# patch-cache producer (utils/data_loading.py:287-300 is_valid_patch,
# 370-397 the window loop): per-window integer counts
# ----------------------------------------------------------------------------
def patch_window_stats(img, mask, patch, stride):
    """img [C, H, W] float32, mask [1, H, W]; windows at stride over
    range(0, H - patch + 1, stride) x range(0, W - patch + 1, stride) (row
    major).  Returns (ny, nx, black, lesion): black = #pixels whose channel
    mean (fp32 left-to-right sum, then / C, as torch's CPU mean over dim 0)
    is < 0.1; lesion = #mask pixels > 0.5."""
    import numpy as np
    a = np.asarray(img, dtype=np.float32)
    m = np.asarray(mask, dtype=np.float32)[0]
    s = a[0].copy()
    for k in range(1, a.shape[0]):
        s = (s + a[k]).astype(np.float32)
    is_black = (s / np.float32(a.shape[0])) < np.float32(0.1)
    is_lesion = m > np.float32(0.5)
    _, h, w = a.shape
    ys, xs = list(range(0, h - patch + 1, stride)), list(range(0, w - patch + 1, stride))
    black = np.array([int(is_black[y:y + patch, x:x + patch].sum()) for y in ys for x in xs], np.int64)
    lesion = np.array([int(is_lesion[y:y + patch, x:x + patch].sum()) for y in ys for x in xs], np.int64)
    return len(ys), len(xs), black, lesion
