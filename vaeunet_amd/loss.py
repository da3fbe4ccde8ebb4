"""Training objective (drop-in for the reference's utils/loss.py).

CombinedLoss / dice_loss / DiceLoss / kl_with_free_bits / KLAnnealer with the
reference's signatures and semantics (loss.py:6-63, 114-170), computed by the
fused HIP reduction kernels of csrc/loss.hip: one pass produces the four
global sums (BCE, sum p*t, sum p, sum t) in fp64, the loss is formed on the
device and the backward is one elementwise kernel — no host synchronisation
(the reference's ``isnan().any()`` check at loss.py:12 becomes a per-element
NaN->0 inside the kernel, which is what its nan_to_num achieves).

Deviation, documented: the reference's ``.view(-1)`` (loss.py:17-18) raises on
channels_last logits with more than one class; here the sums are taken in
memory order, which equals the reference's result whenever it runs.
"""
import torch
import torch.nn as nn

from . import _lib
from ._lib import ptr, call, query, stream

CL = torch.channels_last


def _dense_pair(inputs, targets):
    if inputs.device.type != "cuda":
        raise RuntimeError("vaeunet_amd losses run on MI355X (HIP) devices only")
    x = inputs.float() if inputs.dtype != torch.float32 else inputs
    fmt = CL if (x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=CL)) \
        else torch.contiguous_format
    x = x.contiguous(memory_format=fmt)
    t = targets.to(device=x.device, dtype=torch.float32)
    if t.shape != x.shape:
        raise ValueError(f"target shape {tuple(t.shape)} != input shape {tuple(x.shape)}")
    t = t.contiguous(memory_format=fmt)
    return x, t


class _BceDice(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, t, smooth, w_bce, w_dice):
        n = x.numel()
        sums = torch.empty(4, dtype=torch.float64, device=x.device)
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        parts = torch.empty(2, dtype=torch.float32, device=x.device)
        ws = torch.empty(query("vu_loss_workspace_bytes") // 8 + 1, dtype=torch.float64,
                         device=x.device)
        call("vu_bce_dice_fwd2", ptr(x), ptr(t), n, ptr(sums), smooth, w_bce, w_dice, ptr(loss),
             ptr(parts), ptr(ws), stream())
        ctx.save_for_backward(x, t, sums)
        ctx.cfg = (smooth, w_bce, w_dice)
        ctx.mark_non_differentiable(parts)
        # no zero gradient materialised for `parts` (one fill launch less per step)
        ctx.set_materialize_grads(False)
        return loss, parts

    @staticmethod
    def backward(ctx, gout, _gparts):
        x, t, sums = ctx.saved_tensors
        smooth, w_bce, w_dice = ctx.cfg
        if gout is None:
            return None, None, None, None, None
        g = gout.float().contiguous()
        grad = torch.empty_like(x)
        call("vu_bce_dice_bwd", ptr(x), ptr(t), x.numel(), ptr(sums), smooth, w_bce, w_dice,
             ptr(g), ptr(grad), stream())
        return grad, None, None, None, None


def _combined(inputs, targets, smooth, w_bce, w_dice):
    x, t = _dense_pair(inputs, targets)
    loss, parts = _BceDice.apply(x, t, float(smooth), float(w_bce), float(w_dice))
    return loss, parts


def dice_loss(inputs, targets, smooth=1.0):
    """1 - soft Dice over the whole batch (loss.py:6-28)."""
    return _combined(inputs, targets, smooth, 0.0, 1.0)[0]


class DiceLoss(nn.Module):
    def __init__(self, smooth=1.0):
        super().__init__()
        self.smooth = smooth

    def forward(self, inputs, targets):
        return dice_loss(inputs, targets, self.smooth)


class CombinedLoss(nn.Module):
    """bce_weight * BCEWithLogits(mean) + dice_weight * dice_loss (loss.py:44-63).

    After a call, ``self.last_parts`` holds the device tensor [total, bce,
    dice_loss] (for logging without an extra pass)."""

    def __init__(self, bce_weight=0.5, dice_weight=0.5):
        super().__init__()
        self.bce_weight = bce_weight
        self.dice_weight = dice_weight
        self.last_parts = None

    def forward(self, inputs, targets):
        loss, parts = _combined(inputs, targets, 1.0, self.bce_weight, self.dice_weight)
        self.last_parts = parts
        return loss


class KLAnnealer:
    """KL weight schedule (loss.py:114-145); host arithmetic."""

    def __init__(self, kl_start=0.0, kl_end=1.0, warmup_epochs=10, strategy='linear'):
        self.kl_start = kl_start
        self.kl_end = kl_end
        self.warmup_epochs = warmup_epochs
        self.strategy = strategy

    def get_weight(self, epoch, batch=None, num_batches=None):
        if self.strategy == 'constant':
            return self.kl_end
        if batch is not None and num_batches is not None:
            progress = (epoch + batch / num_batches) / self.warmup_epochs
        else:
            progress = epoch / self.warmup_epochs
        progress = min(progress, 1.0)
        span = self.kl_end - self.kl_start
        if self.strategy == 'linear':
            return self.kl_start + progress * span
        if self.strategy == 'cyclical':
            return self.kl_start + (progress % 1.0) * span
        return self.kl_end


class _KL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, logvar, free_bits):
        B, L = mu.shape
        val = torch.empty((), dtype=torch.float32, device=mu.device)
        call("vu_kl_free_bits2", ptr(mu), ptr(logvar), B, L, free_bits, None, ptr(val), None, None,
             stream())
        ctx.save_for_backward(mu, logvar)
        ctx.fb = free_bits
        return val

    @staticmethod
    def backward(ctx, g):
        mu, logvar = ctx.saved_tensors
        B, L = mu.shape
        gmu = torch.empty_like(mu)
        glv = torch.empty_like(logvar)
        gs = g.float().contiguous()
        call("vu_kl_free_bits2", ptr(mu), ptr(logvar), B, L, ctx.fb, ptr(gs), None, ptr(gmu),
             ptr(glv), stream())
        return gmu, glv, None


def kl_with_free_bits(mu, logvar, free_bits=1e-4):
    """KL(q||N(0,I)) per latent dim, clamp +-100, free-bits floor, sum(1).mean() (loss.py:148-170)."""
    if mu.device.type != "cuda":
        raise RuntimeError("vaeunet_amd losses run on MI355X (HIP) devices only")
    m = mu.float().contiguous()
    v = logvar.float().contiguous()
    if m.dim() != 2:
        m, v = m.reshape(m.shape[0], -1), v.reshape(v.shape[0], -1)
    return _KL.apply(m, v, float(free_bits))
