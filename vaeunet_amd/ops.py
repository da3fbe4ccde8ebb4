"""Dispatcher-level operators: ``torch.ops.vaeunet.*``.

The reference's plugin API is ``torch.nn.Module`` + autograd (the drop-in
classes in this package); §8(b) additionally asks for the hot-path kernels as
custom operators in a ``vaeunet`` library namespace, so they compose with the
dispatcher (fake / meta tensors, ``torch.library.opcheck``,
``torch.compile``, autograd) independently of the module classes.  Each op is
a thin host wrapper over the same C-ABI launches the modules use
(``include/vaeunet.h``); registered for CUDA (HIP) only — on any other device
the dispatcher raises, there is no CPU fallback.

Layout contract (as the modules): activations [N, C, H, W] in
``channels_last`` memory (NHWC in HBM), bf16 (autocast storage) or fp32
(parity mode); 3×3 weights [Cout, Cin, 3, 3] fp32 (the parameter itself; the
kernel layouts are derived caches).  C_in must be a multiple of 8 (the
3-channel image is packed to 8 channels by the UNet module itself).

Reference ops each one replaces:
  conv3x3_fwd / _dgrad / _wgrad  nn.Conv2d(k=3, p=1, bias=False)  unet_parts.py:40,43
  conv_bn_relu                   Conv2d -> BatchNorm2d(train) -> ReLU  unet_parts.py:39-46
  bn_relu_backward               BatchNorm2d(train) + ReLU backward    (autograd of :41-45)
  bn_finalize                    BatchNorm2d(train) statistics + running update (:41,44)
  maxpool2d / maxpool2d_backward nn.MaxPool2d(2)                  unet_parts.py:58
  convT2x2_fwd / _bwd            nn.ConvTranspose2d(in, in//2, 2, 2)   unet_parts.py:76
  upsample_bilinear_ac_fwd / _bwd F.interpolate(bilinear, align_corners=True)  unet_parts.py:73,
                                 unet_resnet.py:79,93,221,238
  attn_gate_fwd / _bwd           AttentionGate (train-mode BatchNorms)  unet_parts.py:7-30
  vae_bottleneck_fwd / _bwd      mu/logvar heads + reparameterize   unet_resnet.py:140-147,191-194
  bce_dice_loss                  CombinedLoss.forward             utils/loss.py:45-63
"""
import ctypes as C
import types
import torch

from . import _lib
from . import engine as E
from . import kernels as K
from ._lib import call, ptr, query, stream
from .engine import conv_layout, convT_layout, w3x3_dgrad, w3x3_fwd, wT_dgrad, wT_fwd
from .loss import _dense_pair

_NS = "vaeunet"


def _act(x, what):
    if x.device.type != "cuda":
        raise RuntimeError(f"vaeunet::{what} runs on MI355X (HIP) devices only; got {x.device}")
    if x.dim() != 4:
        raise ValueError(f"vaeunet::{what}: expected a 4-d [N, C, H, W] activation")
    return x.contiguous(memory_format=torch.channels_last)


def _check_conv(x, w, what):
    if w.dim() != 4 or tuple(w.shape[2:]) != (3, 3) or w.shape[1] != x.shape[1]:
        raise ValueError(f"vaeunet::{what}: weight {tuple(w.shape)} does not match input channels {x.shape[1]}")
    if x.shape[1] % 8:
        raise ValueError(f"vaeunet::{what}: input channels must be a multiple of 8 (got {x.shape[1]})")


def _cl_empty(N, C, H, W, like):
    return torch.empty((N, C, H, W), dtype=like.dtype, device=like.device, memory_format=torch.channels_last)


# ---- conv3x3 ----------------------------------------------------------------
@torch.library.custom_op(f"{_NS}::conv3x3_fwd", mutates_args=(), device_types="cuda")
def conv3x3_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """y = conv2d(x, w, bias, padding=1) on the implicit-GEMM MFMA kernels."""
    x = _act(x, "conv3x3_fwd")
    _check_conv(x, w, "conv3x3_fwd")
    d = K.dcode(x.dtype)
    N, _, H, W = x.shape
    co = w.shape[0]
    y = K.empty_act(N, co, H, W, x.dtype, x.device)
    K.gemm_fwd(K.gather3x3([x]), w3x3_fwd(w, d), co, y, d,
               bias=None if bias is None else bias.float().contiguous())
    return y


@conv3x3_fwd.register_fake
def _(x, w, bias=None):
    return _cl_empty(x.shape[0], w.shape[0], x.shape[2], x.shape[3], x)


@torch.library.custom_op(f"{_NS}::conv3x3_dgrad", mutates_args=(), device_types="cuda")
def conv3x3_dgrad(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dx = conv_transpose2d(dy, w, padding=1): the input gradient of conv3x3_fwd."""
    dy = _act(dy, "conv3x3_dgrad")
    if w.dim() != 4 or tuple(w.shape[2:]) != (3, 3) or w.shape[0] != dy.shape[1]:
        raise ValueError(f"vaeunet::conv3x3_dgrad: weight {tuple(w.shape)} does not match dy {tuple(dy.shape)}")
    d = K.dcode(dy.dtype)
    N, _, H, W = dy.shape
    ci = w.shape[1]
    dx = K.empty_act(N, ci, H, W, dy.dtype, dy.device)
    K.gemm_fwd(K.gather3x3([dy]), w3x3_dgrad(w, d), ci, dx, d, kind="dgrad")
    return dx


@conv3x3_dgrad.register_fake
def _(dy, w):
    return _cl_empty(dy.shape[0], w.shape[1], dy.shape[2], dy.shape[3], dy)


@torch.library.custom_op(f"{_NS}::conv3x3_wgrad", mutates_args=(), device_types="cuda")
def conv3x3_wgrad(x: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    """dw[co, ci, r, s] = sum over pixels of dy * shifted x (fp32 [Cout, Cin, 3, 3])."""
    x = _act(x, "conv3x3_wgrad")
    dy = _act(dy, "conv3x3_wgrad")
    if x.shape[0] != dy.shape[0] or x.shape[2:] != dy.shape[2:] or x.dtype != dy.dtype:
        raise ValueError("vaeunet::conv3x3_wgrad: x and dy must share batch, spatial size and dtype")
    if x.shape[1] % 8:
        raise ValueError(f"vaeunet::conv3x3_wgrad: input channels must be a multiple of 8 (got {x.shape[1]})")
    d = K.dcode(x.dtype)
    co, ci = dy.shape[1], x.shape[1]
    dw = torch.empty((co, ci, 3, 3), dtype=torch.float32, device=x.device)
    K.gemm_wgrad(K.gather1x1([dy]), K.gather3x3([x]), co, 9 * ci, dw, conv_layout(dw), d, False)
    return dw


@conv3x3_wgrad.register_fake
def _(x, dy):
    return torch.empty((dy.shape[1], x.shape[1], 3, 3), dtype=torch.float32, device=x.device)


def _conv_setup(ctx, inputs, output):
    x, w, bias = inputs
    ctx.save_for_backward(x, w)
    ctx.has_bias = bias is not None


def _conv_backward(ctx, gy):
    x, w = ctx.saved_tensors
    gy = gy.to(x.dtype)
    dx = conv3x3_dgrad(gy, w) if ctx.needs_input_grad[0] else None
    dw = conv3x3_wgrad(x, gy).to(w.dtype) if ctx.needs_input_grad[1] else None
    db = None
    if ctx.has_bias and ctx.needs_input_grad[2]:
        db = torch.empty(w.shape[0], dtype=torch.float32, device=x.device)
        K.chan_sum(_act(gy, "conv3x3_fwd backward"), db, False, K.dcode(x.dtype))
    return dx, dw, db


conv3x3_fwd.register_autograd(_conv_backward, setup_context=_conv_setup)


# ---- conv -> BatchNorm2d(train) -> ReLU ------------------------------------
@torch.library.custom_op(f"{_NS}::conv_bn_relu", mutates_args=(), device_types="cuda")
def conv_bn_relu(x: torch.Tensor, w: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor,
                 running_mean: torch.Tensor, running_var: torch.Tensor, momentum: float,
                 eps: float) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """Train-mode conv3x3 -> BN -> ReLU as the modules run it: the batch
    statistics come from the GEMM epilogue, one finalize launch forms
    (scale, shift, mean, invstd) and the momentum update of the running
    statistics (unbiased variance), one stream applies scale/shift + ReLU.
    Functional (so that it is differentiable through the dispatcher): returns
    (a, y, coef, new_running_mean, new_running_var) -- the activation, the
    pre-BN conv output, the [4, Cout] coefficients bn_relu_backward takes, and
    the updated running statistics (nn.BatchNorm2d updates its buffers in
    place; copy them back for that)."""
    x = _act(x, "conv_bn_relu")
    _check_conv(x, w, "conv_bn_relu")
    d = K.dcode(x.dtype)
    N, _, H, W = x.shape
    co = w.shape[0]
    y = K.empty_act(N, co, H, W, x.dtype, x.device)
    st = K.gemm_fwd(K.gather3x3([x]), w3x3_fwd(w, d), co, y, d, stats=True)
    rm, rv = running_mean.float().clone(), running_var.float().clone()
    coef = K.bn_finalize(st, co, gamma, beta, rm, rv, None, momentum, eps)
    a = K.empty_act(N, co, H, W, x.dtype, x.device)
    K.bn_apply(y, a, coef, True, d)
    return a, y, coef, rm, rv


@conv_bn_relu.register_fake
def _(x, w, gamma, beta, running_mean, running_var, momentum, eps):
    y = _cl_empty(x.shape[0], w.shape[0], x.shape[2], x.shape[3], x)
    co = w.shape[0]
    f32 = dict(dtype=torch.float32, device=x.device)
    return (torch.empty_like(y), torch.empty_like(y), torch.empty((4, co), **f32), torch.empty(co, **f32),
            torch.empty(co, **f32))


@torch.library.custom_op(f"{_NS}::bn_relu_backward", mutates_args=(), device_types="cuda")
def bn_relu_backward(da: torch.Tensor, y: torch.Tensor, coef: torch.Tensor, gamma: torch.Tensor,
                     relu: bool) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Backward of a = relu(BN_train(y)) given coef from conv_bn_relu: returns
    (dy, dgamma, dbeta); the two per-channel sums are a deterministic
    two-stage reduction (fp32 per block, fp64 across blocks)."""
    da = _act(da, "bn_relu_backward").to(y.dtype)
    y = _act(y, "bn_relu_backward")
    C_ = y.shape[1]
    dy = torch.empty_like(y)
    dgamma = torch.empty(C_, dtype=torch.float32, device=y.device)
    dbeta = torch.empty_like(dgamma)
    K.bn_backward(da, y, coef.contiguous(), gamma, relu, dgamma, dbeta, False, dy, K.dcode(y.dtype))
    return dy, dgamma, dbeta


@bn_relu_backward.register_fake
def _(da, y, coef, gamma, relu):
    return (_cl_empty(*y.shape, y), torch.empty(y.shape[1], dtype=torch.float32, device=y.device),
            torch.empty(y.shape[1], dtype=torch.float32, device=y.device))


def _cbr_setup(ctx, inputs, output):
    x, w, gamma = inputs[0], inputs[1], inputs[2]
    y, coef = output[1], output[2]
    ctx.save_for_backward(x, w, gamma, y, coef)


def _cbr_backward(ctx, ga, _gy, _gcoef, _grm, _grv):
    x, w, gamma, y, coef = ctx.saved_tensors
    dy, dgamma, dbeta = bn_relu_backward(ga, y, coef, gamma, True)
    dx = conv3x3_dgrad(dy, w) if ctx.needs_input_grad[0] else None
    dw = conv3x3_wgrad(x, dy) if ctx.needs_input_grad[1] else None
    return dx, dw, dgamma, dbeta, None, None, None, None


conv_bn_relu.register_autograd(_cbr_backward, setup_context=_cbr_setup)


# ---- MaxPool2d(2) ------------------------------------------------------------
@torch.library.custom_op(f"{_NS}::maxpool2d", mutates_args=(), device_types="cuda")
def maxpool2d(x: torch.Tensor) -> torch.Tensor:
    """nn.MaxPool2d(2) (floor; the first maximum wins ties, as ATen)."""
    x = _act(x, "maxpool2d")
    return K.maxpool_fwd(x, K.dcode(x.dtype))


@maxpool2d.register_fake
def _(x):
    return _cl_empty(x.shape[0], x.shape[1], x.shape[2] // 2, x.shape[3] // 2, x)


@torch.library.custom_op(f"{_NS}::maxpool2d_backward", mutates_args=(), device_types="cuda")
def maxpool2d_backward(x: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    x = _act(x, "maxpool2d_backward")
    dy = _act(dy, "maxpool2d_backward").to(x.dtype)
    dx = torch.empty_like(x)
    return K.maxpool_bwd(x, dy, dx, None, K.dcode(x.dtype))


@maxpool2d_backward.register_fake
def _(x, dy):
    return _cl_empty(*x.shape, x)


def _pool_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])


def _pool_backward(ctx, gy):
    (x,) = ctx.saved_tensors
    return maxpool2d_backward(x, gy)


maxpool2d.register_autograd(_pool_backward, setup_context=_pool_setup)


# ---- CombinedLoss ------------------------------------------------------------
@torch.library.custom_op(f"{_NS}::bce_dice_loss", mutates_args=(), device_types="cuda")
def bce_dice_loss(logits: torch.Tensor, target: torch.Tensor, smooth: float, w_bce: float,
                  w_dice: float) -> tuple[torch.Tensor, torch.Tensor]:
    """w_bce * BCEWithLogits(mean) + w_dice * (1 - soft Dice) in one fused
    reduction (fp64 block sums, loss formed on the device, no host sync).
    Returns (loss, sums): sums = the four fp64 global sums the backward uses."""
    x, t = _dense_pair(logits, target)
    sums = torch.empty(4, dtype=torch.float64, device=x.device)
    loss = torch.empty((), dtype=torch.float32, device=x.device)
    parts = torch.empty(2, dtype=torch.float32, device=x.device)
    ws = torch.empty(query("vu_loss_workspace_bytes") // 8 + 1, dtype=torch.float64, device=x.device)
    call("vu_bce_dice_fwd2", ptr(x), ptr(t), x.numel(), ptr(sums), smooth, w_bce, w_dice, ptr(loss),
         ptr(parts), ptr(ws), stream())
    return loss, sums


@bce_dice_loss.register_fake
def _(logits, target, smooth, w_bce, w_dice):
    return (torch.empty((), dtype=torch.float32, device=logits.device),
            torch.empty(4, dtype=torch.float64, device=logits.device))


def _loss_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0], inputs[1], output[1])
    ctx.cfg = inputs[2:]


def _loss_backward(ctx, g, _gsums):
    logits, target, sums = ctx.saved_tensors
    x, t = _dense_pair(logits, target)
    smooth, w_bce, w_dice = ctx.cfg
    grad = torch.empty_like(x)
    call("vu_bce_dice_bwd", ptr(x), ptr(t), x.numel(), ptr(sums), smooth, w_bce, w_dice,
         ptr(g.float().contiguous()), ptr(grad), stream())
    return grad.to(logits.dtype), None, None, None, None


bce_dice_loss.register_autograd(_loss_backward, setup_context=_loss_setup)

# ---- BatchNorm2d statistics ------------------------------------------------------
@torch.library.custom_op(f"{_NS}::bn_finalize", mutates_args=(), device_types="cuda")
def bn_finalize(psum: torch.Tensor, pm2: torch.Tensor, tile_rows: int, rows: int, gamma: torch.Tensor,
                beta: torch.Tensor, running_mean: torch.Tensor, running_var: torch.Tensor, momentum: float,
                eps: float) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Combine per-tile (sum, centered M2) partials [tiles, C] (the GEMM
    epilogue's, Chan's formula in fp64, fixed order) into coef [4, C] = (scale,
    shift, mean, invstd) with y * scale + shift = BN_train(y); returns (coef,
    new running_mean, new running_var) (momentum update, unbiased variance)."""
    if psum.device.type != "cuda":
        raise RuntimeError("vaeunet::bn_finalize runs on MI355X (HIP) devices only")
    tiles, C_ = psum.shape
    st = K.Stats(psum.float().contiguous(), pm2.float().contiguous(), tiles, tile_rows, rows)
    rm, rv = running_mean.float().clone(), running_var.float().clone()
    coef = K.bn_finalize(st, C_, gamma.float().contiguous(), beta.float().contiguous(), rm, rv, None, momentum, eps)
    return coef, rm, rv


@bn_finalize.register_fake
def _(psum, pm2, tile_rows, rows, gamma, beta, running_mean, running_var, momentum, eps):
    C_ = psum.shape[1]
    f32 = dict(dtype=torch.float32, device=psum.device)
    return torch.empty((4, C_), **f32), torch.empty(C_, **f32), torch.empty(C_, **f32)


# ---- ConvTranspose2d(k=2, s=2) -------------------------------------------------------
@torch.library.custom_op(f"{_NS}::convT2x2_fwd", mutates_args=(), device_types="cuda")
def convT2x2_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """y = conv_transpose2d(x, w [Cin, Cout, 2, 2], bias, stride=2): one GEMM
    [N*H*W, Cin] x [Cin, 4*Cout] whose epilogue does the pixel shuffle."""
    x = _act(x, "convT2x2_fwd")
    if w.dim() != 4 or tuple(w.shape[2:]) != (2, 2) or w.shape[0] != x.shape[1]:
        raise ValueError(f"vaeunet::convT2x2_fwd: weight {tuple(w.shape)} does not match input {tuple(x.shape)}")
    d = K.dcode(x.dtype)
    N, _, H, W = x.shape
    co = w.shape[1]
    y = K.empty_act(N, co, 2 * H, 2 * W, x.dtype, x.device)
    K.gemm_fwd(K.gather1x1([x]), wT_fwd(w, d), 4 * co, y, d, bias=None if bias is None else bias.float().contiguous(),
               convT=(2 * H, 2 * W, 0, 0, co))
    return y


@convT2x2_fwd.register_fake
def _(x, w, bias=None):
    return _cl_empty(x.shape[0], w.shape[1], 2 * x.shape[2], 2 * x.shape[3], x)


@torch.library.custom_op(f"{_NS}::convT2x2_bwd", mutates_args=(), device_types="cuda")
def convT2x2_bwd(x: torch.Tensor, dy: torch.Tensor, w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dx, dw, dbias) of convT2x2_fwd: dx = the 2x2 sub-pixel gather of dy
    times the weights, dw = x^T x gather(dy) (deterministic split-K), dbias =
    per-channel sum of dy."""
    x = _act(x, "convT2x2_bwd")
    dy = _act(dy, "convT2x2_bwd").to(x.dtype)
    d = K.dcode(x.dtype)
    N, ci, h, wd = x.shape
    co = w.shape[1]
    g = K.gather_convT(dy, N, h, wd)
    dx = K.empty_act(N, ci, h, wd, x.dtype, x.device)
    K.gemm_fwd(g, wT_dgrad(w, d), ci, dx, d)
    dw = torch.empty((ci, co, 2, 2), dtype=torch.float32, device=x.device)
    K.gemm_wgrad(K.gather1x1([x]), K.gather_convT(dy, N, h, wd), ci, 4 * co, dw, convT_layout(dw), d, False)
    db = torch.empty(co, dtype=torch.float32, device=x.device)
    K.chan_sum(dy, db, False, d)
    return dx, dw, db


@convT2x2_bwd.register_fake
def _(x, dy, w):
    f32 = dict(dtype=torch.float32, device=x.device)
    return _cl_empty(*x.shape, x), torch.empty(tuple(w.shape), **f32), torch.empty(w.shape[1], **f32)


def _convT_setup(ctx, inputs, output):
    x, w, bias = inputs
    ctx.save_for_backward(x, w)
    ctx.has_bias = bias is not None


def _convT_backward(ctx, gy):
    x, w = ctx.saved_tensors
    dx, dw, db = convT2x2_bwd(x, gy.to(x.dtype), w)
    return (dx if ctx.needs_input_grad[0] else None, dw.to(w.dtype) if ctx.needs_input_grad[1] else None,
            db if ctx.has_bias and ctx.needs_input_grad[2] else None)


convT2x2_fwd.register_autograd(_convT_backward, setup_context=_convT_setup)


# ---- bilinear resize, align_corners=True -----------------------------------------------
@torch.library.custom_op(f"{_NS}::upsample_bilinear_ac_fwd", mutates_args=(), device_types="cuda")
def upsample_bilinear_ac_fwd(x: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """F.interpolate(x, size=(H, W), mode='bilinear', align_corners=True):
    src = dst * (in - 1) / (out - 1), one coalesced NHWC gather pass."""
    x = _act(x, "upsample_bilinear_ac_fwd")
    y = K.empty_act(x.shape[0], x.shape[1], H, W, x.dtype, x.device)
    return K.upsample_fwd(x, y, H, W, 0, 0, K.dcode(x.dtype))


@upsample_bilinear_ac_fwd.register_fake
def _(x, H, W):
    return _cl_empty(x.shape[0], x.shape[1], H, W, x)


@torch.library.custom_op(f"{_NS}::upsample_bilinear_ac_bwd", mutates_args=(), device_types="cuda")
def upsample_bilinear_ac_bwd(dy: torch.Tensor, h: int, w: int) -> torch.Tensor:
    """Input gradient of upsample_bilinear_ac_fwd to size (h, w): the
    transposed gather (no atomics: deterministic)."""
    dy = _act(dy, "upsample_bilinear_ac_bwd")
    dx = K.empty_act(dy.shape[0], dy.shape[1], h, w, dy.dtype, dy.device)
    return K.upsample_bwd(dy, dx, dy.shape[2], dy.shape[3], 0, 0, False, K.dcode(dy.dtype))


@upsample_bilinear_ac_bwd.register_fake
def _(dy, h, w):
    return _cl_empty(dy.shape[0], dy.shape[1], h, w, dy)


def _up_setup(ctx, inputs, output):
    ctx.hw = (inputs[0].shape[2], inputs[0].shape[3])
    ctx.dtype = inputs[0].dtype


def _up_backward(ctx, gy):
    return upsample_bilinear_ac_bwd(gy.to(ctx.dtype), *ctx.hw), None, None


upsample_bilinear_ac_fwd.register_autograd(_up_backward, setup_context=_up_setup)


# ---- AttentionGate ------------------------------------------------------------------
def _param(t):
    """a fresh leaf standing in for an nn.Parameter inside a functional op (the
    engine writes parameter gradients into .grad)"""
    return t.detach().float().contiguous().requires_grad_(True)


def _bn_shim(gamma, beta, rm, rv, momentum, eps):
    return types.SimpleNamespace(weight=_param(gamma), bias=_param(beta), running_mean=rm, running_var=rv,
                                 num_batches_tracked=None, momentum=momentum, eps=eps, training=True,
                                 track_running_stats=rm is not None)


def _conv_shim(w, b):
    return types.SimpleNamespace(weight=_param(w), bias=_param(b), out_channels=w.shape[0])


def _gate_shim(params, running, momentum, eps):
    wg, bg, gg, betag, wx, bx, gx, betax, wp, bp, gp, betap = params
    rm = [r.float().clone() for r in running]
    att = types.SimpleNamespace(
        W_g=(_conv_shim(wg, bg), _bn_shim(gg, betag, rm[0], rm[1], momentum, eps)),
        W_x=(_conv_shim(wx, bx), _bn_shim(gx, betax, rm[2], rm[3], momentum, eps)),
        psi=(_conv_shim(wp, bp), _bn_shim(gp, betap, rm[4], rm[5], momentum, eps)))
    att.psi = _PsiShim(att.psi)
    return att, rm


class _PsiShim(tuple):
    """AttentionGate.psi stand-in: indexable, no forward hooks"""
    _forward_hooks = {}


_GATE_DOC = """g, x: gate / skip activations [N, F_g|F_l, H, W] (NHWC); params: W_g conv
(weight [F_int, F_g, 1, 1], bias), its BN (gamma, beta), W_x conv + BN, psi
conv ([1, F_int, 1, 1], bias) + BN(1); running: the six running-statistic
tensors (W_g mean, var, W_x mean, var, psi mean, var)."""


@torch.library.custom_op(f"{_NS}::attn_gate_fwd", mutates_args=(), device_types="cuda")
def attn_gate_fwd(g: torch.Tensor, x: torch.Tensor, params: list[torch.Tensor], running: list[torch.Tensor],
                  momentum: float, eps: float) -> tuple[torch.Tensor, torch.Tensor, list[torch.Tensor]]:
    """AttentionGate forward, train-mode BatchNorms: out = x * sigmoid(BN(psi(
    relu(BN(W_g g) + BN(W_x x))))).  Returns (out, psi map [N, 1, H, W] fp32,
    the six updated running statistics)."""
    g = _act(g, "attn_gate_fwd")
    x = _act(x, "attn_gate_fwd")
    M = E.Mode(K.dcode(x.dtype), x.device)
    att, rm = _gate_shim(params, running, momentum, eps)
    out, saved = E.attention_fwd(M, att, g, x)
    return out, saved[-1].clone(), rm


@attn_gate_fwd.register_fake
def _(g, x, params, running, momentum, eps):
    N, _, H, W = x.shape
    return (_cl_empty(*x.shape, x), torch.empty((N, 1, H, W), dtype=torch.float32, device=x.device),
            [torch.empty_like(r, dtype=torch.float32) for r in running])


@torch.library.custom_op(f"{_NS}::attn_gate_bwd", mutates_args=(), device_types="cuda")
def attn_gate_bwd(g: torch.Tensor, x: torch.Tensor, dout: torch.Tensor, params: list[torch.Tensor],
                  running: list[torch.Tensor], momentum: float,
                  eps: float) -> tuple[torch.Tensor, torch.Tensor, list[torch.Tensor]]:
    """(dg, dx, [d params in attn_gate_fwd's order]) of attn_gate_fwd at the
    same inputs (the forward is re-run to rebuild its saved tensors: batch
    statistics are a function of the inputs)."""
    g = _act(g, "attn_gate_bwd")
    x = _act(x, "attn_gate_bwd")
    dout = _act(dout, "attn_gate_bwd").to(x.dtype)
    M = E.Mode(K.dcode(x.dtype), x.device)
    att, _ = _gate_shim(params, running, momentum, eps)
    _, saved = E.attention_fwd(M, att, g, x)
    dg = K.zeros_act(*g.shape, g.dtype, g.device)
    dx = E.attention_bwd(M, att, saved, dout, (dg, 0), True)
    leaves = [att.W_g[0].weight, att.W_g[0].bias, att.W_g[1].weight, att.W_g[1].bias,
              att.W_x[0].weight, att.W_x[0].bias, att.W_x[1].weight, att.W_x[1].bias,
              att.psi[0].weight, att.psi[0].bias, att.psi[1].weight, att.psi[1].bias]
    grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in leaves]
    return dg, dx, [gr.view(pr.shape) for gr, pr in zip(grads, params)]


@attn_gate_bwd.register_fake
def _(g, x, dout, params, running, momentum, eps):
    return _cl_empty(*g.shape, g), _cl_empty(*x.shape, x), [torch.empty_like(p, dtype=torch.float32) for p in params]


def _gate_setup(ctx, inputs, output):
    g, x, params, running, momentum, eps = inputs
    ctx.save_for_backward(g, x, *params, *running)
    ctx.np = len(params)
    ctx.cfg = (momentum, eps)


def _gate_backward(ctx, gout, _gpsi, _grun):
    t = ctx.saved_tensors
    g, x, params, running = t[0], t[1], list(t[2:2 + ctx.np]), list(t[2 + ctx.np:])
    dg, dx, dps = attn_gate_bwd(g, x, gout, params, running, *ctx.cfg)
    return dg, dx, dps, [None] * len(running), None, None


attn_gate_fwd.register_autograd(_gate_backward, setup_context=_gate_setup)
attn_gate_fwd.__doc__ += _GATE_DOC


# ---- VAE bottleneck: heads + reparameterize ----------------------------------------
@torch.library.custom_op(f"{_NS}::vae_bottleneck_fwd", mutates_args=(), device_types="cuda")
def vae_bottleneck_fwd(f4: torch.Tensor, w_mu: torch.Tensor, b_mu: torch.Tensor, w_lv: torch.Tensor,
                       b_lv: torch.Tensor, eps: torch.Tensor | None) -> tuple[torch.Tensor, torch.Tensor,
                                                                              torch.Tensor, torch.Tensor]:
    """mu_head / logvar_head (1x1 conv + AdaptiveAvgPool2d) and reparameterize
    in ONE launch (one block per sample; vu_vae_heads_fwd): returns (mu,
    logvar, z = mu + eps * exp(logvar / 2) (z = mu when eps is None), the
    pooled features [N, C] the backward reads)."""
    f4 = _act(f4, "vae_bottleneck_fwd")
    N, C4, H, W = f4.shape
    L = w_mu.shape[0]
    dev = f4.device
    pooled = torch.empty((N, C4), dtype=torch.float32, device=dev)
    mu = torch.empty((N, L), dtype=torch.float32, device=dev)
    lv, z = torch.empty_like(mu), torch.empty_like(mu)
    wm, wl = w_mu.float().reshape(L, C4).contiguous(), w_lv.float().reshape(L, C4).contiguous()
    e = None if eps is None else eps.float().contiguous()
    call("vu_vae_heads_fwd", ptr(f4), K.pstride(f4), N, H * W, C4, ptr(wm), ptr(b_mu.float().contiguous()), ptr(wl),
         ptr(b_lv.float().contiguous()), L, ptr(e), ptr(pooled), ptr(mu), ptr(lv), ptr(z), K.dcode(f4.dtype),
         stream())
    return mu, lv, z, pooled


@vae_bottleneck_fwd.register_fake
def _(f4, w_mu, b_mu, w_lv, b_lv, eps):
    N, L = f4.shape[0], w_mu.shape[0]
    f32 = dict(dtype=torch.float32, device=f4.device)
    return (torch.empty((N, L), **f32), torch.empty((N, L), **f32), torch.empty((N, L), **f32),
            torch.empty((N, f4.shape[1]), **f32))


@torch.library.custom_op(f"{_NS}::vae_bottleneck_bwd", mutates_args=(), device_types="cuda")
def vae_bottleneck_bwd(f4: torch.Tensor, pooled: torch.Tensor, w_mu: torch.Tensor, w_lv: torch.Tensor,
                       logvar: torch.Tensor, eps: torch.Tensor | None, dmu: torch.Tensor | None,
                       dlogvar: torch.Tensor | None, dz: torch.Tensor | None) -> list[torch.Tensor]:
    """[d f4, d w_mu, d b_mu, d w_lv, d b_lv] of vae_bottleneck_fwd: the
    reparameterize backward, both heads' backward in one block
    (vu_latent_bwd with no consumers) and the broadcast of d pooled / HW."""
    f4 = _act(f4, "vae_bottleneck_bwd")
    N, C4, H, W = f4.shape
    L = w_mu.shape[0]
    dev = f4.device
    z = torch.zeros((N, L), dtype=torch.float32, device=dev)
    f32 = dict(dtype=torch.float32, device=dev)
    dwm, dbm = torch.empty((L, C4), **f32), torch.empty(L, **f32)
    dwl, dbl = torch.empty((L, C4), **f32), torch.empty(L, **f32)
    dpooled = torch.empty((N, C4), **f32)
    wm, wl = w_mu.float().reshape(L, C4).contiguous(), w_lv.float().reshape(L, C4).contiguous()
    keep = [t.float().contiguous() if t is not None else None for t in (eps, logvar, dmu, dlogvar, dz)]
    e, lv, gm, gl, gz = keep
    h = _lib.VuLatentHeads()
    h.z, h.eps, h.logvar = z.data_ptr(), ptr(e), lv.data_ptr()
    h.dmu_in, h.dlv_in, h.dz_in = ptr(gm), ptr(gl), ptr(gz)
    h.pooled, h.w_mu, h.w_lv = pooled.float().contiguous().data_ptr(), wm.data_ptr(), wl.data_ptr()
    h.dw_mu, h.db_mu, h.dw_lv, h.db_lv = dwm.data_ptr(), dbm.data_ptr(), dwl.data_ptr(), dbl.data_ptr()
    h.dpooled, h.C, h.grad_acc = dpooled.data_ptr(), C4, 0
    ws = K.workspace_f32(query("vu_latent_bwd_workspace_bytes", N, L, 0), dev)
    call("vu_latent_bwd", None, 0, C.byref(h), N, L, ptr(ws), stream())
    df4 = K.empty_act(N, C4, H, W, f4.dtype, dev)
    call("vu_sample_broadcast", ptr(dpooled), N, H * W, C4, 1.0 / (H * W), ptr(df4), K.pstride(df4), 0,
         K.dcode(f4.dtype), stream())
    return [df4, dwm.view(w_mu.shape), dbm, dwl.view(w_lv.shape), dbl]


@vae_bottleneck_bwd.register_fake
def _(f4, pooled, w_mu, w_lv, logvar, eps, dmu, dlogvar, dz):
    f32 = dict(dtype=torch.float32, device=f4.device)
    L = w_mu.shape[0]
    return [_cl_empty(*f4.shape, f4), torch.empty(tuple(w_mu.shape), **f32), torch.empty(L, **f32),
            torch.empty(tuple(w_lv.shape), **f32), torch.empty(L, **f32)]


def _vb_setup(ctx, inputs, output):
    f4, w_mu, b_mu, w_lv, b_lv, eps = inputs
    mu, lv, z, pooled = output
    ctx.save_for_backward(f4, pooled, w_mu, w_lv, lv, eps)


def _vb_backward(ctx, gmu, glv, gz, _gpooled):
    f4, pooled, w_mu, w_lv, lv, eps = ctx.saved_tensors
    df4, dwm, dbm, dwl, dbl = vae_bottleneck_bwd(f4, pooled, w_mu, w_lv, lv, eps, gmu, glv, gz)
    return df4.to(f4.dtype), dwm, dbm, dwl, dbl, None


vae_bottleneck_fwd.register_autograd(_vb_backward, setup_context=_vb_setup)


OPS = ("conv3x3_fwd", "conv3x3_dgrad", "conv3x3_wgrad", "conv_bn_relu", "bn_relu_backward", "bn_finalize",
       "maxpool2d", "maxpool2d_backward", "convT2x2_fwd", "convT2x2_bwd", "upsample_bilinear_ac_fwd",
       "upsample_bilinear_ac_bwd", "attn_gate_fwd", "attn_gate_bwd", "vae_bottleneck_fwd", "vae_bottleneck_bwd",
       "bce_dice_loss")
