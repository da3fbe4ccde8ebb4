"""fp8 (OCP e4m3fn) 3x3 convolution forward path -- BASELINE.json configs[4]
("fp8 NHWC implicit-GEMM 3x3 conv path on CDNA4 fp8 MFMA, 3x1024x1024").

The reference has no fp8 path.  This is the
DoubleConv convolution (unet_parts.py:40,43) with

* activations quantised to e4m3 with ONE scale per tensor (448 / amax; the
  concat sources of an Up block share it),
* weights quantised to e4m3 with one scale per output channel,
* fp32 accumulation on the gfx950 f8f6f4 MFMA (csrc/conv_fp8.hip), the two
  dequantisation scales and the bias applied in the epilogue, bf16 output
  and the BatchNorm partial statistics of that output.

Parity: the kernel equals fp32 convolution of the DEQUANTISED operands up to
fp32 summation order and the bf16 output rounding, and the quantisers are
bit-exact against ``torch.float8_e4m3fn`` (tests/test_gpu_fp8.py); the error
against the unquantised fp32 convolution is reported by tools/fp8_bench.py.
There is no fallback: shapes the kernel does not serve raise.
"""
import ctypes as C

import torch

from . import _lib
from . import engine as E
from . import kernels as K
from ._lib import VuConvFp8, call, query, stream

E4M3 = torch.float8_e4m3fn


def amax(srcs):
    """max |x| over all sources (device fp32 [1])."""
    out = torch.empty(1, dtype=torch.float32, device=srcs[0].device)
    for i, t in enumerate(srcs):
        N, Cc, H, W = t.shape
        call("vu_amax", C.c_void_p(t.data_ptr()), K.pstride(t), N * H * W, Cc, C.c_void_p(out.data_ptr()),
             1 if i else 0, K.dcode(t.dtype), stream())
    return out


def quantize(x, am):
    """x (bf16/fp32 NHWC) -> (e4m3 NHWC, dequant scale [1]) with s = 448/amax."""
    N, Cc, H, W = x.shape
    q = torch.empty((N, Cc, H, W), dtype=E4M3, device=x.device, memory_format=K.CL)
    dq = torch.empty(1, dtype=torch.float32, device=x.device)
    call("vu_quant_fp8", C.c_void_p(x.data_ptr()), K.pstride(x), N * H * W, Cc, C.c_void_p(am.data_ptr()),
         C.c_void_p(q.data_ptr()), K.pstride(q), C.c_void_p(dq.data_ptr()), K.dcode(x.dtype), stream())
    return q, dq


class DelayedScale:
    """Delayed (previous-step) per-tensor scaling of one fp8 activation site.

    ``ring`` holds three fp32 amax slots on the device: step t quantises with
    s = 448 / ring[t % 3] (the amax step t-1 recorded), max-accumulates its
    own max |x| into ring[(t+1) % 3] and clears ring[(t+2) % 3] -- all inside
    the quantising kernel (vu_bn_apply_fp8), so the step adds no launch and
    no host sync.  The first step has no history: a calibration pass of the
    same kernel measures max |x| into ring[0] first.  Values above the stale
    amax saturate at +-448 (standard delayed-scaling behaviour)."""

    def __init__(self, device):
        self.ring = torch.zeros(3, dtype=torch.float32, device=device)
        self.t = 0

    @property
    def slot(self):
        return self.t % 3

    def advance(self):
        self.t += 1


def _q8_args(x, coef, relu, ds):
    N, Cc, H, W = x.shape
    sc = C.c_void_p(coef[0].data_ptr()) if coef is not None else None
    sh = C.c_void_p(coef[1].data_ptr()) if coef is not None else None
    return (N * H * W, Cc, sc, sh, 1 if relu else 0, C.c_void_p(ds.ring.data_ptr()), ds.slot)


def calibrate(x, coef, relu, ds):
    """First step of a site (no history): max-accumulate max |z| of this
    source into the scale slot bn_apply_quant is about to read."""
    call("vu_bn_apply_fp8", C.c_void_p(x.data_ptr()), K.pstride(x), None, 0, *_q8_args(x, coef, relu, ds), 1,
         None, K.dcode(x.dtype), stream())


def bn_apply_quant(x, coef, relu, ds):
    """e4m3 NHWC relu?(x * coef[0] + coef[1]) (coef None: relu?(x)) with the
    delayed scale ``ds``; returns (q, dequant scale [1]).  One pass over x;
    the caller advances ``ds`` once per step (after every source of a site)."""
    N, Cc, H, W = x.shape
    q = torch.empty((N, Cc, H, W), dtype=E4M3, device=x.device, memory_format=K.CL)
    dq = torch.empty(1, dtype=torch.float32, device=x.device)
    call("vu_bn_apply_fp8", C.c_void_p(x.data_ptr()), K.pstride(x), C.c_void_p(q.data_ptr()), K.pstride(q),
         *_q8_args(x, coef, relu, ds), 0, C.c_void_p(dq.data_ptr()), K.dcode(x.dtype), stream())
    return q, dq


def quantize_rows(m):
    """fp32 [rows][cols] -> (e4m3 [rows][cols], per-row dequant scale [rows])."""
    rows, cols = m.shape
    q = torch.empty((rows, cols), dtype=E4M3, device=m.device)
    dq = torch.empty(rows, dtype=torch.float32, device=m.device)
    call("vu_quant_rows_fp8", C.c_void_p(m.data_ptr()), rows, cols, C.c_void_p(q.data_ptr()), cols,
         C.c_void_p(dq.data_ptr()), stream())
    return q, dq


def quantize_weight(w):
    """Conv weight [Cout, Cin, 3, 3] -> (e4m3 [Cout][9*Cin] with k = tap*Cin + c,
    dequant scale per output channel), cached per parameter version."""
    ver = (w._version, w.data_ptr())
    ent = w.__dict__.get("_vu_fp8")
    if ent is None or ent[0] != ver:
        wf = E.w3x3_fwd(w, _lib.F32)       # fp32 [Cout][9*Cin], the bf16 kernels' k order
        ent = (ver, quantize_rows(wf.contiguous()))
        w.__dict__["_vu_fp8"] = ent
    return ent[1]


def conv3x3(xqs, x_dq, wq, w_dq, ncol, out=None, out_coff=0, bias=None, stats=False, minmax=False):
    """out[m][co] = x_dq * w_dq[co] * sum_k xq[m][k] wq[co][k] (+bias), bf16 NHWC.
    xqs: 1-3 e4m3 NHWC sources (channel concat, 64-channel aligned).
    minmax: also the per-tile per-channel min / max of the output where the
    serving kernel emits them (vu_conv3x3_fp8_minmax_ok), returned as
    ``(pmin, pmax)`` in ``Stats.minmax`` (``Stats.minmax`` None where it does
    not; a Stats is then returned even without ``stats``)."""
    N, _, H, W = xqs[0].shape
    if out is None:
        out = K.empty_act(N, ncol, H, W, torch.bfloat16, xqs[0].device)
    a = VuConvFp8()
    a.a = K.gather3x3(xqs)
    a.w = wq.data_ptr()
    a.ldw = wq.shape[1]
    a.ncol = ncol
    a.out_coff = out_coff
    a.x_scale = x_dq.data_ptr()
    a.w_scale = w_dq.data_ptr()
    a.bias = bias.data_ptr() if bias is not None else None
    a.out = out.data_ptr()
    a.out_stride = K.pstride(out)
    a.stat_sum = a.stat_m2 = a.stat_min = a.stat_max = None
    rows = N * H * W
    bm = query("vu_conv3x3_fp8_row_tile", C.byref(a))
    if bm <= 0:
        raise ValueError(f"fp8 3x3 conv: shape not served (C={a.a.C}, ncol={ncol}, H={H}, W={W})")
    st = None
    tiles = (rows + bm - 1) // bm
    if stats:
        psum = torch.empty((tiles, ncol), dtype=torch.float32, device=out.device)
        pm2 = torch.empty_like(psum)
        a.stat_sum, a.stat_m2 = psum.data_ptr(), pm2.data_ptr()
        st = K.Stats(psum, pm2, tiles, bm, rows)
    if minmax:
        if st is None:
            st = K.Stats(None, None, tiles, bm, rows)
        st.minmax = None
        if query("vu_conv3x3_fp8_minmax_ok", C.byref(a)):
            pmin = torch.empty((tiles, ncol), dtype=torch.float32, device=out.device)
            pmax = torch.empty_like(pmin)
            a.stat_min, a.stat_max = pmin.data_ptr(), pmax.data_ptr()
            st.minmax = (pmin, pmax)
    a.workspace = None
    nb = query("vu_conv3x3_fp8_workspace_bytes", C.byref(a))
    ws = None
    if nb > 0:
        ws = torch.empty(nb // 4, dtype=torch.float32, device=out.device)
        a.workspace = ws.data_ptr()
    K._timed("conv3x3_fp8_fwd", 2 * rows * ncol * 9 * a.a.C,
             lambda: call("vu_conv3x3_fp8", C.byref(a), stream()))
    return out, st


def conv3x3_q(srcs, weight, bias=None, stats=False, minmax=False):
    """Quantise the (bf16) sources with one shared scale and the weights, then
    run the fp8 conv.  Returns (bf16 output, Stats or None)."""
    am = amax(srcs)
    qs, dq = [], None
    for t in srcs:
        q, dq = quantize(t, am)
        qs.append(q)
    wq, ws = quantize_weight(weight)
    return conv3x3(qs, dq, wq, ws, weight.shape[0], bias=bias, stats=stats, minmax=minmax)


def relu_amax_scale(minmax, coef, relu, device):
    """A fresh single-use DelayedScale whose slot 0 holds the just-in-time
    amax of relu?(y * coef[0] + coef[1]) (vu_fp8_relu_amax, from the producing
    conv's per-tile min / max: no pass over y)."""
    pmin, pmax = minmax
    ds = DelayedScale(device)
    call("vu_fp8_relu_amax", C.c_void_p(pmin.data_ptr()), C.c_void_p(pmax.data_ptr()), pmin.shape[0],
         pmin.shape[1], C.c_void_p(coef[0].data_ptr()) if coef is not None else None,
         C.c_void_p(coef[1].data_ptr()) if coef is not None else None, 1 if relu else 0,
         C.c_void_p(ds.ring.data_ptr()), stream())
    return ds


# just-in-time fp8 DoubleConv: conv2's input scale from conv1's min / max
# epilogue and BN1 + ReLU applied with the e4m3 quantise in one pass (round 6),
# instead of BN1 apply (bf16) + an amax pass + a quantise pass (A/B switch)
JIT_MINMAX = True


def _site_scales(mod, device):
    """The module's three DelayedScale sites (input, mid, output).  They are
    not module state (not in state_dict, not moved by .to()): a module used
    on another device starts a fresh history (calibration step) there."""
    ent = mod.__dict__.get("_vu_fp8_scales")
    if ent is None or ent[0].ring.device != torch.device(device):
        ent = (DelayedScale(device), DelayedScale(device), DelayedScale(device))
        mod.__dict__["_vu_fp8_scales"] = ent
    return ent


def reset_scales(mod):
    """Forget the delayed-scaling history of ``mod`` (e.g. between train and
    eval, or before inputs with a different range): the next delayed call
    calibrates again."""
    mod.__dict__.pop("_vu_fp8_scales", None)


@torch.no_grad()
def double_conv_forward(mod, x, delayed=False, x_q=None, out_fp8=False):
    """DoubleConv.forward (unet_parts.py:32-49) with both 3x3 convs in fp8:
    conv -> BatchNorm (batch statistics from the fp8 conv epilogue in train
    mode, running statistics in eval mode) -> ReLU, twice; bf16 NHWC out.
    x: a bf16 NHWC tensor, or the list of channel-concat sources of an Up
    block's DoubleConv (they share one scale, as in conv3x3_q).

    delayed=False (default): just-in-time scaling, every call self-contained:
    an amax pass + a quantise pass of the input; conv2's input scale is the
    exact max of relu(BN1(y1)) formed from conv1's per-tile per-channel
    min / max (its epilogue, vu_fp8_relu_amax), and BN1 + ReLU is applied and
    quantised in one pass (vu_bn_apply_fp8) -- round 6; before, BN1 was
    applied to a bf16 tensor that was then read twice more (amax, quantise).
    delayed=True (opt-in, for step loops over same-range data): both
    activation quantisations use the amax the previous call recorded
    (DelayedScale, one per site, kept on the module; ``reset_scales`` drops
    it): the input is quantised in one pass (no amax pass) and BN1 + ReLU is
    applied and quantised in the same pass (vu_bn_apply_fp8), so conv2's
    input is never stored in bf16.  Values above the previous call's amax
    saturate at +-448.  The host-side slot counter advances per call: a
    captured graph would freeze it, so delayed calls are not graph-safe.

    Chained fp8 blocks: ``x_q = (e4m3 sources, dequant scale)`` is an input
    already quantised by the producing block, and ``out_fp8=True`` applies
    BN2 + ReLU fused with the e4m3 quantisation of the block's output and
    returns ``(q, dq)`` -- the activations between fp8 blocks are then never
    stored in bf16.  Delayed: the output's own delayed scale.  Just in time
    (round 6): the exact amax of relu(BN2(y2)) from conv2's min / max
    epilogue, as conv2's input scale is formed from conv1's (a calibration
    pass over y2 where the serving kernel emits no min / max)."""
    conv1, bn1, _, conv2, bn2, _ = mod.double_conv
    srcs = list(x) if isinstance(x, (list, tuple)) else ([x] if x is not None else [])
    if (x_q is not None or out_fp8) and not delayed and not JIT_MINMAX:
        raise ValueError("fp8.double_conv_forward: x_q / out_fp8 (chained fp8 blocks) need delayed=True "
                         "or the min/max just-in-time path (JIT_MINMAX)")
    if not delayed:
        if JIT_MINMAX:
            if x_q is not None:
                qs, xdq = list(x_q[0]), x_q[1]
            else:
                # the input: exact amax by the calibration pass (max-accumulated
                # over the sources), one quantising pass per source with that scale
                ds_x = DelayedScale(srcs[0].device)
                for t in srcs:
                    calibrate(t, None, False, ds_x)
                qs = []
                for t in srcs:
                    q, xdq = bn_apply_quant(t, None, False, ds_x)
                    qs.append(q)
            w1, s1 = quantize_weight(conv1.weight)
            y1, st1 = conv3x3(qs, xdq, w1, s1, conv1.out_channels, stats=bn1.training, minmax=True)
        else:
            y1, st1 = conv3x3_q(srcs, conv1.weight, stats=bn1.training)
        coef1 = E.bn_coef(bn1, st1 if bn1.training else None, conv1.out_channels)
        w2, s2 = quantize_weight(conv2.weight)
        if JIT_MINMAX and st1 is not None and st1.minmax is not None:
            # exact just-in-time scale of relu(BN1(y1)) from the min / max
            # partials, then BN1 + ReLU + e4m3 in one pass (no bf16 a1)
            ds = relu_amax_scale(st1.minmax, coef1, True, y1.device)
            aq, adq = bn_apply_quant(y1, coef1, True, ds)
            y2, st2 = conv3x3([aq], adq, w2, s2, conv2.out_channels, stats=bn2.training, minmax=out_fp8)
        else:
            a1 = torch.empty_like(y1)
            K.bn_apply(y1, a1, coef1, True, _lib.BF16)
            y2, st2 = conv3x3_q([a1], conv2.weight, stats=bn2.training, minmax=out_fp8)
        coef2 = E.bn_coef(bn2, st2 if bn2.training else None, conv2.out_channels)
        if out_fp8:
            if st2 is not None and st2.minmax is not None:
                ds = relu_amax_scale(st2.minmax, coef2, True, y2.device)
            else:
                ds = DelayedScale(y2.device)
                calibrate(y2, coef2, True, ds)
            return bn_apply_quant(y2, coef2, True, ds)
        out = torch.empty_like(y2)
        K.bn_apply(y2, out, coef2, True, _lib.BF16)
        return out
    if x_q is not None:
        qs, xdq = list(x_q[0]), x_q[1]
        dev = qs[0].device
    else:
        dev = srcs[0].device
    ds_in, ds_mid, ds_out = _site_scales(mod, dev)
    if x_q is None:
        if ds_in.t == 0:
            for t in srcs:           # every source first: they share the scale
                calibrate(t, None, False, ds_in)
        qs = []
        for t in srcs:
            q, xdq = bn_apply_quant(t, None, False, ds_in)
            qs.append(q)
    w1, s1 = quantize_weight(conv1.weight)
    y1, st1 = conv3x3(qs, xdq, w1, s1, conv1.out_channels, stats=bn1.training)
    coef1 = E.bn_coef(bn1, st1, conv1.out_channels)
    if ds_mid.t == 0:
        calibrate(y1, coef1, True, ds_mid)
    aq, adq = bn_apply_quant(y1, coef1, True, ds_mid)
    w2, s2 = quantize_weight(conv2.weight)
    y2, st2 = conv3x3([aq], adq, w2, s2, conv2.out_channels, stats=bn2.training)
    coef2 = E.bn_coef(bn2, st2, conv2.out_channels)
    if out_fp8:
        if ds_out.t == 0:
            calibrate(y2, coef2, True, ds_out)
        out = bn_apply_quant(y2, coef2, True, ds_out)
    else:
        out = torch.empty_like(y2)
        K.bn_apply(y2, out, coef2, True, _lib.BF16)
    # a site's step counter counts its own quantisations
    for ds, used in ((ds_in, x_q is None), (ds_mid, True), (ds_out, out_fp8)):
        if used:
            ds.advance()
    return out
