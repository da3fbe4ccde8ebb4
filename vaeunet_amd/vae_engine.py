"""Fused sequences for the VAE-U-Net (unet/unet_resnet.py:31-279).

* ResNet34 encoder (timm ``resnet34`` features_only, unet_resnet.py:131-137):
  7x7/s2 stem + BN + ReLU, 3x3/s2 max-pool, BasicBlocks [3, 4, 6, 3].  All
  convolutions run on the implicit-GEMM kernels; stride-2 convolutions get
  their input gradient as four parity-class GEMMs (out_mode 2), so no
  zero-inserted tensor is ever built.
* VAE bottleneck: the conv1x1 + AdaptiveAvgPool2d heads (unet_resnet.py:
  140-147) are computed as a per-sample channel mean followed by a [L x C]
  map (pool and 1x1 conv commute), reparameterisation (191-194), and the
  latent broadcast ``interpolate(z[..., None, None], size, align_corners=True)``
  which is an exact per-sample broadcast (217-221, 93).
* DecoderBlock (31-101): bilinear(align_corners) to the skip size, attention
  gate, z_proj, three-source channel concat fed straight into conv1's K loop.
"""
import ctypes as C

import torch

from . import _lib
from . import engine as E
from . import kernels as K
from ._lib import F32


# ---------------------------------------------------------------------------
# generic convolution (square kernel k, stride s, padding p, no dilation)
# ---------------------------------------------------------------------------
def _geom(conv):
    return conv.kernel_size[0], conv.stride[0], conv.padding[0]


def conv_gather(srcs, conv):
    N, _, H, W = srcs[0].shape
    k, s, p = _geom(conv)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    return K.gather(srcs, N, Ho, Wo, R=k, S=k, sy=s, sx=s, oy=-p, ox=-p), Ho, Wo


def conv_fwd(M, srcs, conv, stats, cin_pad=None):
    g, Ho, Wo = conv_gather(srcs, conv)
    co = conv.out_channels
    y = M.act(srcs[0].shape[0], co, Ho, Wo)
    st = K.gemm_fwd(g, E.w3x3_fwd(conv.weight, M.d, cin_pad), co, y, M.d,
                    bias=conv.bias, stats=stats)
    return y, st


def conv_wgrad(M, dy, srcs, conv, cvalid=None, bn=None):
    """Weight (and bias) gradient, forked onto the side stream (engine.OVERLAP_WGRAD);
    bn: the BatchNorm the conv feeds (a train-mode one zeroes the bias gradient)."""
    def wg():
        gw, acc = E.grad_sink(conv.weight)
        if gw is not None:
            g, _, _ = conv_gather(srcs, conv)
            K.gemm_wgrad(K.gather1x1([dy]), g, dy.shape[1], g.R * g.S * g.C, gw, E.conv_layout(gw), M.d,
                         acc, cvalid=cvalid)
        if conv.bias is not None:
            E.bias_grad(dy, conv.bias, M, bn=bn)
    M.side(wg, dy, *srcs)


def _parity_w(w, py, px, p, d):
    """Input-gradient weights of one parity class of a stride-2 conv:
    B[ci][(ry*Sx + rx)*Cout + co] over the taps r = py+p (mod 2), descending."""
    co, ci, k, _ = w.shape
    ry = [r for r in range(k) if (r - py - p) % 2 == 0]
    rx = [r for r in range(k) if (r - px - p) % 2 == 0]
    if not ry or not rx:
        return None, ry, rx

    def build():
        s = w.stride()
        base = max(ry) * s[2] + max(rx) * s[3]
        return K.permute4(w.detach(), base, (s[1], -2 * s[2], -2 * s[3], s[0]),
                          (ci, len(ry), len(rx), co), co, d).view(ci, -1)
    return E._cached(w, ("wpar", d, py, px), build), ry, rx


def conv_dgrad(M, dy, conv, dx, accumulate, bnb=None):
    """dx (N, Cin, H, W) (+)= conv input gradient of dy.  bnb=(x, coef, relu):
    also the BN-backward partials of dx for the BN over x (stride 1; returns
    (dx, part), part None when the kernel cannot)."""
    k, s, p = _geom(conv)
    N, ci, H, W = dx.shape
    if s == 1:
        if 2 * p != k - 1:
            raise NotImplementedError("stride-1 conv input gradient needs 'same' padding")
        g = K.gather([dy], N, H, W, R=k, S=k, oy=p - (k - 1), ox=p - (k - 1))
        part = K.gemm_fwd(g, E.w3x3_dgrad(conv.weight, M.d), ci, dx, M.d, accumulate=accumulate,
                          kind="dgrad", bnb=bnb if E.FUSE_BN_BWD_REDUCE else None)
        return (dx, part) if bnb is not None else dx
    if bnb is not None:
        raise NotImplementedError("BN-backward partials from a strided input gradient")
    if s != 2:
        raise NotImplementedError("only stride 1 and 2 convolutions")
    Ho, Wo = dy.shape[2], dy.shape[3]
    if E.S2_ZERO_INSERT_DGRAD and M.d != F32 and k == 3 and p == 1 and dy.shape[1] % 64 == 0 \
            and ci % 64 == 0 and H <= 2 * Ho and W <= 2 * Wo:
        # dx[y] = sum_ky dy[(y + 1 - ky) / 2] w[ky] over the even (y + 1 - ky):
        # the stride-1 input gradient of the zero-inserted dy (one halo-kernel
        # conv with 4x the MACs, instead of four small parity-class GEMMs)
        up = M.act(N, dy.shape[1], H, W)
        # roofline accounting (bench.py): the zero fill's time and only the
        # algorithmic MACs of the stride-2 gradient (a quarter of the launch's)
        K._timed("conv3x3_dgrad", 0,
                 lambda: K.call("vu_zero_insert2", K.ptr(dy), K.pstride(dy), N, Ho, Wo, dy.shape[1], K.ptr(up),
                                K.pstride(up), H, W, M.d, K.stream()))
        g = K.gather([up], N, H, W, R=3, S=3, oy=-1, ox=-1)
        K.gemm_fwd(g, E.w3x3_dgrad(conv.weight, M.d), ci, dx, M.d, accumulate=accumulate, kind="dgrad",
                   flops=2 * N * Ho * Wo * dy.shape[1] * 9 * ci)
        return dx
    classes = []
    for py in (0, 1):
        for px in (0, 1):
            wmat, ry, rx = _parity_w(conv.weight, py, px, p, M.d)
            hp, wp = (H - py + 1) // 2, (W - px + 1) // 2
            if hp <= 0 or wp <= 0:
                continue
            classes.append((py, px, wmat, ry, rx, hp, wp))
    # the four parity classes write disjoint pixel sub-lattices that cover dx:
    # with every class non-empty, each one overwrites its lattice (no zero fill)
    covering = all(c[2] is not None for c in classes)
    if not accumulate and not covering:
        K.zero(dx)
    for py, px, wmat, ry, rx, hp, wp in classes:
        if wmat is None:
            continue
        oy = (py + p - max(ry)) // 2
        ox = (px + p - max(rx)) // 2
        g = K.gather([dy], N, hp, wp, R=len(ry), S=len(rx), oy=oy, ox=ox, Hs=Ho, Ws=Wo)
        K.gemm_fwd(g, wmat, ci, dx, M.d, accumulate=accumulate or not covering, kind="dgrad",
                   strided=(H, W, py, px))
    return dx


# ---------------------------------------------------------------------------
# ResNet34 BasicBlock (timm) and encoder
# ---------------------------------------------------------------------------
def conv_bn_relu_fold(M, srcs, conv, bn, cin_pad=None):
    """relu(BN(conv(x))) with an eval-mode BN folded into the conv and the
    ReLU in the GEMM epilogue (inference only: engine.can_fold)."""
    g, Ho, Wo = conv_gather(srcs, conv)
    wf, bf = E.fold_bn_eval(M, conv, bn, cin_pad)
    a = M.act(srcs[0].shape[0], conv.out_channels, Ho, Wo)
    K.gemm_fwd(g, wf, conv.out_channels, a, M.d, bias=bf, relu=True)
    return a


def basic_fwd(M, blk, x):
    train = blk.bn1.training
    if E.can_fold(M, blk.bn1):
        y1 = st1 = c1 = None
        a1 = conv_bn_relu_fold(M, [x], blk.conv1, blk.bn1)
    else:
        y1, st1 = conv_fwd(M, [x], blk.conv1, train)
        a1 = torch.empty_like(y1)
        c1 = E.bn_fwd_apply(blk.bn1, st1, y1, a1, True, M)
    y2, st2 = conv_fwd(M, [a1], blk.conv2, train)
    yd = cd = None
    if blk.downsample is not None:
        yd, std = conv_fwd(M, [x], blk.downsample[0], train)
        cd = E.bn_coef(blk.downsample[1], std, yd.shape[1])
    out = torch.empty_like(y2)
    r = yd if yd is not None else x
    # out = relu(bn2(y2) + (bn_d(yd) | x))  (timm BasicBlock)
    c2 = E.bn_fwd_apply(blk.bn2, st2, y2, out, True, M, res=r, rcoef=cd)
    return out, (x, y1, c1, a1, y2, c2, yd, cd, out)


def basic_bwd(M, blk, saved, dout, need_dx=True):
    x, y1, c1, a1, y2, c2, yd, cd, out = saved
    N, C_, H, W = out.shape
    g = torch.empty_like(out)
    K.call("vu_relu_mask", K.ptr(dout), K.pstride(dout), K.ptr(out), K.pstride(out), N * H * W, C_,
           K.ptr(g), K.pstride(g), M.d, K.stream())
    dy2 = E.bn_bwd(g, y2, c2, blk.bn2, False, M)
    conv_wgrad(M, dy2, [a1], blk.conv2)
    # conv2 is 3x3 stride 1: its input gradient also emits bn1's first
    # backward reduction stage
    da1, part = conv_dgrad(M, dy2, blk.conv2, torch.empty_like(a1), False, bnb=(y1, c1, True))
    dy1 = E.bn_bwd(da1, y1, c1, blk.bn1, True, M, part=part)
    conv_wgrad(M, dy1, [x], blk.conv1)
    M.notify([blk.conv1.weight, blk.conv2.weight, blk.bn1.weight, blk.bn1.bias,
              blk.bn2.weight, blk.bn2.bias])
    dx = None
    if blk.downsample is not None:
        if need_dx:
            dx = conv_dgrad(M, dy1, blk.conv1, torch.empty_like(x), False)
        dyd = E.bn_bwd(g, yd, cd, blk.downsample[1], False, M)
        conv_wgrad(M, dyd, [x], blk.downsample[0])
        M.notify([blk.downsample[0].weight, blk.downsample[1].weight, blk.downsample[1].bias])
        if need_dx:
            conv_dgrad(M, dyd, blk.downsample[0], dx, True)
    elif need_dx:
        # identity shortcut: dx = g + conv1's input gradient, accumulated by the
        # GEMM epilogue into g itself (g is dead after bn2's backward)
        dx = conv_dgrad(M, dy1, blk.conv1, g, True)
    return dx


def encoder_fwd(M, enc, xa, cin_pad):
    train = enc.bn1.training
    if E.can_fold(M, enc.bn1):
        y0 = c0 = None
        f0 = conv_bn_relu_fold(M, [xa], enc.conv1, enc.bn1, cin_pad=cin_pad)
    else:
        y0, st0 = conv_fwd(M, [xa], enc.conv1, train, cin_pad=cin_pad)
        f0 = torch.empty_like(y0)
        c0 = E.bn_fwd_apply(enc.bn1, st0, y0, f0, True, M)
    N, C_, H, W = f0.shape
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    pm = M.act(N, C_, Ho, Wo)
    idx = torch.empty((N, Ho, Wo, C_), dtype=torch.uint8, device=f0.device)
    K.call("vu_maxpool3s2_fwd", K.ptr(f0), K.pstride(f0), N, H, W, C_, K.ptr(pm), K.pstride(pm),
           K.ptr(idx), M.d, K.stream())
    feats = [f0]
    states = []
    h = pm
    for layer in (enc.layer1, enc.layer2, enc.layer3, enc.layer4):
        ls = []
        for blk in layer:
            h, s = basic_fwd(M, blk, h)
            ls.append(s)
        states.append(ls)
        feats.append(h)
    return feats, (xa, y0, c0, f0, idx, states)


def encoder_bwd(M, enc, state, dfeats, cvalid):
    """dfeats: gradients of the five features (None = no gradient)."""
    xa, y0, c0, f0, idx, states = state
    layers = (enc.layer1, enc.layer2, enc.layer3, enc.layer4)
    d = None
    for li in range(3, -1, -1):
        df = dfeats[li + 1]
        if df is not None:
            if d is None:
                d = df
            else:
                K.copy(df, d, accumulate=True)
        if d is None:
            continue
        for blk, s in zip(reversed(list(layers[li])), reversed(states[li])):
            d = basic_bwd(M, blk, s, d)
    N, C_, H, W = f0.shape
    dfz = torch.empty_like(f0)
    if d is not None:
        K.call("vu_maxpool3s2_bwd", K.ptr(d), K.pstride(d), K.ptr(idx), N, H, W, C_, K.ptr(dfz),
               K.pstride(dfz), 0, M.d, K.stream())
    else:
        dfz.zero_()
    if dfeats[0] is not None:
        K.copy(dfeats[0], dfz, accumulate=True)
    dy0 = E.bn_bwd(dfz, y0, c0, enc.bn1, True, M)
    conv_wgrad(M, dy0, [xa], enc.conv1, cvalid=cvalid)
    M.notify([enc.conv1.weight, enc.bn1.weight, enc.bn1.bias])


# ---------------------------------------------------------------------------
# 1x1 conv + BN + ReLU on a latent broadcast (z_initial 150-154, z_proj 37-41)
# ---------------------------------------------------------------------------
def latent_map(M, z, N, H, W):
    """[B, L] fp32 -> spatially constant NHWC [B, L, H, W] in the storage dtype."""
    L = z.shape[1]
    zb = M.act(N, L, H, W)
    K.call("vu_sample_broadcast", K.ptr(z), N, H * W, L, 1.0, K.ptr(zb), K.pstride(zb), 0, M.d,
           K.stream())
    return zb


def cbr1x1_fwd(M, seq, x, out=None):
    conv, bn = seq[0], seq[1]
    if E.can_fold(M, bn) and out is None:
        return conv_bn_relu_fold(M, [x], conv, bn), None
    y, st = conv_fwd(M, [x], conv, bn.training)
    a = torch.empty_like(y) if out is None else out
    c = E.bn_fwd_apply(bn, st, y, a, True, M)
    return a, (x, y, c)


def cbr1x1_bwd(M, seq, saved, da):
    conv, bn = seq[0], seq[1]
    x, y, c = saved
    dy = E.bn_bwd(da, y, c, bn, True, M)
    conv_wgrad(M, dy, [x], conv, bn=bn)
    M.notify([conv.weight, conv.bias, bn.weight, bn.bias])
    dx = torch.empty_like(x)
    K.gemm_fwd(K.gather1x1([dy]), E.w1x1_dgrad(conv.weight, M.d), x.shape[1], dx, M.d,
               kind="dgrad")
    return dx


def sample_sum(M, x, scale=1.0, out=None, accumulate=False):
    N, C_, H, W = x.shape
    if out is None:
        out = torch.empty((N, C_), dtype=torch.float32, device=x.device)
    ws = torch.empty(K.query("vu_sample_sum_workspace_bytes", N, C_) // 4 + 1, dtype=torch.float32,
                     device=x.device)
    K.call("vu_sample_sum", K.ptr(x), K.pstride(x), N, H * W, C_, float(scale), K.ptr(out),
           1 if accumulate else 0, K.ptr(ws), K.dcode(x.dtype), K.stream())
    return out


# ---------------------------------------------------------------------------
# DecoderBlock (unet_resnet.py:31-101)
# ---------------------------------------------------------------------------
def decoder_fwd(M, blk, x, skip, z, zp_vec=None):
    """zp_vec: the block's z_proj map already written by the latent vector
    path (latent_fwd; cpad channels incl. the zero padding) -- its backward
    is then deferred to latent_bwd (decoder_bwd returns the map's gradient);
    or a ZShortcut (round 5): no map at all, conv1 contracts over [x, skip]
    and adds the z part as its per-sample border-class bias table."""
    N = x.shape[0]
    if skip is not None:
        H, W = skip.shape[2], skip.shape[3]
    else:
        H, W = 2 * x.shape[2], 2 * x.shape[3]
    xu = M.act(N, x.shape[1], H, W)
    K.upsample_fwd(x, xu, H, W, 0, 0, M.d)
    srcs = [xu]
    satt = None
    if skip is not None and blk.use_skip:
        if blk.use_attention:
            sk, satt = E.attention_fwd(M, blk.attention, xu, skip)
        else:
            sk = skip
        srcs.append(sk)
    szp = None
    cpad = None
    zsc = zp_vec if isinstance(zp_vec, ZShortcut) else None
    if zsc is not None:
        szp = zsc
    elif blk.use_latent and zp_vec is not None:
        L = blk.z_proj[0].out_channels
        lead = sum(t.shape[1] for t in srcs)
        if zp_vec.shape[1] != L:
            cpad = lead + zp_vec.shape[1]
        srcs.append(zp_vec)
        szp = "vec"
    elif blk.use_latent:
        if z.dim() == 2:
            # interpolate([B, L, 1, 1] -> (H, W), align_corners) is a broadcast
            zb = latent_map(M, z, N, H, W)
        else:
            # a spatial z [B, L, h, w] (the reference's z_spatial, unet_resnet.py:93)
            zb = M.act(N, z.shape[1], H, W)
            K.upsample_fwd(z, zb, H, W, 0, 0, M.d)
        L = blk.z_proj[0].out_channels
        lead = sum(t.shape[1] for t in srcs)
        Lp = -(-L // 64) * 64
        if lead % 64 == 0 and Lp != L:
            # pad the z_proj source to 64 channels (zeros): every concat group
            # is then 64-aligned, so conv1's weight gradient runs on the halo
            # kernel and its input gradient keeps a tile-multiple column count
            zp = M.act(N, Lp, H, W)
            K.zero(zp[:, L:])
            _, szp = cbr1x1_fwd(M, blk.z_proj, zb, out=zp[:, :L])
            cpad = lead + Lp
        else:
            zp, szp = cbr1x1_fwd(M, blk.z_proj, zb)
        srcs.append(zp)
    if zsc is not None:
        a1, s1 = E.conv_bn_relu_fwd(M, srcs, blk.conv1[0], blk.conv1[1], zbias=zsc.table, cin_use=zsc.lead)
    else:
        a1, s1 = E.conv_bn_relu_fwd(M, srcs, blk.conv1[0], blk.conv1[1], cin_pad=cpad)
    a2, s2 = E.conv_bn_relu_fwd(M, [a1], blk.conv2[0], blk.conv2[1])
    return a2, (x, skip, xu, srcs, satt, szp, a1, s1, s2, cpad)


def decoder_bwd(M, blk, saved, dout, z=None):
    """-> (dx, dskip or None, dz or None): dz is [B, L] fp32 for a vector z,
    an NHWC map like ``z`` for a spatial one."""
    x, skip, xu, srcs, satt, szp, a1, s1, s2, cpad = saved
    da1, part = E.conv_bn_relu_bwd(M, [a1], blk.conv2[0], blk.conv2[1], s2, dout, True,
                                   feeds=(s1, blk.conv1[1]))
    conv1 = blk.conv1[0]
    zsc = szp if isinstance(szp, ZShortcut) else None
    if zsc is not None:
        # one gradient sink for both writers of conv1.weight.grad (the GEMM:
        # the [x, skip] columns; latent_bwd's vu_zbias_bwd: the z columns)
        zsc.sink = E.grad_sink(conv1.weight)
    dsrc = E.conv_bn_relu_bwd(M, srcs, conv1, blk.conv1[1], s1, da1, True,
                              cvalid=conv1.in_channels if cpad else None, cin_pad=cpad, da_part=part,
                              shortcut=zsc)
    cx = xu.shape[1]
    off = cx
    dskip = dz = None
    if skip is not None and blk.use_skip:
        cs = skip.shape[1]
        dsk = dsrc[:, off:off + cs]
        if blk.use_attention:
            dskip = E.attention_bwd(M, blk.attention, satt, dsk, (dsrc, 0), True)
        else:
            dskip = dsk
        off += cs
    if zsc is not None:
        dz = ("shortcut", zsc)   # the z part's backward runs in latent_bwd (vu_zbias_bwd)
    elif blk.use_latent and szp == "vec":
        # the z_proj backward runs on the sample vectors (latent_bwd)
        dz = ("vec", dsrc[:, off:off + blk.z_proj[0].out_channels])
    elif blk.use_latent:
        dzp = dsrc[:, off:off + blk.z_proj[0].out_channels]
        dzb = cbr1x1_bwd(M, blk.z_proj, szp, dzp)
        if z is not None and z.dim() == 4:
            dz = torch.empty_like(z)
            K.upsample_bwd(dzb, dz, dzb.shape[2], dzb.shape[3], 0, 0, False, M.d)
        else:
            dz = sample_sum(M, dzb)
    dx = torch.empty_like(x)
    H, W = xu.shape[2], xu.shape[3]
    K.upsample_bwd(dsrc[:, :cx], dx, H, W, 0, 0, False, M.d)
    return dx, dskip, dz


# ---------------------------------------------------------------------------
# latent vector path (round 4; csrc/latent.hip): the bottleneck heads,
# reparameterize and every consumer of z (z_initial, the DecoderBlocks'
# z_proj) on the [N, L] sample vectors -- downstream of z every map is a
# per-sample constant (interpolate of z[..., None, None] is a broadcast), so a
# 1x1 conv + train-mode BatchNorm + ReLU of it is the same arithmetic on the N
# vectors, with the batch statistics over N * HW pixels equal to those of the
# vectors.  4 launches per step instead of ~50 (sample sums, two heads,
# reparameterize, 5 broadcasts, 5 1x1 GEMMs, their BatchNorm passes, and the
# same again backwards).
# ---------------------------------------------------------------------------
LATENT_VECTORS = True  # A/B switch: False = the round-3 map path


def _consumer_ok(M, seq):
    conv, bn = seq[0], seq[1]
    co = conv.out_channels
    return (conv.kernel_size == (1, 1) and conv.stride == (1, 1) and conv.groups == 1
            and (bn.training or bn.running_mean is not None) and bn.momentum is not None
            and co % 8 == 0 and (co // 8) & (co // 8 - 1) == 0 and co <= 2048)


def latent_vectors_ok(M, model, N):
    """The vector path serves this model / batch (otherwise the map path)."""
    if not LATENT_VECTORS or N > 64 or model.latent_dim > 64:
        return False
    c4 = model.mu_head[0].in_channels
    if c4 % 8 or (c4 // 8) & (c4 // 8 - 1) or c4 > 2048:
        return False
    seqs = ([model.z_initial] if model.use_bottleneck else []) + \
        [b.z_proj for b in model.decoder_blocks if b.use_latent]
    sum_co = sum(s[0].out_channels for s in seqs)
    if not K.query("vu_latent_bwd_supported", N, model.latent_dim, sum_co, c4):
        return False
    return all(_consumer_ok(M, s) for s in seqs)


def heads_fwd(M, model, f4, eps):
    """pooled [N, C], mu, logvar, z [N, L] (fp32) in one launch."""
    N, C4, H4, W4 = f4.shape
    L = model.latent_dim
    dev = f4.device
    pooled = torch.empty((N, C4), dtype=torch.float32, device=dev)
    mu = torch.empty((N, L), dtype=torch.float32, device=dev)
    logvar = torch.empty_like(mu)
    z = torch.empty_like(mu)
    hm, hl = model.mu_head[0], model.logvar_head[0]
    K.call("vu_vae_heads_fwd", K.ptr(f4), K.pstride(f4), N, H4 * W4, C4, K.ptr(hm.weight), K.ptr(hm.bias),
           K.ptr(hl.weight), K.ptr(hl.bias), L, K.ptr(eps), K.ptr(pooled), K.ptr(mu), K.ptr(logvar), K.ptr(z),
           K.dcode(f4.dtype), K.stream())
    return pooled, mu, logvar, z


class LatentConsumer:
    """One 1x1 conv + BatchNorm + ReLU applied to the broadcast latent: its
    output map (``out``, cpad >= co channels, zeros past co) and the saved
    vectors y [N, co] (pre-BN) and coef [4, co] (scale, shift, mean, invstd)."""

    def __init__(self, seq, out, shape=None):
        """out None (the latent shortcut): no map; shape = (N, H, W, device)
        and the activated vectors land in ``act`` [N, co]."""
        self.conv, self.bn = seq[0], seq[1]
        self.out = out
        if out is not None:
            N, _, H, W = out.shape
            dev = out.device
        else:
            N, H, W, dev = shape
        co = self.conv.out_channels
        self.HW = H * W
        self.y = torch.empty((N, co), dtype=torch.float32, device=dev)
        self.coef = torch.empty((4, co), dtype=torch.float32, device=dev)
        self.act = torch.empty((N, co), dtype=torch.float32, device=dev) if out is None else None
        self.dmap = None
        self.zsc = None   # the ZShortcut this consumer feeds

    def job(self):
        conv, bn = self.conv, self.bn
        j = _lib.VuLatentJob()
        track = bn.running_mean is not None
        j.w, j.bias = conv.weight.data_ptr(), (conv.bias.data_ptr() if conv.bias is not None else None)
        j.gamma, j.beta = bn.weight.data_ptr(), bn.bias.data_ptr()
        j.running_mean = bn.running_mean.data_ptr() if track else None
        j.running_var = bn.running_var.data_ptr() if track else None
        j.num_batches_tracked = bn.num_batches_tracked.data_ptr() if track and bn.training else None
        j.momentum, j.eps = float(bn.momentum), float(bn.eps)
        j.train = 1 if bn.training else 0
        if self.out is not None:
            j.co, j.cpad, j.HW = conv.out_channels, self.out.shape[1], self.HW
            j.out, j.out_stride = self.out.data_ptr(), K.pstride(self.out)
        else:
            j.co, j.cpad, j.HW = conv.out_channels, conv.out_channels, self.HW
            j.out, j.out_stride = None, 0
        j.act = K.ptr(self.act)
        j.y, j.coef = self.y.data_ptr(), self.coef.data_ptr()
        return j


def _jobs(cons):
    arr = (_lib.VuLatentJob * len(cons))()
    for i, c in enumerate(cons):
        arr[i] = c.job()
    return arr


def latent_consumers(M, model, feats, N, skip_always=False):
    """The consumers of z for a batch of N over encoder features ``feats``:
    z_initial (if the bottleneck is used) and the z_proj of every latent
    DecoderBlock, each with its output map allocated at the size that block
    sees (the skip's, or twice its input's) -- the z_proj maps channel-padded
    to 64 when the concat before them is 64-aligned (decoder_fwd's layout).
    Returns (consumers, per-block z_proj map, ZShortcut (the round-5 latent
    shortcut: no map) or None)."""
    f4 = feats[-1]
    H4, W4 = f4.shape[2], f4.shape[3]
    cons, zps = [], [None] * len(model.decoder_blocks)
    if model.use_bottleneck:
        cons.append(LatentConsumer(model.z_initial, M.act(N, model.z_initial[0].out_channels, H4, W4)))
    size = (H4, W4)
    for i, blk in enumerate(model.decoder_blocks):
        use = i < len(feats) - 1 and (skip_always or model.use_skip)
        skip = feats[-(i + 2)] if use else None
        size = (skip.shape[2], skip.shape[3]) if skip is not None else (2 * size[0], 2 * size[1])
        if blk.use_latent:
            Lb = blk.z_proj[0].out_channels
            lead = blk.conv1[0].in_channels - Lb
            if shortcut_ok(M, blk, N, size):
                c = LatentConsumer(blk.z_proj, None, (N, size[0], size[1], f4.device))
                c.zsc = ZShortcut(blk, c, lead, size[0], size[1])
                cons.append(c)
                zps[i] = c.zsc
                continue
            Lp = -(-Lb // 64) * 64
            cpad = Lp if (lead % 64 == 0 and Lp != Lb) else Lb
            cons.append(LatentConsumer(blk.z_proj, M.act(N, cpad, size[0], size[1])))
            zps[i] = cons[-1].out
    return cons, zps


# The latent shortcut (round 5, csrc/zbias.hip): a DecoderBlock conv1 whose
# z_proj source is the per-sample constant map of the vector path contracts
# over [x, skip] only; the z part is a per-sample, per-border-class bias of
# its GEMM epilogue, its backward per-sample region sums of conv1's dy.
LATENT_SHORTCUT = True   # A/B switch: False = the round-4 map (64-channel padded z_proj source)
# Round 6: conv1's BatchNorm backward apply -- the pass
# that writes dy -- also writes the shortcut's region partials
# (vu_bn_bwd_apply_zrs), so vu_zbias_bwd skips its re-read of dy.  A/B switch.
FUSE_ZBIAS_REGIONS = True


def shortcut_ok(M, blk, N, size):
    conv1 = blk.conv1[0]
    Lb = blk.z_proj[0].out_channels
    lead = conv1.in_channels - Lb
    epc = 8 if M.d != F32 else 4
    return (LATENT_SHORTCUT and size[0] >= 2 and size[1] >= 2 and lead > 0 and lead % epc == 0
            and conv1.kernel_size == (3, 3) and conv1.stride == (1, 1) and conv1.padding == (1, 1)
            and conv1.groups == 1 and conv1.bias is None
            and bool(K.query("vu_zbias_supported", N, Lb, conv1.out_channels)))


class ZShortcut:
    """One DecoderBlock's latent shortcut: conv1's input channels [lead,
    lead + L) are the consumer's constant map c_n (consumer.act)."""

    def __init__(self, blk, cons, lead, H, W):
        self.blk, self.cons, self.lead, self.H, self.W = blk, cons, lead, H, W
        N = cons.act.shape[0]
        self.table = torch.empty((N, 9, blk.conv1[0].out_channels), dtype=torch.float32,
                                 device=cons.act.device)
        self.row_scale = None    # eval-mode BN folded into conv1 (inference)
        self.dy = None           # backward: conv1's pre-BN gradient (engine.conv_bn_relu_bwd)
        self.sink = None         # backward: (conv1.weight.grad, accumulate)
        self.zrs = None          # backward: K.ZbiasRegions (region partials from the BN apply pass)

    def regions(self, y):
        """The region-partial buffer conv1's BatchNorm backward apply fills
        (FUSE_ZBIAS_REGIONS; None = the separate region pass)."""
        self.zrs = None
        if FUSE_ZBIAS_REGIONS:
            N, co = y.shape[0], self.blk.conv1[0].out_channels
            self.zrs = K.ZbiasRegions(torch.empty(K.query("vu_zbias_rs_floats", N, co, self.H, self.W),
                                                  dtype=torch.float32, device=y.device))
        return self.zrs

    def job(self):
        conv1 = self.blk.conv1[0]
        w = conv1.weight
        j = _lib.VuZbJob()
        j.w = w.data_ptr()
        j.ws_co, j.ws_ci, j.ws_ky, j.ws_kx = w.stride()
        j.cz0, j.L, j.co, j.H, j.W = self.lead, self.cons.conv.out_channels, conv1.out_channels, self.H, self.W
        j.act = self.cons.act.data_ptr()
        j.row_scale = K.ptr(self.row_scale)
        j.table = self.table.data_ptr()
        return j


def _zb_jobs(zscs):
    arr = (_lib.VuZbJob * len(zscs))()
    for i, z in enumerate(zscs):
        arr[i] = z.job()
    return arr


def zbias_tables(M, zscs):
    """Every shortcut block's [N][9][co] table from the consumers' vectors (one launch)."""
    if not zscs:
        return
    for z in zscs:
        bn1 = z.blk.conv1[1]
        z.row_scale = E.bn_coef(bn1, None, z.blk.conv1[0].out_channels)[0] if E.can_fold(M, bn1) else None
    K.call("vu_zbias_fwd", _zb_jobs(zscs), len(zscs), zscs[0].table.shape[0], K.stream())


def zbias_backward(M, zscs, parts):
    """The shortcut blocks' z-part backward (two launches): conv1.weight.grad's
    z columns and the consumers' dc partials (into ``parts``), then conv1's
    weight reported to the DP reducer (behind its GEMM weight gradient)."""
    N = zscs[0].table.shape[0]
    arr = _zb_jobs(zscs)
    keep, fix = [], []
    for i, z in enumerate(zscs):
        conv1 = z.blk.conv1[0]
        g, acc = z.sink
        if g is not None and g.stride() != conv1.weight.stride():
            # the kernel addresses dW with the weight's strides: a gradient of
            # another layout takes the z columns through a weight-layout buffer
            tmp = torch.empty_like(conv1.weight)
            fix.append((g, acc, tmp, z.lead, z.lead + z.cons.conv.out_channels))
            g, acc = tmp, False
        # the region pass skips a job whose BatchNorm apply pass wrote its partials
        ready = z.zrs is not None and z.zrs.ready
        rs = z.zrs.rs if ready else torch.empty(K.query("vu_zbias_rs_floats", N, conv1.out_channels, z.H, z.W),
                                                dtype=torch.float32, device=z.table.device)
        keep.append(rs)
        arr[i].dy, arr[i].dy_stride = z.dy.data_ptr(), K.pstride(z.dy)
        arr[i].rs, arr[i].part = rs.data_ptr(), parts[i].data_ptr()
        arr[i].dw, arr[i].grad_acc = K.ptr(g), 1 if acc else 0
        arr[i].rs_ready = 1 if ready else 0
    K.call("vu_zbias_bwd", arr, len(zscs), N, K.dcode(zscs[0].dy.dtype), K.stream())
    for g, acc, tmp, a, b in fix:
        if acc:
            g[:, a:b].add_(tmp[:, a:b])
        else:
            g[:, a:b].copy_(tmp[:, a:b])
    ws = [z.blk.conv1[0].weight for z in zscs if z.sink[0] is not None]
    M.side(lambda: M.notify(ws), *[z.dy for z in zscs])
    for z in zscs:
        z.dy = None
        z.sink = None
        z.zrs = None
    return keep


def latent_fwd(M, z, cons):
    """Every consumer's map from z [N, L] in one launch."""
    if not cons:
        return
    for c in cons:
        if c.out is not None:
            K.call("vu_latent_check_job", c.conv.out_channels, c.out.shape[1], K.pstride(c.out), M.d)
    K.call("vu_latent_fwd", _jobs(cons), len(cons), K.ptr(z), z.shape[0], z.shape[1], M.d, K.stream())


def latent_bwd(M, model, cons, z, eps, logvar, pooled, dmu, dlogvar):
    """Backward of the consumers (their map gradients in ``c.dmap``), of
    reparameterize and of both heads -> dpooled [N, C4] (fp32)."""
    N, L = z.shape
    dev = z.device
    arr = _jobs(cons)
    keep = []
    parts = []
    for i, c in enumerate(cons):
        part = torch.empty(K.query("vu_latent_part_floats", N, c.conv.out_channels), dtype=torch.float32,
                           device=dev)
        keep.append(part)
        parts.append(part)
        if c.zsc is None:
            arr[i].dmap, arr[i].dmap_stride = c.dmap.data_ptr(), K.pstride(c.dmap)
        arr[i].part = part.data_ptr()
        gw, accw = E.grad_sink(c.conv.weight)
        gb, accb = E.grad_sink(c.conv.bias) if c.conv.bias is not None else (None, accw)
        gg, gbe, accn = E.bn_grad_sinks(c.bn)
        accs = {a for g, a in ((gw, accw), (gb, accb), (gg, accn)) if g is not None}
        if len(accs) > 1:
            raise RuntimeError("latent consumer: inconsistent gradient state")
        arr[i].grad_acc = 1 if accs == {True} else 0
        arr[i].dw, arr[i].dbias = K.ptr(gw), K.ptr(gb)
        arr[i].dgamma, arr[i].dbeta = K.ptr(gg), K.ptr(gbe)
    zi = [i for i, c in enumerate(cons) if c.zsc is not None]
    if zi:
        keep += zbias_backward(M, [cons[i].zsc for i in zi], [parts[i] for i in zi])
    mi = [i for i, c in enumerate(cons) if c.zsc is None]
    if mi:
        sub = (_lib.VuLatentJob * len(mi))()
        for k, i in enumerate(mi):
            sub[k] = arr[i]
        K.call("vu_latent_bwd_sums", sub, len(mi), N, K.dcode(cons[mi[0]].dmap.dtype), K.stream())
    hm, hl = model.mu_head[0], model.logvar_head[0]
    h = _lib.VuLatentHeads()
    dpooled = torch.empty_like(pooled)
    dmu_c = dmu.float().contiguous() if dmu is not None else None
    dlv_c = dlogvar.float().contiguous() if dlogvar is not None else None
    h.z, h.eps, h.logvar = z.data_ptr(), K.ptr(eps), logvar.data_ptr()
    h.dmu_in, h.dlv_in = K.ptr(dmu_c), K.ptr(dlv_c)
    h.pooled, h.w_mu, h.w_lv = pooled.data_ptr(), hm.weight.data_ptr(), hl.weight.data_ptr()
    sinks = [E.grad_sink(p) for p in (hm.weight, hm.bias, hl.weight, hl.bias)]
    accs = {a for g, a in sinks if g is not None}
    if len(accs) > 1:
        raise RuntimeError("VAE heads: inconsistent gradient state")
    h.dw_mu, h.db_mu, h.dw_lv, h.db_lv = (K.ptr(g) for g, _ in sinks)
    h.dpooled, h.C, h.grad_acc = dpooled.data_ptr(), pooled.shape[1], 1 if accs == {True} else 0
    sum_co = sum(c.conv.out_channels for c in cons)
    ws = K.workspace_f32(K.query("vu_latent_bwd_workspace_bytes", N, L, sum_co), dev)  # dz partials
    keep.append(ws)
    K.call("vu_latent_bwd", arr, len(cons), C.byref(h), N, L, K.ptr(ws), K.stream())
    ps = [hm.weight, hm.bias, hl.weight, hl.bias]
    for c in cons:
        ps += [c.conv.weight, c.conv.bias, c.bn.weight, c.bn.bias]
    M.notify(ps)
    return dpooled


# ---------------------------------------------------------------------------
# whole UNetResNet forward / backward (unet_resnet.py:196-240)
# ---------------------------------------------------------------------------
def vae_fwd(M, model, x, eps):
    N, cin, Hin, Win = x.shape
    cp = (cin + 7) // 8 * 8
    xa = E.to_act(M, x, cp)
    feats, senc = encoder_fwd(M, model.encoder, xa, cp)
    out, mu, logvar, stail = vae_tail_fwd(M, model, feats, Hin, Win, eps)
    return out, mu, logvar, (senc, stail, cin)


def vae_bwd(M, model, state, dout, dmu, dlogvar):
    senc, stail, cin = state
    dfeats = vae_tail_bwd(M, model, stail, dout, dmu, dlogvar)
    encoder_bwd(M, model.encoder, senc, dfeats, cin)


def vae_tail_fwd(M, model, feats, Hin, Win, eps):
    """Everything after the encoder (unet_resnet.py:203-240): heads, reparameterize,
    bottleneck, the four DecoderBlocks, final_conv and the resize to the input size."""
    f4 = feats[-1]
    N = f4.shape[0]
    dev = f4.device
    H4, W4 = f4.shape[2], f4.shape[3]
    L = model.latent_dim
    sampling = model.latent_injection not in ("none", "inject_no_bottleneck")
    if not sampling:
        eps = None
    vec = latent_vectors_ok(M, model, N)
    cons, zps = [], [None] * len(model.decoder_blocks)
    if vec:
        pooled, mu, logvar, z = heads_fwd(M, model, f4, eps)
        cons, zps = latent_consumers(M, model, feats, N)
        latent_fwd(M, z, cons)
        zbias_tables(M, [c.zsc for c in cons if c.zsc is not None])
    else:
        pooled = sample_sum(M, f4, 1.0 / (H4 * W4))
        mu = torch.empty((N, L), dtype=torch.float32, device=dev)
        logvar = torch.empty_like(mu)
        for head, out in ((model.mu_head[0], mu), (model.logvar_head[0], logvar)):
            K.call("vu_linear_small_fwd", K.ptr(pooled), N, f4.shape[1], K.ptr(head.weight),
                   K.ptr(head.bias), L, K.ptr(out), K.stream())
        z = torch.empty_like(mu)
        K.call("vu_reparam_fwd", K.ptr(mu), K.ptr(logvar), K.ptr(eps), N * L, K.ptr(z), K.stream())
    szi = None
    if model.use_bottleneck:
        if vec:
            h = cons[0].out
        else:
            h, szi = cbr1x1_fwd(M, model.z_initial, latent_map(M, z, N, H4, W4))
    else:
        h = f4
    sdec = []
    for i, blk in enumerate(model.decoder_blocks):
        skip = feats[-(i + 2)] if (i < len(feats) - 1 and model.use_skip) else None
        h, s = decoder_fwd(M, blk, h, skip, z, zp_vec=zps[i])
        sdec.append(s)
    small, sfc = E.outconv_fwd(M, model.final_conv, h)
    out = torch.empty((N, small.shape[1], Hin, Win), dtype=torch.float32, device=dev,
                      memory_format=torch.channels_last)
    K.upsample_fwd(small, out, Hin, Win, 0, 0, F32)
    return out, mu, logvar, (feats, pooled, eps, logvar, szi, sdec, sfc, small, (cons, z) if vec else None)


def vae_tail_bwd(M, model, state, dout, dmu, dlogvar):
    """-> gradients of the five encoder features (None where none flows)."""
    feats, pooled, eps, logvar, szi, sdec, sfc, small, lat = state
    N = small.shape[0]
    dsmall = torch.empty_like(small)
    if dout is not None:
        dout = dout.float().contiguous(memory_format=torch.channels_last)
        K.upsample_bwd(dout, dsmall, dout.shape[2], dout.shape[3], 0, 0, False, F32)
    else:
        dsmall.zero_()
    dh = E.outconv_bwd(M, model.final_conv, sfc, dsmall)
    L = model.latent_dim
    dfeats = [None] * len(feats)
    f4 = feats[-1]
    C4, HW4 = f4.shape[1], f4.shape[2] * f4.shape[3]
    if lat is not None:
        cons, z = lat
        byblk = {}
        k = 1 if model.use_bottleneck else 0
        for i, blk in enumerate(model.decoder_blocks):
            if blk.use_latent:
                byblk[i] = cons[k]
                k += 1
        for i in range(len(model.decoder_blocks) - 1, -1, -1):
            dh, dskip, dzi = decoder_bwd(M, model.decoder_blocks[i], sdec[i], dh)
            if dskip is not None:
                dfeats[len(feats) - 2 - i] = dskip
            if dzi is not None and dzi[0] == "vec":
                byblk[i].dmap = dzi[1]
        df4 = None
        if model.use_bottleneck:
            cons[0].dmap = dh
        else:
            df4 = dh
        dpooled = latent_bwd(M, model, cons, z, eps, logvar, pooled, dmu, dlogvar)
        if df4 is None:
            df4 = M.act(N, C4, f4.shape[2], f4.shape[3])
        K.call("vu_sample_broadcast", K.ptr(dpooled), N, HW4, C4, 1.0 / HW4, K.ptr(df4),
               K.pstride(df4), 0 if df4 is not dh else 1, M.d, K.stream())
        dfeats[-1] = df4
        return dfeats
    dz = torch.zeros((N, L), dtype=torch.float32, device=small.device)
    for i in range(len(model.decoder_blocks) - 1, -1, -1):
        dh, dskip, dzi = decoder_bwd(M, model.decoder_blocks[i], sdec[i], dh)
        if dskip is not None:
            dfeats[len(feats) - 2 - i] = dskip
        if dzi is not None:
            K.call("vu_sample_broadcast", K.ptr(dzi), 1, 1, N * L, 1.0, K.ptr(dz), N * L, 1, F32,
                   K.stream())
    if model.use_bottleneck:
        dzs = cbr1x1_bwd(M, model.z_initial, szi, dh)
        sample_sum(M, dzs, 1.0, out=dz, accumulate=True)
        df4 = None
    else:
        df4 = dh
    dmu_t = dmu.float().contiguous().clone() if dmu is not None else torch.zeros_like(dz)
    dlv_t = dlogvar.float().contiguous().clone() if dlogvar is not None else torch.zeros_like(dz)
    K.call("vu_reparam_bwd", K.ptr(logvar), K.ptr(eps), K.ptr(dz), N * L, K.ptr(dmu_t),
           K.ptr(dlv_t), 1, K.stream())
    dpooled = torch.empty((N, C4), dtype=torch.float32, device=f4.device)
    first = True
    for head, dh_ in ((model.mu_head[0], dmu_t), (model.logvar_head[0], dlv_t)):
        gw, acc = E.grad_sink(head.weight)
        gb, _ = E.grad_sink(head.bias)
        K.call("vu_linear_small_bwd", K.ptr(pooled), N, C4, K.ptr(head.weight), L, K.ptr(dh_),
               K.ptr(dpooled), 0 if first else 1, K.ptr(gw), K.ptr(gb), 1 if acc else 0, K.stream())
        first = False
        M.notify([head.weight, head.bias])
    if df4 is None:
        df4 = M.act(N, C4, f4.shape[2], f4.shape[3])
        K.call("vu_sample_broadcast", K.ptr(dpooled), N, HW4, C4, 1.0 / HW4, K.ptr(df4),
               K.pstride(df4), 0, M.d, K.stream())
    else:
        K.call("vu_sample_broadcast", K.ptr(dpooled), N, HW4, C4, 1.0 / HW4, K.ptr(df4),
               K.pstride(df4), 1, M.d, K.stream())
    dfeats[-1] = df4
    return dfeats
