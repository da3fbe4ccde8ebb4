"""VAE-U-Net (drop-in for the reference's unet/unet_resnet.py:1-279).

``UNetResNet`` keeps the reference's constructor signature, attribute tree
(``encoder`` / ``mu_head`` / ``logvar_head`` / ``z_initial`` /
``decoder_blocks`` / ``final_conv``) and all 389 state_dict keys.  The
encoder is a from-scratch ResNet34 feature extractor with timm's
``resnet34`` parameter names (conv1, bn1, layer1..4 of BasicBlocks with
conv1/bn1/conv2/bn2/downsample), so timm-format checkpoints load unchanged;
timm itself is not required (and pretrained weights cannot be downloaded in
an offline run: ``pretrained=True`` warns and keeps the random init).

The whole network runs as one autograd node over the fused HIP sequences of
vae_engine.py; ``DecoderBlock`` also runs standalone (called directly by the
reference's inference code, utils/vae_utils.py:63-65).
"""
import warnings

import torch
import torch.nn as nn

from . import engine as E
from . import vae_engine as V
from .functional import BlockFn, Runner, run_block, act_grad
from .unet_parts import AttentionGate


class _FeatureInfo:
    def __init__(self, chs, reductions):
        self._chs, self._red = chs, reductions

    def channels(self):
        return list(self._chs)

    def reduction(self):
        return list(self._red)


class BasicBlock(nn.Module):
    """timm ResNet BasicBlock parameter layout: conv1/bn1/conv2/bn2(/downsample)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.act2 = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or inplanes != planes:
            self.downsample = nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride=stride, bias=False),
                                            nn.BatchNorm2d(planes))


class ResNet34Features(nn.Module):
    """ResNet34 ``features_only`` encoder: [act1 (/2), layer1 (/4), layer2 (/8),
    layer3 (/16), layer4 (/32)] with channels [64, 64, 128, 256, 512]."""

    def __init__(self, in_chans=3):
        super().__init__()
        self.conv1 = nn.Conv2d(in_chans, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.act1 = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        cfg = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]
        inpl = 64
        for li, (planes, n, stride) in enumerate(cfg):
            blocks = [BasicBlock(inpl, planes, stride)]
            blocks += [BasicBlock(planes, planes) for _ in range(n - 1)]
            setattr(self, f"layer{li + 1}", nn.Sequential(*blocks))
            inpl = planes
        self.feature_info = _FeatureInfo([64, 64, 128, 256, 512], [2, 4, 8, 16, 32])
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        M = E.current_mode(x.device)
        cp = (x.shape[1] + 7) // 8 * 8
        with torch.no_grad():
            feats, _ = V.encoder_fwd(M, self, E.to_act(M, x, cp), cp)
        return feats


def _cbr1x1(cin, cout):
    return nn.Sequential(nn.Conv2d(cin, cout, 1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


def _cbr3x3(cin, cout):
    return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout),
                         nn.ReLU(inplace=True))


class DecoderBlock(nn.Module):
    """bilinear(align_corners) -> [attention(skip)] -> [z_proj] -> cat -> 2x conv3x3+BN+ReLU
    (unet_resnet.py:31-101)."""

    def __init__(self, in_channels, skip_channels, out_channels, latent_dim, use_attention=True,
                 use_skip=True, use_latent=True):
        super().__init__()
        self.use_latent = use_latent
        if use_latent:
            self.z_proj = _cbr1x1(latent_dim, latent_dim)
        self.use_skip = use_skip
        self.use_attention = use_attention and use_skip
        if self.use_attention:
            self.attention = AttentionGate(in_channels, skip_channels, in_channels // 4)
        cin = in_channels + (skip_channels if use_skip else 0) + (latent_dim if use_latent else 0)
        self.conv1 = _cbr3x3(cin, out_channels)
        self.conv2 = _cbr3x3(out_channels, out_channels)

    def forward(self, x, skip, z):
        """z: [B, L], [B, L, 1, 1] or the reference's spatial z_spatial
        [B, L, h, w] (utils/vae_utils.py:55-65, visualize_vae.py:71-77), which
        is resampled to the skip size exactly as unet_resnet.py:93 does."""
        M = E.current_mode(x.device)
        spatial = z.dim() == 4 and z.shape[2] * z.shape[3] > 1
        if self.use_latent and (z.shape[1] if z.dim() > 1 else -1) != self.z_proj[0].in_channels:
            raise ValueError("z must be [B, latent_dim] or [B, latent_dim, h, w]")
        zv = None if spatial else z.reshape(z.shape[0], -1).float().contiguous()
        inputs = (x, skip, z) if skip is not None else (x, z)

        def fwd(inp):
            xa = E.to_act(M, inp[0])
            sa = E.to_act(M, inp[1]) if skip is not None else None
            za = E.to_act(M, inp[-1]) if spatial else zv
            out, st = V.decoder_fwd(M, self, xa, sa, za)
            return out, (st, za)

        def bwd(state, dout):
            st, za = state
            dx, dskip, dz = V.decoder_bwd(M, self, st, act_grad(M, dout), za)
            gx = E.from_act(dx, x)
            if dz is None:
                gz = None
            elif spatial:
                gz = E.from_act(dz, z)
            else:
                gz = dz.view(z.shape).to(z.dtype)
            if skip is None:
                return gx, gz
            gs = E.from_act(dskip, skip) if dskip is not None else None
            return gx, gs, gz
        return run_block(self, fwd, bwd, inputs)


class _Reparam(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, logvar, eps):
        from . import kernels as K
        z = torch.empty_like(mu)
        K.call("vu_reparam_fwd", K.ptr(mu), K.ptr(logvar), K.ptr(eps), mu.numel(), K.ptr(z),
               K.stream())
        ctx.save_for_backward(logvar, eps)
        return z

    @staticmethod
    def backward(ctx, dz):
        from . import kernels as K
        logvar, eps = ctx.saved_tensors
        dz = dz.contiguous()
        dmu = torch.empty_like(dz)
        dlv = torch.empty_like(dz)
        K.call("vu_reparam_bwd", K.ptr(logvar), K.ptr(eps), K.ptr(dz), dz.numel(), K.ptr(dmu),
               K.ptr(dlv), 0, K.stream())
        return dmu, dlv, None


class UNetResNet(nn.Module):
    def __init__(self, n_channels, n_classes, backbone='resnet34', pretrained=True, latent_dim=32,
                 use_attention=True, use_skip=True, latent_injection='all'):
        super().__init__()
        if backbone != 'resnet34':
            raise NotImplementedError("only the reference's default backbone (resnet34) is built")
        if pretrained:
            warnings.warn("UNetResNet(pretrained=True): pretrained ResNet34 weights cannot be "
                          "downloaded here; keeping the random initialisation (load a "
                          "checkpoint with load_state_dict instead)")
        self.n_channels = n_channels
        self.n_classes = n_classes
        self.latent_dim = latent_dim
        self.latent_injection = latent_injection
        self.encoder = ResNet34Features(n_channels)
        ch = self.encoder.feature_info.channels()
        self.mu_head = nn.Sequential(nn.Conv2d(ch[-1], latent_dim, kernel_size=1), nn.AdaptiveAvgPool2d(1))
        self.logvar_head = nn.Sequential(nn.Conv2d(ch[-1], latent_dim, kernel_size=1),
                                         nn.AdaptiveAvgPool2d(1))
        self.z_initial = _cbr1x1(latent_dim, 512)
        modes = {'all': [True] * 4, 'inject_no_bottleneck': [True] * 4,
                 'first': [True, False, False, False], 'last': [False, False, False, True],
                 'bottleneck': [False] * 4, 'none': [False] * 4}
        if isinstance(latent_injection, list):
            use_latent = [i in latent_injection for i in range(4)]
        elif latent_injection in modes:
            use_latent = modes[latent_injection]
        else:
            use_latent = [True] * 4
            latent_injection = 'all'
            self.latent_injection = 'all'
        self.use_bottleneck = latent_injection not in ['none', 'inject_no_bottleneck']
        self.use_skip = use_skip
        self.use_attention = use_attention and use_skip
        self.decoder_blocks = nn.ModuleList([
            DecoderBlock(512, ch[-2], 512, latent_dim, use_attention, use_skip, use_latent[0]),
            DecoderBlock(512, ch[-3], 256, latent_dim, use_attention, use_skip, use_latent[1]),
            DecoderBlock(256, ch[-4], 128, latent_dim, use_attention, use_skip, use_latent[2]),
            DecoderBlock(128, ch[0], 64, latent_dim, use_attention, use_skip, use_latent[3]),
        ])
        self.final_conv = nn.Conv2d(64, n_classes, kernel_size=1)
        self.eps_override = None   # tests / reproducible sampling: fixed N(0,1) draw [B, L]
        self.grad_ready = None

    def reparameterize(self, mu, logvar):
        eps = torch.randn_like(mu)
        return _Reparam.apply(mu.float().contiguous(), logvar.float().contiguous(), eps)

    def _eps(self, B, device):
        if self.latent_injection in ('none', 'inject_no_bottleneck'):
            return None
        if self.eps_override is not None:
            return self.eps_override.to(device=device, dtype=torch.float32).reshape(B, -1).contiguous()
        return torch.randn((B, self.latent_dim), device=device)

    def forward(self, x):
        M = E.current_mode(x.device, self.grad_ready)
        E.refresh_weights(self.parameters())
        eps = self._eps(x.shape[0], x.device)
        if not isinstance(self.encoder, ResNet34Features):
            return self._forward_foreign_encoder(M, x, eps)
        params = [p for p in self.parameters() if p.requires_grad]
        if not (torch.is_grad_enabled() and (params or x.requires_grad)):
            out, mu, lv, _ = V.vae_fwd(M, self, x, eps)
            return out, mu, lv

        def fwd(inp):
            out, mu, lv, st = V.vae_fwd(M, self, inp[0], eps)
            return (out, mu, lv), st

        def bwd(state, douts):
            dout, dmu, dlv = douts
            V.vae_bwd(M, self, state, dout, dmu, dlv)
            return (None,)
        return BlockFn.apply(Runner(fwd, bwd), 1, x, *params)

    def _forward_foreign_encoder(self, M, x, eps):
        """``self.encoder`` replaced by any module returning the five feature
        maps (a timm ``features_only`` backbone, or a test double): it runs
        under torch autograd, everything after it (heads, reparameterize,
        bottleneck, decoder, final conv + resize) is the fused HIP tail."""
        feats = list(self.encoder(x))
        Hin, Win = x.shape[2], x.shape[3]
        params = [p for n, p in self.named_parameters() if not n.startswith("encoder.") and p.requires_grad]

        def fwd(inp):
            fa = [E.to_act(M, f) for f in inp]
            out, mu, lv, st = V.vae_tail_fwd(M, self, fa, Hin, Win, eps)
            return (out, mu, lv), st

        if not (torch.is_grad_enabled() and (params or any(f.requires_grad for f in feats))):
            return fwd(feats)[0]

        def bwd(state, douts):
            dfe = V.vae_tail_bwd(M, self, state, *douts)
            return tuple(E.from_act(d, f) if d is not None else None for d, f in zip(dfe, feats))
        return BlockFn.apply(Runner(fwd, bwd), len(feats), *feats, *params)

    def encode(self, x):
        M = E.current_mode(x.device)
        cp = (x.shape[1] + 7) // 8 * 8
        with torch.no_grad():
            feats, _ = V.encoder_fwd(M, self.encoder, E.to_act(M, x, cp), cp)
            f4 = feats[-1]
            pooled = V.sample_sum(M, f4, 1.0 / (f4.shape[2] * f4.shape[3]))
            outs = []
            for head in (self.mu_head[0], self.logvar_head[0]):
                o = torch.empty((x.shape[0], self.latent_dim), dtype=torch.float32, device=x.device)
                V.K.call("vu_linear_small_fwd", V.K.ptr(pooled), x.shape[0], f4.shape[1],
                         V.K.ptr(head.weight), V.K.ptr(head.bias), self.latent_dim, V.K.ptr(o),
                         V.K.stream())
                outs.append(o)
        return outs[0], outs[1]

    @torch.no_grad()
    def decode(self, z, input_size=None):
        """unet_resnet.py:250-279, including its quirk: skip features come from a
        512x512 all-zeros probe image, broadcast over the batch of z."""
        M = E.current_mode(z.device)
        B = z.shape[0]
        cp = (self.n_channels + 7) // 8 * 8
        probe = torch.zeros(1, self.n_channels, 512, 512, device=z.device)
        feats, _ = V.encoder_fwd(M, self.encoder, E.to_act(M, probe, cp), cp)
        feats = [f.expand(B, -1, -1, -1).contiguous(memory_format=torch.channels_last) for f in feats]
        zv = z.reshape(B, -1).float().contiguous()
        H4, W4 = feats[-1].shape[2], feats[-1].shape[3]
        if self.use_bottleneck:
            h, _ = V.cbr1x1_fwd(M, self.z_initial, V.latent_map(M, zv, B, H4, W4))
        else:
            h = M.zeros(B, 512, H4, W4)
        for i, blk in enumerate(self.decoder_blocks):
            skip = feats[-(i + 2)] if (i < len(feats) - 1 and self.use_skip) else None
            h, _ = V.decoder_fwd(M, blk, h, skip, zv)
        out, _ = E.outconv_fwd(M, self.final_conv, h)
        if input_size is not None:
            full = torch.empty((B, out.shape[1], input_size[0], input_size[1]), dtype=torch.float32,
                               device=z.device, memory_format=torch.channels_last)
            V.K.upsample_fwd(out, full, input_size[0], input_size[1], 0, 0, 0)
            out = full
        return out
