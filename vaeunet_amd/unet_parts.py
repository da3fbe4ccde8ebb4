"""U-Net building blocks (drop-in for the reference's unet/unet_parts.py).

Same class names, constructor signatures, attribute trees and state_dict keys
as unet_parts.py:7-103, so reference checkpoints load unchanged and code that
reaches into submodules (``.double_conv``, ``.maxpool_conv``, ``.up``,
``.conv``, ``.attention``, ``.psi`` hooks) keeps working.  The submodules are
parameter holders: ``forward`` runs the fused HIP sequences of engine.py
instead of one ATen call per submodule.
"""
import torch
import torch.nn as nn

from . import engine as E
from .functional import run_block, act_grad


def _cbr(cin, cout):
    """conv3x3(pad 1, no bias) -> BatchNorm2d -> ReLU, as three Sequential slots."""
    return [nn.Conv2d(cin, cout, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(cout), nn.ReLU(inplace=True)]


def _conv_bn(cin, cout, k=1):
    return nn.Sequential(nn.Conv2d(cin, cout, kernel_size=k), nn.BatchNorm2d(cout))


def _pad8(c):
    return (c + 7) // 8 * 8


class AttentionGate(nn.Module):
    """x * sigmoid(BN(psi(relu(BN(W_g g) + BN(W_x x)))))  (unet_parts.py:7-30)."""

    def __init__(self, F_g, F_l, F_int):
        super().__init__()
        self.W_g = _conv_bn(F_g, F_int)
        self.W_x = _conv_bn(F_l, F_int)
        self.psi = nn.Sequential(nn.Conv2d(F_int, 1, kernel_size=1), nn.BatchNorm2d(1), nn.Sigmoid())
        self.relu = nn.ReLU(inplace=True)

    def forward(self, g, x):
        M = E.current_mode(x.device)

        def fwd(inp):
            ga, xa = E.to_act(M, inp[0]), E.to_act(M, inp[1])
            out, st = E.attention_fwd(M, self, ga, xa)
            return out, (st, ga)

        def bwd(state, dout):
            st, ga = state
            dg = M.zeros(*ga.shape)
            dx = E.attention_bwd(M, self, st, act_grad(M, dout), (dg, 0), True)
            return E.from_act(dg, g), E.from_act(dx, x)
        return run_block(self, fwd, bwd, (g, x))


class DoubleConv(nn.Module):
    """(convolution => [BN] => ReLU) * 2  (unet_parts.py:32-49)."""

    def __init__(self, in_channels, out_channels, mid_channels=None):
        super().__init__()
        mid = mid_channels if mid_channels else out_channels
        self.double_conv = nn.Sequential(*_cbr(in_channels, mid), *_cbr(mid, out_channels))

    def forward(self, x):
        M = E.current_mode(x.device)
        cin = x.shape[1]
        cp = _pad8(cin)

        def fwd(inp):
            xa = E.to_act(M, inp[0], cp)
            return E.double_conv_fwd(M, self.double_conv, [xa], cin_pad=cp)

        def bwd(state, dout):
            dx = E.double_conv_bwd(M, self.double_conv, state, act_grad(M, dout),
                                   x.requires_grad, cvalid=cin)
            return (E.from_act(dx, x) if dx is not None else None,)
        return run_block(self, fwd, bwd, (x,))


class Down(nn.Module):
    """Downscaling with maxpool then double conv  (unet_parts.py:51-63)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), DoubleConv(in_channels, out_channels))

    def forward(self, x):
        M = E.current_mode(x.device)

        def fwd(inp):
            return E.down_fwd(M, self, E.to_act(M, inp[0]))[1:]

        def bwd(state, dout):
            # a standalone Down has no producing BN to hand the pooled gradient to
            return (E.from_act(E.down_bwd(M, self, state, act_grad(M, dout)).materialize(M), x),)
        return run_block(self, fwd, bwd, (x,))


class Up(nn.Module):
    """Upscaling (+pad) -> attention gate -> concat -> double conv  (unet_parts.py:65-95)."""

    def __init__(self, in_channels, out_channels, bilinear=True):
        super().__init__()
        if bilinear:
            self.up = nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True)
            self.conv = DoubleConv(in_channels, out_channels, in_channels // 2)
        else:
            self.up = nn.ConvTranspose2d(in_channels, in_channels // 2, kernel_size=2, stride=2)
            self.conv = DoubleConv(in_channels, out_channels)
        self.attention = AttentionGate(F_g=in_channels // 2, F_l=in_channels // 2,
                                       F_int=in_channels // 4)

    def forward(self, x1, x2):
        M = E.current_mode(x1.device)

        def fwd(inp):
            return E.up_fwd(M, self, E.to_act(M, inp[0]), E.to_act(M, inp[1]))

        def bwd(state, dout):
            dx1, dx2 = E.up_bwd(M, self, state, act_grad(M, dout))
            return E.from_act(dx1, x1), E.from_act(dx2, x2)
        return run_block(self, fwd, bwd, (x1, x2))


class OutConv(nn.Module):
    """1x1 conv to class logits  (unet_parts.py:97-103)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=1)

    def forward(self, x):
        M = E.current_mode(x.device)

        def fwd(inp):
            return E.outconv_fwd(M, self.conv, E.to_act(M, inp[0]))

        def bwd(state, dout):
            return (E.from_act(E.outconv_bwd(M, self.conv, state, dout), x),)
        return run_block(self, fwd, bwd, (x,))
