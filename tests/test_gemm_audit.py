"""CPU checks of the per-element GEMM audit (tests/gemm_audit.py) itself:
launches emulated with torch ops of the semantics include/vaeunet.h states
must pass it, and a wrong element or a write outside the output region must
be caught.  (The audit is the checker of test_gpu_production_parity.py.)"""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from gemm_audit import GemmAudit

CL = torch.channels_last


class _CpuAudit(GemmAudit):
    @staticmethod
    def kernel_of(a, dtype):
        return -1


def _lib():
    from vaeunet_amd import _lib as L
    return L


def _act(t, dt=torch.bfloat16):
    return t.to(dt).contiguous(memory_format=CL)


def _fwd_args(g, wmat, ncol, out, coff=0, bias=None, acc=False, convT=None):
    L = _lib()
    a = L.VuGemmFwd()
    a.a = g
    a.b = wmat.data_ptr()
    a.ldb = wmat.shape[-1]
    a.ncol = ncol
    a.out_coff = coff
    a.accumulate = 1 if acc else 0
    a.relu = 0
    if convT is not None:
        a.out_mode = 1
        a.oH, a.oW, a.opy, a.opx, a.cout = convT
    else:
        a.out_mode = 0
    return a


def _conv3x3_case(perturb=None):
    from vaeunet_amd import kernels as K
    g_ = torch.Generator().manual_seed(3)
    x1 = _act(torch.randn(2, 16, 9, 12, generator=g_))
    x2 = _act(torch.randn(2, 8, 9, 12, generator=g_))
    w = torch.randn(24, 24, 3, 3, generator=g_) / 12
    wmat = w.to(torch.bfloat16).permute(0, 2, 3, 1).reshape(24, -1).contiguous()
    bias = torch.randn(24, generator=g_)
    out = _act(torch.randn(2, 40, 9, 12, generator=g_))
    g = K.gather3x3([x1, x2])
    a = _fwd_args(g, wmat, 24, out, coff=8, bias=bias, acc=True)
    audit = _CpuAudit(strict=False)

    def launch():
        ref = F.conv2d(torch.cat([x1, x2], 1).float(), wmat.float().view(24, 3, 3, 24).permute(0, 3, 1, 2),
                       bias, padding=1)
        new = (out[:, 8:32].float() + ref.to(torch.bfloat16).float()).to(torch.bfloat16)
        out[:, 8:32] = new
        if perturb == "value":
            out[1, 20, 4, 5] = out[1, 20, 4, 5].float() * 1.05 + 0.1
        elif perturb == "outside":
            out[0, 3, 0, 0] = 7.0
    audit.gemm_fwd(a, 1, g, wmat, out, bias, None, launch)
    return audit.records[0]


def test_audit_accepts_a_correct_3x3_launch():
    r = _conv3x3_case()
    assert r["off"] == 0 and r["untouched"] and r["worst"] < 1.0, r


@pytest.mark.parametrize("what", ["value", "outside"])
def test_audit_catches_a_wrong_launch(what):
    r = _conv3x3_case(what)
    if what == "value":
        assert r["off"] == 1, r
    else:
        assert not r["untouched"], r


def test_audit_convT_pixel_shuffle_with_pad_offset():
    from vaeunet_amd import kernels as K
    g_ = torch.Generator().manual_seed(4)
    x = _act(torch.randn(2, 16, 4, 5, generator=g_))
    w = torch.randn(16, 8, 2, 2, generator=g_) / 4
    b = torch.randn(8, generator=g_)
    wmat = w.to(torch.bfloat16).permute(2, 3, 1, 0).reshape(32, 16).contiguous()
    out = _act(torch.zeros(2, 8, 9, 11))
    g = K.gather1x1([x])
    a = _fwd_args(g, wmat, 32, out, bias=b, convT=(9, 11, 0, 1, 8))
    audit = _CpuAudit(strict=False)

    def launch():
        y = F.conv_transpose2d(x.float(), w.to(torch.bfloat16).float(), b, stride=2)
        out[:, :, 0:8, 1:11] = y.to(torch.bfloat16)
    audit.gemm_fwd(a, 1, g, wmat, out, b, None, launch)
    r = audit.records[0]
    assert r["off"] == 0 and r["untouched"], r


@pytest.mark.parametrize("acc", [False, True])
def test_audit_wgrad_3x3_with_padded_channels(acc):
    from vaeunet_amd import kernels as K
    L = _lib()
    g_ = torch.Generator().manual_seed(5)
    x = torch.randn(2, 16, 8, 10, generator=g_)
    x[:, 13:] = 0                       # 3 zero-padded input channels (cvalid = 13)
    x = _act(x)
    dy = _act(torch.randn(2, 12, 8, 10, generator=g_))
    grad = torch.randn(12, 13, 3, 3, generator=g_) if acc else torch.zeros(12, 13, 3, 3)
    from vaeunet_amd import engine as E
    layout = E.conv_layout(grad)
    gp, gq = K.gather1x1([dy]), K.gather3x3([x])
    w = L.VuGemmWgrad()
    audit = _CpuAudit(strict=False)

    def launch():
        ref = torch.nn.grad.conv2d_weight(x.float()[:, :13], (12, 13, 3, 3), dy.float(), padding=1)
        if acc:
            grad.add_(ref)
        else:
            grad.copy_(ref)
    audit.gemm_wgrad(w, 1, 3, gp, gq, 12, 9 * 16, grad, layout, acc, 13, launch)
    r = audit.records[0]
    assert r["off"] == 0 and r["untouched"], r
