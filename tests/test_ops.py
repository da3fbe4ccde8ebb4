"""torch.ops.vaeunet.* (SURVEY.md §8(b) dispatcher ops), CPU side: the schemas
are registered, shape propagation works on meta tensors (the fake impls that
torch.compile / FakeTensorMode use), and a CPU tensor is refused (no CPU
fallback).  Numerics and opcheck run on the GPU (tests/test_gpu_ops.py)."""
import pytest
import torch

from vaeunet_amd import ops

CL = torch.channels_last


def _m(*shape, dtype=torch.bfloat16, cl=True):
    t = torch.empty(shape, device="meta", dtype=dtype)
    return t.contiguous(memory_format=CL) if cl else t


def test_ops_registered():
    for n in ops.OPS:
        op = getattr(torch.ops.vaeunet, n).default
        assert op._schema.name == f"vaeunet::{n}"


def test_meta_shapes():
    v = torch.ops.vaeunet
    x, w = _m(2, 16, 12, 10), _m(32, 16, 3, 3, dtype=torch.float32, cl=False)
    y = v.conv3x3_fwd(x, w)
    assert y.shape == (2, 32, 12, 10) and y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=CL)
    assert v.conv3x3_dgrad(_m(2, 32, 12, 10), w).shape == (2, 16, 12, 10)
    dw = v.conv3x3_wgrad(x, _m(2, 32, 12, 10))
    assert dw.shape == (32, 16, 3, 3) and dw.dtype == torch.float32
    g = _m(32, dtype=torch.float32, cl=False)
    a, y2, coef, rm, rv = v.conv_bn_relu(x, w, g, g, g, g, 0.1, 1e-5)
    assert a.shape == y2.shape == (2, 32, 12, 10) and coef.shape == (4, 32) and rm.shape == rv.shape == (32,)
    dy, dg, db = v.bn_relu_backward(a, y2, coef, g, True)
    assert dy.shape == y2.shape and dg.shape == db.shape == (32,)
    assert v.maxpool2d(_m(2, 16, 13, 10)).shape == (2, 16, 6, 5)
    assert v.maxpool2d_backward(x, _m(2, 16, 6, 5)).shape == x.shape
    loss, sums = v.bce_dice_loss(_m(2, 1, 8, 8, dtype=torch.float32), _m(2, 1, 8, 8, dtype=torch.float32),
                                 1.0, 0.5, 0.5)
    assert loss.shape == () and sums.shape == (4,) and sums.dtype == torch.float64


def test_cpu_tensors_refused():
    x = torch.randn(1, 8, 4, 4).contiguous(memory_format=CL)
    w = torch.randn(8, 8, 3, 3)
    with pytest.raises((NotImplementedError, RuntimeError)):
        torch.ops.vaeunet.conv3x3_fwd(x, w)
