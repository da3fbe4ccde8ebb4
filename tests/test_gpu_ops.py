"""torch.ops.vaeunet.* on the GPU: each op vs a plain PyTorch fp32 reference
of the same op, autograd through the registered formulas, and
torch.library.opcheck (schema, fake-tensor, autograd registration, AOT
dispatch).  Shapes are small; fp32 storage (parity mode) unless noted."""
import pytest
import torch
import torch.nn.functional as F

from vaeunet_amd import ops  # noqa: F401  (registers the ops)

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last
v = torch.ops.vaeunet


def _act(t, dtype=torch.float32):
    return t.to(DEV, dtype).contiguous(memory_format=CL)


def _close(got, ref, rtol, what):
    got, ref = got.detach().float().cpu(), ref.detach().float().cpu()
    err = (got - ref).abs().max().item()
    scale = max(ref.abs().max().item(), 1e-3)
    assert err <= rtol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("dtype,rtol", [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
def test_conv3x3_ops_vs_torch(dtype, rtol):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 16, 20, 24, generator=g)
    w = torch.randn(32, 16, 3, 3, generator=g) * 0.1
    b = torch.randn(32, generator=g)
    dy = torch.randn(2, 32, 20, 24, generator=g)
    xr = x.to(dtype).float()
    wr, dyr = w, dy.to(dtype).float()
    _close(v.conv3x3_fwd(_act(x, dtype), w.to(DEV), b.to(DEV)), F.conv2d(xr, wr, b, padding=1), rtol, "fwd")
    _close(v.conv3x3_dgrad(_act(dy, dtype), w.to(DEV)), F.conv_transpose2d(dyr, wr, padding=1), rtol, "dgrad")
    xg = xr.clone().requires_grad_(True)
    wg = wr.clone().requires_grad_(True)
    F.conv2d(xg, wg, padding=1).backward(dyr)
    _close(v.conv3x3_wgrad(_act(x, dtype), _act(dy, dtype)), wg.grad, rtol, "wgrad")


def test_conv3x3_autograd():
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 8, 16, 16, generator=g)
    w = torch.randn(16, 8, 3, 3, generator=g) * 0.2
    b = torch.randn(16, generator=g)
    xd = _act(x).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    bd = b.to(DEV).requires_grad_(True)
    (v.conv3x3_fwd(xd, wd, bd) ** 2).sum().backward()
    xr, wr, br = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    (F.conv2d(xr, wr, br, padding=1) ** 2).sum().backward()
    for got, ref, n in ((xd.grad, xr.grad, "dx"), (wd.grad, wr.grad, "dw"), (bd.grad, br.grad, "db")):
        _close(got, ref, 1e-4, n)


def test_conv_bn_relu_and_backward_vs_torch():
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 16, 16, 12, generator=g)
    w = torch.randn(24, 16, 3, 3, generator=g) * 0.1
    gamma = torch.rand(24, generator=g) + 0.5
    beta = torch.randn(24, generator=g)
    rm, rv = torch.zeros(24), torch.ones(24)
    xd = _act(x).requires_grad_(True)
    wd, gd, bd = (t.to(DEV).requires_grad_(True) for t in (w, gamma, beta))
    a, y, coef, rm_new, rv_new = v.conv_bn_relu(xd, wd, gd, bd, rm.to(DEV), rv.to(DEV), 0.1, 1e-5)
    da = torch.randn(a.shape, generator=g)
    a.backward(_act(da))
    xr, wr, gr, br = (t.clone().requires_grad_(True) for t in (x, w, gamma, beta))
    rmr, rvr = rm.clone(), rv.clone()
    ar = F.relu(F.batch_norm(F.conv2d(xr, wr, padding=1), rmr, rvr, gr, br, True, 0.1, 1e-5))
    ar.backward(da)
    _close(a, ar, 1e-4, "a")
    _close(rm_new, rmr, 1e-5, "running_mean")
    _close(rv_new, rvr, 1e-5, "running_var")
    for got, ref, n in ((xd.grad, xr.grad, "dx"), (wd.grad, wr.grad, "dw"), (gd.grad, gr.grad, "dgamma"),
                        (bd.grad, br.grad, "dbeta")):
        _close(got, ref, 2e-4, n)


def test_maxpool_ops():
    g = torch.Generator().manual_seed(8)
    x = torch.randn(2, 8, 14, 10, generator=g)
    xd = _act(x).requires_grad_(True)
    y = v.maxpool2d(xd)
    dy = torch.randn(y.shape, generator=g)
    y.backward(_act(dy))
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 2)
    yr.backward(dy)
    assert torch.equal(y.detach().cpu(), yr.detach())
    assert torch.equal(xd.grad.cpu(), xr.grad)


def test_bce_dice_loss_op():
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 1, 32, 32, generator=g)
    t = (torch.rand(2, 1, 32, 32, generator=g) < 0.2).float()
    xd = x.to(DEV).requires_grad_(True)
    loss, _ = v.bce_dice_loss(xd, t.to(DEV), 1.0, 0.5, 0.5)
    loss.backward()
    xr = x.clone().requires_grad_(True)
    p = torch.sigmoid(xr)
    dice = 1 - (2 * (p * t).sum() + 1) / (p.sum() + t.sum() + 1)
    ref = 0.5 * F.binary_cross_entropy_with_logits(xr, t) + 0.5 * dice
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-5
    _close(xd.grad, xr.grad, 1e-4, "dloss")


def test_opcheck():
    g = torch.Generator().manual_seed(10)
    x = _act(torch.randn(2, 8, 8, 8, generator=g))
    w = (torch.randn(8, 8, 3, 3, generator=g) * 0.1).to(DEV)
    gamma, beta = torch.ones(8, device=DEV), torch.zeros(8, device=DEV)
    rm, rv = torch.zeros(8, device=DEV), torch.ones(8, device=DEV)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    cases = [
        (v.conv3x3_fwd.default, (xr, wr, None)),
        (v.conv3x3_dgrad.default, (x, w)),
        (v.conv3x3_wgrad.default, (x, x)),
        (v.conv_bn_relu.default, (xr, wr, gamma, beta, rm, rv, 0.1, 1e-5)),
        (v.maxpool2d.default, (xr,)),
    ]
    for op, args in cases:
        torch.library.opcheck(op, args, test_utils=("test_schema", "test_faketensor",
                                                    "test_autograd_registration"))
