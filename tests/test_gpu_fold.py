"""Eval-mode BatchNorm folded into the convolutions for inference
(engine.fold_bn_eval + the GEMM epilogue ReLU, VuGemmFwd.relu): a no-grad
eval forward with folding vs without (conv, then the separate BN + ReLU
pass), fp32 and bf16, both model families (unet_parts.py:32-49 DoubleConv,
unet_resnet.py BasicBlock / stem / z_initial; the inference path of
visualize_vae.py:61-87,578-652)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _randomise_bn(model, g):
    # non-trivial running statistics and affine parameters
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            with torch.no_grad():
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.2)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.num_features, generator=g) * 0.1)


def _run(model, x, fold, bf16):
    from vaeunet_amd import engine as E
    old = E.FOLD_BN_EVAL
    E.FOLD_BN_EVAL = fold
    try:
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            out = model(x)
        torch.cuda.synchronize()
    finally:
        E.FOLD_BN_EVAL = old
    return out if isinstance(out, tuple) else (out,)


@pytest.mark.parametrize("bf16,batch", [(False, 2), (True, 2), (True, 8)])
@pytest.mark.parametrize("family", ["unet", "vae"])
def test_eval_bn_folding_matches_unfolded(family, bf16, batch):
    """batch 8 at 512^2 puts the VAE decoder blocks' conv1 (latent shortcut
    table + folded BN + ReLU) on the ping-pong kernel."""
    from vaeunet_amd import UNet, UNetResNet
    from vaeunet_amd.init import seeded_init_
    g = torch.Generator().manual_seed(3)
    if family == "unet":
        model = UNet(3, 2)
        x = torch.randn(batch, 3, 128, 128, generator=g)
    else:
        model = UNetResNet(3, 1, pretrained=False)
        x = torch.randn(batch, 3, 512, 512, generator=g)
    model = seeded_init_(model, 0)
    _randomise_bn(model, g)
    model = model.to(DEV).to(memory_format=torch.channels_last).eval()
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    if family == "vae":
        torch.manual_seed(0)
    a = _run(model, xd, True, bf16)
    if family == "vae":
        torch.manual_seed(0)
    b = _run(model, xd, False, bf16)
    for u, v in zip(a, b):
        u, v = u.float(), v.float()
        scale = v.abs().max().item() + 1e-6
        err = (u - v).abs().max().item()
        # fp32: rounding of the folded weights / summation order; bf16: the
        # unfolded path rounds the conv output to bf16 BEFORE the BN affine,
        # the folded one does not (one bf16 rounding fewer per layer)
        tol = 1e-4 if not bf16 else 6e-2
        assert err <= tol * scale, (family, bf16, err, scale)
