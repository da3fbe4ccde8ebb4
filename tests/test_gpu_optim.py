"""Optimizer tail (train.py:406-411): vaeunet_amd.optim.clip_grad_norm_ and
FusedAdamW against torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW (the
reference's own calls) on the same parameters and gradients."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 3, 3, 3), (64,), (128, 64, 3, 3), (32, 64, 1, 1), (1,), (2, 64, 1, 1), (9000,)]
    ps = []
    for i, s in enumerate(shapes):
        t = torch.randn(s, generator=g)
        if len(s) == 4 and i % 2 == 0:
            t = t.contiguous(memory_format=torch.channels_last)
        ps.append(t)
    return ps


def _grads(ps, seed, scale):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(p.shape, generator=g) * scale for p in ps]


@pytest.mark.parametrize("max_norm,scale", [(1.0, 1.0), (1.0, 1e-4), (0.5, 3.0)])
def test_clip_grad_norm_matches_torch(max_norm, scale):
    from vaeunet_amd.optim import clip_grad_norm_
    ps = _params(0)
    gs = _grads(ps, 1, scale)
    a = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    b = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    for pa, pb, g in zip(a, b, gs):
        pa.grad = g.to(DEV).contiguous(memory_format=torch.preserve_format)
        pb.grad = g.to(DEV)
    n_ref = torch.nn.utils.clip_grad_norm_(a, max_norm, foreach=True)
    n_got = clip_grad_norm_(b, max_norm)
    assert n_got.device.type == "cuda"
    torch.testing.assert_close(n_got.cpu(), n_ref.cpu(), rtol=1e-6, atol=0)
    for pa, pb in zip(a, b):
        torch.testing.assert_close(pb.grad.cpu(), pa.grad.cpu(), rtol=2e-6, atol=1e-12)


def test_fused_adamw_matches_torch_adamw():
    """Three steps (bias corrections change), lr 1e-4 / wd 1e-5 as in train.py,
    clip before each step; state_dict moves between the two optimizers."""
    from vaeunet_amd.optim import FusedAdamW, clip_grad_norm_
    ps = _params(3)
    a = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    b = [torch.nn.Parameter(p.to(DEV)) for p in ps]
    oa = torch.optim.AdamW(a, lr=1e-4, weight_decay=1e-5, foreach=True)
    ob = FusedAdamW(b, lr=1e-4, weight_decay=1e-5)
    for it in range(3):
        gs = _grads(ps, 10 + it, 0.3)
        for pa, pb, g in zip(a, b, gs):
            pa.grad = g.to(DEV)
            pb.grad = g.to(DEV)
        torch.nn.utils.clip_grad_norm_(a, 1.0, foreach=True)
        clip_grad_norm_(b, 1.0)
        oa.step()
        ob.step()
        for pa, pb in zip(a, b):
            # one fp32 rounding of difference per op at most (fma contraction)
            torch.testing.assert_close(pb.detach().cpu(), pa.detach().cpu(), rtol=1e-6, atol=1e-9)
    sa, sb = oa.state_dict(), ob.state_dict()
    assert sa["param_groups"][0]["lr"] == sb["param_groups"][0]["lr"]
    for k in sa["state"]:
        assert float(sa["state"][k]["step"]) == float(sb["state"][k]["step"]) == 3.0
        for name in ("exp_avg", "exp_avg_sq"):
            want, got = sa["state"][k][name].cpu(), sb["state"][k][name].cpu()
            # moments that nearly cancel carry the ulp-level differences of
            # their inputs (clip coefficient, fma contraction) at a few 1e-5
            # relative: bound the error by the tensor's scale
            torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-6 * float(want.abs().max()))
    # torch AdamW state loads into FusedAdamW and continues identically
    oc = FusedAdamW([torch.nn.Parameter(p.detach().clone()) for p in a], lr=1e-4, weight_decay=1e-5)
    oc.load_state_dict(sa)
    assert float(oc.state_dict()["state"][0]["step"]) == 3.0


def test_fused_optimizer_training_loop_matches_torch():
    """End to end: UNet train steps with FusedAdamW + fused clip give the same
    losses as with torch's AdamW + clip, i.e. the in-place HIP update is seen
    by the next forward (derived bf16/fp32 weight layouts are invalidated)."""
    from vaeunet_amd import UNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss
    from vaeunet_amd.optim import FusedAdamW, clip_grad_norm_
    g = torch.Generator().manual_seed(4)
    x = torch.rand(2, 3, 64, 64, generator=g).to(DEV)
    t = (torch.rand(2, 1, 64, 64, generator=g) < 0.1).float().to(DEV)
    losses = {}
    for kind in ("torch", "fused"):
        model = seeded_init_(UNet(3, 1), 0).to(DEV).train()
        if kind == "torch":
            opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5, foreach=True)
            clip = lambda ps: torch.nn.utils.clip_grad_norm_(ps, 1.0, foreach=True)  # noqa: E731
        else:
            opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
            clip = lambda ps: clip_grad_norm_(ps, 1.0)  # noqa: E731
        crit = CombinedLoss()
        out = []
        for _ in range(4):
            loss = crit(model(x), t)
            loss.backward()
            clip(model.parameters())
            opt.step()
            opt.zero_grad(set_to_none=True)
            out.append(float(loss))
        losses[kind] = out
    # step 0 is bitwise the same forward; afterwards ulp-level differences
    # (fp64 vs fp32 clip norm, fma contraction) pass through Adam's
    # sign-like first updates: a stale-weight bug would repeat loss 0 instead
    assert losses["torch"][0] == losses["fused"][0]
    for a, b in zip(losses["torch"][1:], losses["fused"][1:]):
        assert abs(a - b) < 2e-4 * max(1.0, abs(a)), losses
    assert losses["fused"][3] != losses["fused"][0]
