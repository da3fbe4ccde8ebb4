"""Model-level parity on the GPU, round 2:

* config 2 exactly as benchmarked (UNet(3,2), B=8, 3x512x512, bf16 autocast:
  the production conv3x3_pp / halo / wgrad3x3_halo dispatch) against the fp32
  CPU oracle, with the bf16 tolerances stated per assertion;
* the UNetResNet tail (heads, reparameterize, injection modes, DecoderBlocks,
  final conv + resize) against fixtures recorded from
  the reference's own UNetResNet class (fp64, fixed-feature encoder double);
* the reference's training-loop semantics: eval-mode forward after a step,
  grad accumulation x2 with GradScaler (train.py:401-411), eval-mode
  BatchNorm backward, F.pad with negative pads (crop), fp16 autocast,
  dice_score (utils/metrics.py:8-35).
"""
import warnings

import numpy as np
import pytest
import torch
import torch.nn as nn

from golden_util import (load, relerr, seed_vae_tail, vae_feature, vae_feature_shapes, vae_eps,
                         vae_target, state_of)

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


def _unet(nc, bil=False, seed=0):
    from vaeunet_amd import UNet
    from vaeunet_amd.init import seeded_init_
    return seeded_init_(UNet(3, nc, bilinear=bil), seed)


# ---------------------------------------------------------------------------
# config 2 (BASELINE configs[1]) at the benchmarked size and precision
# ---------------------------------------------------------------------------
# bf16 storage rounds every activation to 8 significant bits ~40 times between
# input and logits, and a randomly initialised BatchNorm/ReLU U-Net amplifies
# such perturbations with depth.  The yardstick is therefore the REFERENCE's
# own bf16 path (oracle/cpu_ref.py under torch.autocast("cpu", bfloat16):
# train.py's amp mode on CPU) against its fp32 path, on the same batch.  Stated
# tolerances for the HIP bf16 path against the fp32 oracle:
BF16_VS_REF_DRIFT = 1.5   # logit error (max and rms) <= 1.5 x the reference's own bf16 drift (+0.5 %)
BF16_LOSS = 1e-2          # |dloss| (north_star Dice+KL tolerance is 1e-3 in fp32)
BF16_GNORM = 5e-2         # per-parameter gradient norm, relative
BF16_TOTAL = 2e-2         # global gradient norm, relative
BF16_FLIPS = 1.5          # argmax flips <= 1.5 x the reference bf16 path's flips (+0.1 % of pixels)


def _drift(a, ref):
    d = (a - ref).abs()
    return d.max().item() / ref.abs().max().item(), (d.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt()).item()


@pytest.mark.timeout(600)
def test_unet_config2_bf16_b8_vs_oracle():
    from oracle import cpu_ref as R
    from vaeunet_amd.loss import CombinedLoss
    torch.set_num_threads(max(1, min(16, len(__import__("os").sched_getaffinity(0)))))
    model = _unet(2)
    state = model.state_dict()
    ref = R.UNetRef(state)
    g = torch.Generator().manual_seed(1000)   # bench.py synthetic(): rank 0
    x = torch.rand(8, 3, 512, 512, generator=g)
    m = (torch.rand(8, 1, 512, 512, generator=g) < 0.0085).float()
    t = torch.cat([1 - m, m], 1)
    xcl = x.contiguous(memory_format=CL)
    lref = ref.forward(xcl, True)
    loss_ref = R.combined_loss(lref.contiguous(), t)
    loss_ref.backward()
    names = [k for k, _ in model.named_parameters()]
    gref = np.array([float(ref.p[k].grad.double().norm()) for k in names])
    lref = lref.detach().contiguous()
    # the reference's own bf16 drift (CPU autocast), same weights and batch
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        lcpu16 = R.UNetRef(state).forward(xcl, True).float().contiguous()
    ref_max, ref_rms = _drift(lcpu16, lref)
    ref_flips = int((lcpu16.argmax(1) != lref.argmax(1)).sum())

    model = model.to(DEV).to(memory_format=CL).train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lg = model(x.to(DEV).contiguous(memory_format=CL))
        loss = CombinedLoss()(lg, t.to(DEV))
    loss.backward()
    lg = lg.detach().float().cpu().contiguous()
    max_rel, rms_rel = _drift(lg, lref)
    flips = int((lg.argmax(1) != lref.argmax(1)).sum())
    gn = np.array([float(p.grad.double().norm()) for p in model.parameters()])
    big = gref > 1e-3 * gref.max()
    grel = np.abs(gn - gref) / np.maximum(gref, 1e-30)
    worst = sorted(((grel[i], names[i]) for i in np.where(big)[0]), reverse=True)[:5]
    tot = abs(np.sqrt((gn ** 2).sum()) / np.sqrt((gref ** 2).sum()) - 1)
    npx = lg.shape[0] * lg.shape[2] * lg.shape[3]
    print(f"config2 bf16 B=8 vs fp32 oracle: HIP logits max_rel {max_rel:.3e} rms_rel {rms_rel:.3e} "
          f"flips {flips}/{npx}; reference CPU-bf16 max_rel {ref_max:.3e} rms_rel {ref_rms:.3e} "
          f"flips {ref_flips}; loss {loss.item():.6f} vs {loss_ref.item():.6f}; grad-norm worst "
          f"{[(round(float(a), 4), b) for a, b in worst[:3]]}; total {tot:.2e}")
    assert max_rel <= BF16_VS_REF_DRIFT * ref_max + 5e-3
    assert rms_rel <= BF16_VS_REF_DRIFT * ref_rms + 5e-3
    assert flips <= BF16_FLIPS * ref_flips + 1e-3 * npx
    assert abs(loss.item() - loss_ref.item()) < BF16_LOSS
    assert worst[0][0] < BF16_GNORM, worst
    assert tot < BF16_TOTAL


# ---------------------------------------------------------------------------
# UNetResNet tail vs the reference class (rows J/K/L/N)
# ---------------------------------------------------------------------------
class FixedFeatures(nn.Module):
    """Test double for the encoder: returns fixed leaf feature maps."""

    def __init__(self, feats):
        super().__init__()
        self.feats = feats

    def forward(self, x):
        return list(self.feats)


@pytest.mark.parametrize("mode", ["all", "none", "first", "bottleneck"])
def test_vae_tail_fp32_matches_reference(mode):
    from vaeunet_amd import UNetResNet
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    rec = load(f"vae_{mode}_256")
    B, S, seed = int(rec["B"]), int(rec["S"]), int(rec["seed"])
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        model = UNetResNet(3, 1, pretrained=False, latent_injection=mode)
    seed_vae_tail(model, seed)
    feats = [torch.from_numpy(vae_feature(sh, seed, i)).to(DEV).contiguous(memory_format=CL)
             .requires_grad_(True) for i, sh in enumerate(vae_feature_shapes(B, S))]
    model.encoder = FixedFeatures(feats)
    model = model.to(DEV).train()
    model.eps_override = torch.from_numpy(vae_eps(B, seed))
    out, mu, lv = model(torch.zeros(B, 3, S, S, device=DEV))
    t = torch.from_numpy(vae_target(B, S, seed)).to(DEV)
    loss = CombinedLoss()(out, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
    loss.backward()
    assert relerr(out.detach().cpu(), rec["out"]) < 1e-3
    assert relerr(mu.detach().cpu(), rec["mu"]) < 1e-4
    assert relerr(lv.detach().cpu(), rec["logvar"]) < 1e-4
    assert abs(loss.item() - float(rec["loss"])) < 1e-4
    params = dict(model.named_parameters())
    gn = np.array([float(params[str(k)].grad.double().norm()) if params[str(k)].grad is not None else 0.0
                   for k in rec["names"]])
    gr = rec["gnorm"]
    big = gr > 1e-3 * gr.max()
    # fp32 vs the fp64 reference: a ReLU whose input sits within rounding of
    # zero moves upstream gradients by up to a few % at this size (BatchNorm
    # over 2x8x8 bottleneck pixels); the total norm is held to 1 %
    bad = [(str(rec["names"][i]), gn[i], gr[i]) for i in np.where(big)[0] if abs(gn[i] - gr[i]) > 5e-2 * gr[i]]
    assert not bad, bad[:5]
    assert abs(np.sqrt((gn ** 2).sum()) - np.sqrt((gr ** 2).sum())) < 1e-2 * np.sqrt((gr ** 2).sum())
    for i, f in enumerate(feats):
        fg = float(f.grad.double().norm()) if f.grad is not None else 0.0
        assert abs(fg - rec["fgnorm"][i]) <= 2e-2 * rec["fgnorm"][i] + 1e-12, (i, fg, rec["fgnorm"][i])
    for k, b in model.named_buffers():
        if f"buf.{k}" in rec:
            assert relerr(b.cpu(), rec[f"buf.{k}"]) < 1e-3, k


def test_decoder_block_spatial_z_matches_reference():
    """DecoderBlock with a non-constant spatial z [B, L, h, w] (unet_resnet.py:93)."""
    from vaeunet_amd.unet_resnet import DecoderBlock
    rec = load("decoder_zspatial_64_32_48")
    mod = DecoderBlock(64, 32, 48, 8, True, True, True)
    mod.load_state_dict(state_of(rec), strict=False)
    mod = mod.to(DEV).train()
    ins = [torch.from_numpy(rec[f"in{i}"]).to(DEV).requires_grad_(True) for i in range(3)]
    out = mod(*ins)
    assert relerr(out.detach().cpu(), rec["out"]) < 1e-4
    out.backward(torch.from_numpy(rec["gout"]).to(DEV))
    for i, t in enumerate(ins):
        assert relerr(t.grad.cpu(), rec[f"gin{i}"]) < 2e-3, f"input grad {i}"
    gmax = max(float(np.abs(rec[f"grad.{k}"]).max()) for k, _ in mod.named_parameters())
    for k, p in mod.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), rec[f"grad.{k}"], rtol=2e-3,
                                   atol=2e-5 * gmax, err_msg=k)


# ---------------------------------------------------------------------------
# training-loop semantics of the reference
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("tag,nc,bil", [("unet_c1_64", 1, False), ("unet_c2_64", 2, False),
                                        ("unet_c1_bilinear_64", 1, True)])
def test_unet_eval_after_step_matches_reference(tag, nc, bil):
    """train step (fwd, loss, bwd, clip, AdamW) then model.eval() forward:
    the running-statistics path vs the reference's recorded eval_logits."""
    from vaeunet_amd.loss import CombinedLoss
    rec = load(tag)
    model = _unet(nc, bil).to(DEV).to(memory_format=CL).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    x = torch.from_numpy(rec["x"]).to(DEV).contiguous(memory_format=CL)
    logits = model(x)
    CombinedLoss()(logits, torch.from_numpy(rec["target"]).to(DEV)).backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt.step()
    model.eval()
    with torch.no_grad():
        ev = model(x)
    assert relerr(ev.cpu(), rec["eval_logits"]) < 1e-3


def test_grad_accumulation_gradscaler_matches_oracle():
    """train.py:394-411: loss/2 per micro-batch, scaler.scale(loss).backward()
    twice, then unscale_, clip_grad_norm_(1.0), scaler.step, update."""
    from oracle import cpu_ref as R
    from vaeunet_amd.loss import CombinedLoss
    model = _unet(1, seed=4)
    ref = R.UNetRef(model.state_dict())
    model = model.to(DEV).to(memory_format=CL).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 12)
    g = torch.Generator().manual_seed(21)
    batches = [(torch.rand(2, 3, 64, 64, generator=g), (torch.rand(2, 1, 64, 64, generator=g) < 0.05).float())
               for _ in range(2)]
    for x, t in batches:
        loss = CombinedLoss()(model(x.to(DEV).contiguous(memory_format=CL)), t.to(DEV)) / 2
        scaler.scale(loss).backward()
        lr_ = R.combined_loss(ref.forward(x, True), t) / 2
        lr_.backward()
        assert abs(loss.item() - lr_.item()) < 1e-3
    scaler.unscale_(opt)
    total = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    total_r = R.clip_grad_norm(list(ref.p.values()), 1.0)
    assert abs(total.item() - total_r.item()) < 2e-3 * total_r.item()
    names = [k for k, _ in model.named_parameters()]
    gn = np.array([float(p.grad.double().norm()) for p in model.parameters()])
    gr = np.array([float(ref.p[k].grad.double().norm()) for k in names])
    big = gr > 1e-3 * gr.max()
    np.testing.assert_allclose(gn[big], gr[big], rtol=1e-2)
    scaler.step(opt)
    scaler.update()
    assert scaler.get_scale() == 2.0 ** 12, "GradScaler saw inf/NaN gradients"
    for k, b in model.named_buffers():
        if "running" in k:
            assert relerr(b.cpu(), ref.bufs[k]) < 1e-3, k
        if k.endswith("num_batches_tracked"):
            assert int(b) == 2


def test_eval_mode_batchnorm_backward_matches_oracle():
    """Backward through eval-mode BatchNorm (running statistics as constants)."""
    from oracle import cpu_ref as R
    from vaeunet_amd import DoubleConv
    from vaeunet_amd.init import seeded_init_
    mod = seeded_init_(DoubleConv(8, 16), 5)
    gen = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for k, b in mod.named_buffers():
            if k.endswith("running_mean"):
                b.copy_(torch.randn(b.shape, generator=gen) * 0.3)
            elif k.endswith("running_var"):
                b.copy_(torch.rand(b.shape, generator=gen) + 0.5)
    st = mod.state_dict()
    p = {k: v.clone().requires_grad_(True) for k, v in st.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v.clone() for k, v in st.items() if "running" in k or "num_batches" in k}
    x = torch.rand(2, 8, 16, 16, generator=gen) - 0.5
    gout = torch.randn(2, 16, 16, 16, generator=gen)
    xr = x.clone().requires_grad_(True)
    yr = R.double_conv(xr, p, "double_conv.", bufs, False)
    yr.backward(gout)
    mod = mod.to(DEV).eval()
    xg = x.to(DEV).requires_grad_(True)
    y = mod(xg)
    y.backward(gout.to(DEV))
    assert relerr(y.detach().cpu(), yr.detach()) < 1e-4
    assert relerr(xg.grad.cpu(), xr.grad) < 1e-3
    for k, q in mod.named_parameters():
        assert relerr(q.grad.cpu(), p[k].grad) < 1e-3, k


@pytest.mark.parametrize("bil", [True, False])
def test_up_negative_pad_crops_like_reference(bil):
    """Up with an upsampled map larger than the skip: F.pad with negative
    pads crops (unet_parts.py:85-89)."""
    from oracle import cpu_ref as R
    from vaeunet_amd import Up
    from vaeunet_amd.init import seeded_init_
    mod = seeded_init_(Up(64, 32, bilinear=bil), 9)
    st = mod.state_dict()
    p = {k: v.clone().requires_grad_(True) for k, v in st.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v.clone() for k, v in st.items() if "running" in k or "num_batches" in k}
    gen = torch.Generator().manual_seed(9)
    x1 = torch.rand(2, 32 if bil else 64, 5, 5, generator=gen)
    x2 = torch.rand(2, 32, 9, 8, generator=gen)      # upsampled 10x10: pads (-1, -2)
    r1, r2 = x1.clone().requires_grad_(True), x2.clone().requires_grad_(True)
    yr = R.up(r1, r2, p, "", bufs, True, bil)
    gout = torch.randn(yr.shape, generator=gen)
    yr.backward(gout)
    g1, g2 = x1.to(DEV).requires_grad_(True), x2.to(DEV).requires_grad_(True)
    mod = mod.to(DEV).train()
    y = mod(g1, g2)
    y.backward(gout.to(DEV))
    assert relerr(y.detach().cpu(), yr.detach()) < 1e-4
    assert relerr(g1.grad.cpu(), r1.grad) < 2e-3
    assert relerr(g2.grad.cpu(), r2.grad) < 2e-3
    gmax = max(float(q.grad.abs().max()) for q in p.values())
    for k, q in mod.named_parameters():
        np.testing.assert_allclose(q.grad.cpu().numpy(), p[k].grad.numpy(), rtol=2e-3, atol=2e-5 * gmax,
                                   err_msg=k)


def test_fp16_autocast_runs_in_bf16_with_warning():
    """train.py:385's default autocast dtype is fp16: it runs (as bf16) and warns once."""
    from vaeunet_amd import engine
    from vaeunet_amd.loss import CombinedLoss
    engine._FP16_WARNED = False
    model = _unet(1).to(DEV).train()
    x = torch.rand(2, 3, 64, 64, device=DEV)
    t = (torch.rand(2, 1, 64, 64, device=DEV) < 0.05).float()
    with pytest.warns(UserWarning, match="float16 autocast"):
        with torch.autocast("cuda"):
            loss = CombinedLoss()(model(x), t)
    loss.backward()
    assert torch.isfinite(loss)
    assert all(torch.isfinite(p.grad).all() for p in model.parameters())


def test_dice_score_matches_reference():
    """utils/metrics.py:8-35 on the reference's recorded values (bit-exact),
    including the empty case (returns 1.0)."""
    from vaeunet_amd.metrics import dice_score, multiclass_dice_score, dice_loss
    rec = load("losses")
    for case in ("a", "b", "empty", "c2"):
        x = torch.from_numpy(rec[f"{case}.logits"]).to(DEV)
        t = torch.from_numpy(rec[f"{case}.target"]).to(DEV)
        got = dice_score(x, t)
        assert got.item() == float(rec[f"{case}.dice_score"]), case
        assert multiclass_dice_score(x, t).item() == got.item()
        assert abs(dice_loss(x, t).item() - (1 - got.item())) < 1e-7
    with pytest.raises(ValueError):
        dice_score(torch.zeros(2, 1, 4, 4, device=DEV), torch.zeros(2, 1, 4, 5, device=DEV))
