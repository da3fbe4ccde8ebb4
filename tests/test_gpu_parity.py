"""Module-level parity on the GPU: the drop-in modules (fp32 parity mode)
against the reference's own golden fixtures, and against the CPU oracle at
larger sizes; bf16 (autocast) mode against the fp32 oracle with the
tolerances stated per test.
"""
import numpy as np
import pytest
import torch

from golden_util import load, state_of, relerr

pytestmark = pytest.mark.gpu
DEV = "cuda"

BLOCKS = {
    "doubleconv_8_16": ("DoubleConv", (8, 16)),
    "doubleconv_3_16_mid8": ("DoubleConv", (3, 16, 8)),
    "down_16_32": ("Down", (16, 32)),
    "down_odd_16_32": ("Down", (16, 32)),
    "up_64_32_convT": ("Up", (64, 32, False)),
    "up_64_32_bilinear": ("Up", (64, 32, True)),
    "up_odd_64_32_convT": ("Up", (64, 32, False)),
    "up_odd_64_32_bilinear": ("Up", (64, 32, True)),
    "attention_32_32_16": ("AttentionGate", (32, 32, 16)),
    "outconv_16_2": ("OutConv", (16, 2)),
}


def _build(name):
    import vaeunet_amd.unet_parts as P
    cls, args = BLOCKS[name]
    return getattr(P, cls)(*args)


@pytest.mark.parametrize("name", sorted(BLOCKS))
def test_block_fp32_matches_reference(name):
    rec = load(name)
    mod = _build(name)
    st = state_of(rec)
    missing = mod.load_state_dict(st, strict=False)
    assert not missing.unexpected_keys
    assert all("num_batches" in k for k in missing.missing_keys)
    mod = mod.to(DEV).train()
    n_in = len([k for k in rec if k.startswith("in")])
    ins = [torch.from_numpy(rec[f"in{i}"]).to(DEV).requires_grad_(True) for i in range(n_in)]
    out = mod(*ins)
    assert out.dtype == torch.float32
    assert relerr(out.detach().cpu(), rec["out"]) < 1e-4
    out.backward(torch.from_numpy(rec["gout"]).to(DEV))
    for i, t in enumerate(ins):
        assert relerr(t.grad.cpu(), rec[f"gin{i}"]) < 2e-3, f"input grad {i}"
    gmax = max(float(np.abs(rec[f"grad.{k}"]).max()) for k, _ in mod.named_parameters())
    for k, p in mod.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), rec[f"grad.{k}"], rtol=2e-3,
                                   atol=2e-5 * gmax, err_msg=k)
    for k, b in mod.named_buffers():
        if f"buf.{k}" in rec:
            assert relerr(b.cpu(), rec[f"buf.{k}"]) < 1e-4, k
        if k.endswith("num_batches_tracked"):
            assert int(b) == 1


def _unet(nc, bil):
    from vaeunet_amd import UNet
    from vaeunet_amd.init import seeded_init_
    return seeded_init_(UNet(3, nc, bilinear=bil), 0)


@pytest.mark.parametrize("tag,nc,bil", [("unet_c1_64", 1, False), ("unet_c2_64", 2, False),
                                        ("unet_c1_bilinear_64", 1, True)])
def test_unet_train_step_fp32_matches_reference(tag, nc, bil):
    """train.py:381-411 (tiny config) with the HIP path in fp32 parity mode."""
    from vaeunet_amd.loss import CombinedLoss
    rec = load(tag)
    model = _unet(nc, bil).to(DEV).to(memory_format=torch.channels_last).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    x = torch.from_numpy(rec["x"]).to(DEV).contiguous(memory_format=torch.channels_last)
    t = torch.from_numpy(rec["target"]).to(DEV)
    logits = model(x)
    loss = CombinedLoss()(logits, t)
    loss.backward()
    lg = logits.detach().cpu()
    # per-pixel logits within 1e-3 (north_star), class maps bit-exact
    assert relerr(lg, rec["logits"]) < 1e-3
    if nc > 1:
        np.testing.assert_array_equal(lg.argmax(1).numpy(), rec["argmax"])
    else:
        np.testing.assert_array_equal((lg > 0).numpy(), rec["argmax"])
    assert abs(loss.item() - float(rec["loss"])) < 1e-3
    gn = np.array([float(p.grad.double().norm()) for p in model.parameters()])
    big = rec["gnorm"] > 1e-3 * rec["gnorm"].max()
    np.testing.assert_allclose(gn[big], rec["gnorm"][big], rtol=1e-2)
    total = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    assert abs(total.item() - float(rec["total_norm"])) < 2e-3 * float(rec["total_norm"])
    opt.step()
    for k, b in model.named_buffers():
        if f"buf.{k}" in rec:
            assert relerr(b.cpu(), rec[f"buf.{k}"]) < 1e-3, k


def test_unet_bf16_autocast_vs_oracle():
    """Speed mode (autocast -> bf16 storage, fp32 accumulation) vs the fp32
    oracle: logits within 5e-2 relative, loss within 1e-2."""
    from vaeunet_amd.loss import CombinedLoss
    from oracle import cpu_ref as R
    rec = load("unet_c1_64")
    model = _unet(1, False).to(DEV).train()
    x = torch.from_numpy(rec["x"]).to(DEV)
    t = torch.from_numpy(rec["target"]).to(DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        logits = model(x)
        loss = CombinedLoss()(logits, t)
    loss.backward()
    assert relerr(logits.detach().float().cpu(), rec["logits"]) < 5e-2
    assert abs(loss.item() - float(rec["loss"])) < 1e-2
    for p in model.parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all()


def test_unet_512_fp32_vs_oracle():
    """Full-resolution case (3x512x512, B=1) against the CPU oracle: logits
    within 1e-3, loss within 1e-3, class map bit-exact except for flips the
    fp64 oracle adjudicates as fp32 near-ties (golden_util.adjudicate_flips)."""
    from vaeunet_amd.loss import CombinedLoss
    from oracle import cpu_ref as R
    from golden_util import adjudicate_flips, class_margin
    torch.manual_seed(0)
    model = _unet(2, False)
    state = model.state_dict()
    ref = R.UNetRef(state)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(1, 3, 512, 512, generator=g)
    m = (torch.rand(1, 1, 512, 512, generator=g) < 0.0085).float()
    t = torch.cat([1 - m, m], 1)
    with torch.no_grad():
        lref = ref.forward(x, True)
        p64 = {k: v.detach().double() for k, v in ref.p.items()}
        b64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in state.items()
               if "running" in k or "num_batches" in k}
        l64 = R.unet_forward(x.double(), p64, b64, True)
    loss_ref = R.combined_loss(lref, t)
    model = model.to(DEV).to(memory_format=torch.channels_last).train()
    lg = model(x.to(DEV).contiguous(memory_format=torch.channels_last))
    loss = CombinedLoss()(lg, t.to(DEV))
    lgc = lg.detach().cpu()
    assert relerr(lgc, lref.detach()) < 1e-3
    adjudicate_flips("unet 512 B=1 fp32", class_margin(lgc).double(), class_margin(lref).double(),
                     class_margin(l64))
    assert abs(loss.item() - loss_ref.item()) < 1e-3


DEC = {"decoder_64_32_48": (64, 32, 48, 8, True, True, True),
       "decoder_noattn_64_32_48": (64, 32, 48, 8, False, True, False)}


@pytest.mark.parametrize("name", sorted(DEC))
def test_decoder_block_fp32_matches_reference(name):
    """DecoderBlock (unet_resnet.py:31-101) vs the reference's own outputs."""
    from vaeunet_amd.unet_resnet import DecoderBlock
    rec = load(name)
    mod = DecoderBlock(*DEC[name])
    mod.load_state_dict(state_of(rec), strict=False)
    mod = mod.to(DEV).train()
    ins = [torch.from_numpy(rec[f"in{i}"]).to(DEV).requires_grad_(True) for i in range(3)]
    out = mod(*ins)
    assert relerr(out.detach().cpu(), rec["out"]) < 1e-4
    out.backward(torch.from_numpy(rec["gout"]).to(DEV))
    for i, t in enumerate(ins):
        g = t.grad.cpu() if t.grad is not None else torch.zeros_like(t).cpu()
        assert relerr(g, rec[f"gin{i}"]) < 2e-3, f"input grad {i}"
    gmax = max(float(np.abs(rec[f"grad.{k}"]).max()) for k, _ in mod.named_parameters())
    for k, p in mod.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), rec[f"grad.{k}"], rtol=2e-3,
                                   atol=2e-5 * gmax, err_msg=k)


@pytest.mark.parametrize("mode", ["all", "none", "first"])
def test_unet_resnet_fp32_vs_oracle(mode):
    """VAE-U-Net train step (recon + beta*KL) vs the CPU oracle with the same
    eps draw.  The ResNet34 encoder is a restatement (timm absent): parity
    here is against the oracle's restatement, i.e. unpinned by the reference."""
    from vaeunet_amd import UNetResNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    from oracle import cpu_ref as R
    torch.manual_seed(0)
    model = seeded_init_(UNetResNet(3, 1, pretrained=False, latent_injection=mode), 3)
    st = model.state_dict()
    # At small sizes the backward is ill-conditioned: a single ReLU whose
    # pre-activation sits within fp32 rounding of zero flips between fp32 and
    # fp64 and moves every upstream gradient (measured: one flipped element of
    # a 2x512x8x8 decoder activation moves all upstream grads by 0.5 %; at
    # 128x128 input, seed-dependent total-norm moves of 0.1-1.0 %; at 64x64 two
    # fp32 CPU runs differing only in thread count differ by 1.6 %).  The test
    # runs at 256x256 (8x8 bottleneck) with the oracle in fp64 (dtype-generic).
    p = {k: v.clone().double().requires_grad_(True) for k, v in st.items()
         if "running" not in k and "num_batches" not in k}
    bufs = {k: (v.clone().double() if v.is_floating_point() else v.clone())
            for k, v in st.items() if "running" in k or "num_batches" in k}
    g = torch.Generator().manual_seed(11)
    x = torch.rand(2, 3, 256, 256, generator=g)
    t = (torch.rand(2, 1, 256, 256, generator=g) < 0.05).float()
    eps = torch.randn(2, 32, generator=g)
    out_r, mu_r, lv_r = R.unet_resnet_forward(x.double(), p, bufs, eps=eps.double(),
                                             latent_injection=mode)
    loss_r = R.combined_loss(out_r, t.double()) + 1e-3 * R.kl_with_free_bits(mu_r, lv_r, 1e-3)
    loss_r.backward()
    out_r, mu_r, lv_r = out_r.float(), mu_r.float(), lv_r.float()
    model = model.to(DEV).train()
    model.eps_override = eps
    out, mu, lv = model(x.to(DEV))
    loss = CombinedLoss()(out, t.to(DEV)) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
    loss.backward()
    assert relerr(out.detach().cpu(), out_r.detach()) < 1e-3
    assert relerr(mu.detach().cpu(), mu_r.detach()) < 1e-3
    assert relerr(lv.detach().cpu(), lv_r.detach()) < 1e-3
    assert abs(loss.item() - loss_r.item()) < 1e-3
    names = [k for k, _ in model.named_parameters()]
    gn = np.array([float(q.grad.double().norm()) if q.grad is not None else 0.0
                   for q in model.parameters()])
    gr = np.array([float(p[k].grad.double().norm()) if p[k].grad is not None else 0.0
                   for k in names])
    big = gr > 1e-3 * gr.max()
    bad = [(names[i], gn[i], gr[i]) for i in np.where(big)[0]
           if abs(gn[i] - gr[i]) > 5e-2 * gr[i]]
    # the decoder's first attention gate normalises psi over only 32 pixels
    # at this size (BatchNorm2d(1) of a 16x16 map, B=2): its W_g gradient is
    # ill-conditioned and moves a few % with fp32 summation order; the total
    # gradient norm is held to 1%
    assert abs(np.sqrt((gn ** 2).sum()) - np.sqrt((gr ** 2).sum())) < 1e-2 * np.sqrt((gr ** 2).sum())
    assert not bad, bad[:5]
    for k, b in model.named_buffers():
        if "running" in k:
            assert relerr(b.cpu(), bufs[k]) < 1e-3, k


def test_unet_resnet_bf16_512_runs():
    """config 3 shape (3x512x512, bf16 autocast) runs and gives finite grads."""
    from vaeunet_amd import UNetResNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    model = seeded_init_(UNetResNet(3, 1, pretrained=False), 0).to(DEV).train()
    x = torch.rand(2, 3, 512, 512, device=DEV)
    t = (torch.rand(2, 1, 512, 512, device=DEV) < 0.01).float()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out, mu, lv = model(x)
        loss = CombinedLoss()(out, t) + 1e-3 * kl_with_free_bits(mu, lv, 1e-3)
    loss.backward()
    assert out.shape == (2, 1, 512, 512) and mu.shape == (2, 32)
    assert torch.isfinite(loss)
    assert all(q.grad is not None and torch.isfinite(q.grad).all() for q in model.parameters())
