"""Pin the CPU oracle (oracle/cpu_ref.py) to the reference's own outputs.

The fixtures in tests/golden were produced by running the reference modules
(/root/reference) in the build container (oracle/gen_golden.py).  If these
tests pass, the oracle is a faithful restatement and can stand in for the
reference on the GPU box, where the reference does not exist.
"""
import numpy as np
import pytest
import torch

from golden_util import (load, state_of, relerr, seed_vae_tail, vae_feature, vae_feature_shapes,
                         vae_eps, vae_target)
from oracle import cpu_ref as R

torch.set_num_threads(8)

BLOCKS = {
    "doubleconv_8_16": lambda i, p, b: R.double_conv(i[0], p, "double_conv.", b, True),
    "doubleconv_3_16_mid8": lambda i, p, b: R.double_conv(i[0], p, "double_conv.", b, True),
    "down_16_32": lambda i, p, b: R.down(i[0], p, "", b, True),
    "down_odd_16_32": lambda i, p, b: R.down(i[0], p, "", b, True),
    "up_64_32_convT": lambda i, p, b: R.up(i[0], i[1], p, "", b, True, False),
    "up_64_32_bilinear": lambda i, p, b: R.up(i[0], i[1], p, "", b, True, True),
    "up_odd_64_32_convT": lambda i, p, b: R.up(i[0], i[1], p, "", b, True, False),
    "up_odd_64_32_bilinear": lambda i, p, b: R.up(i[0], i[1], p, "", b, True, True),
    "attention_32_32_16": lambda i, p, b: R.attention_gate(i[0], i[1], p, "", b, True),
    "outconv_16_2": lambda i, p, b: R.out_conv(i[0], p, ""),
    "decoder_64_32_48": lambda i, p, b: R.decoder_block(i[0], i[1], i[2], p, "", b, True),
    "decoder_noattn_64_32_48": lambda i, p, b: R.decoder_block(
        i[0], i[1], i[2], p, "", b, True, use_attention=False, use_latent=False),
    "decoder_zspatial_64_32_48": lambda i, p, b: R.decoder_block(i[0], i[1], i[2], p, "", b, True),
}


def _split_state(rec):
    st = state_of(rec)
    params = {k: v.clone().requires_grad_(True) for k, v in st.items()
              if "running" not in k}
    bufs = {k: v.clone() for k, v in st.items() if "running" in k}
    for k in list(bufs):
        if k.endswith("running_mean"):
            bufs[k[: -len("running_mean")] + "num_batches_tracked"] = torch.tensor(0)
    return params, bufs


@pytest.mark.parametrize("name", sorted(BLOCKS))
def test_block_matches_reference(name):
    rec = load(name)
    params, bufs = _split_state(rec)
    n_in = len([k for k in rec if k.startswith("in")])
    ins = [torch.from_numpy(rec[f"in{i}"]).clone().requires_grad_(True) for i in range(n_in)]
    out = BLOCKS[name](ins, params, bufs)
    assert relerr(out.detach(), rec["out"]) < 2e-5
    out.backward(torch.from_numpy(rec["gout"]))
    for i, t in enumerate(ins):
        g = t.grad if t.grad is not None else torch.zeros_like(t)
        # the latent input z of DecoderBlock gathers a 64-pixel broadcast sum
        # through BatchNorm: fp32 summation-order noise reaches ~5e-4 there
        assert relerr(g, rec[f"gin{i}"]) < 2e-3, f"input grad {i}"
    # biases feeding a BatchNorm have a mathematically-zero gradient (~1e-7
    # rounding noise): tolerance is relative to the block's largest gradient
    gmax = max(float(np.abs(rec[f"grad.{k}"]).max()) for k in params)
    for k, p in params.items():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        ref = rec[f"grad.{k}"]
        np.testing.assert_allclose(g.numpy(), ref, rtol=1e-3, atol=1e-5 * gmax, err_msg=k)
    for k, v in bufs.items():
        key = f"buf.{k}"
        if key in rec:
            assert relerr(v, rec[key]) < 1e-5, k


def test_losses_match_reference():
    rec = load("losses")
    for case in ("a", "b", "empty", "c2"):
        x = torch.from_numpy(rec[f"{case}.logits"]).requires_grad_(True)
        t = torch.from_numpy(rec[f"{case}.target"])
        loss = R.combined_loss(x, t)
        loss.backward()
        assert abs(float(loss) - float(rec[f"{case}.loss"])) < 1e-6
        assert relerr(x.grad, rec[f"{case}.grad"]) < 1e-5
        assert abs(float(R.dice_loss(x.detach(), t)) - float(rec[f"{case}.dice_loss"])) < 1e-6
        assert abs(float(R.dice_score(x.detach(), t)) - float(rec[f"{case}.dice_score"])) < 1e-6
    mu, lv = rec["kl.mu"], rec["kl.logvar"]
    for fb in (1e-3, 1e-4, 0.0, 0.5):
        m = torch.from_numpy(mu).clone().requires_grad_(True)
        v = torch.from_numpy(lv).clone().requires_grad_(True)
        kl = R.kl_with_free_bits(m, v, fb)
        kl.backward()
        tag = f"kl_fb{fb:g}"
        assert abs(float(kl) - float(rec[f"{tag}.value"])) <= 1e-6 * max(1, abs(float(kl)))
        np.testing.assert_allclose(m.grad.numpy(), rec[f"{tag}.gmu"], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(v.grad.numpy(), rec[f"{tag}.glogvar"], rtol=1e-6, atol=1e-7)
    w = [R.kl_weight(e, 0.0, 1e-3, 20) for e in range(25)]
    np.testing.assert_allclose(w, rec["annealer"], rtol=1e-12)


def _unet_state(n_classes, bilinear):
    from vaeunet_amd.unet_model import UNet
    from vaeunet_amd.init import seeded_init_
    m = seeded_init_(UNet(3, n_classes, bilinear=bilinear), 0)
    return m.state_dict()


@pytest.mark.parametrize("tag,nc,bil", [("unet_c1_64", 1, False), ("unet_c2_64", 2, False),
                                        ("unet_c1_bilinear_64", 1, True)])
def test_unet_train_step_matches_reference(tag, nc, bil):
    rec = load(tag)
    state = _unet_state(nc, bil)
    names = [k for k in state if "running" not in k and "num_batches" not in k]
    assert names == list(rec["names"]), "state_dict keys differ from the reference"
    model = R.UNetRef(state, bilinear=bil)
    opt = R.AdamW(model.p.values(), lr=1e-4, weight_decay=1e-5)
    x = torch.from_numpy(rec["x"])
    t = torch.from_numpy(rec["target"])
    logits, loss, total = R.train_step(model, opt, x, t)
    assert relerr(logits, rec["logits"]) < 1e-4
    if nc > 1:
        np.testing.assert_array_equal(logits.argmax(1).numpy(), rec["argmax"])
    assert abs(float(loss) - float(rec["loss"])) < 1e-5
    # fp32 summation order (oneDNN algorithm choice, channels_last vs NCHW)
    # moves the pre-clip gradient norm by ~1e-4 relative
    assert abs(float(total) - float(rec["total_norm"])) < 1e-3 * float(rec["total_norm"])
    heads = np.stack([np.pad(p.detach().reshape(-1)[:16].numpy(), (0, 16 - min(16, p.numel())))
                      for p in model.p.values()])
    # AdamW's first step moves every element by ~lr*sign(g): where the
    # gradient is at rounding-noise level (biases in front of a BatchNorm,
    # |g| < 1e-5) the sign is noise, so those elements get a 2*lr tolerance.
    noisy = np.abs(rec["ghead"]) < 1e-5
    d = np.abs(heads - rec["p1head"])
    assert d[~noisy].max() < 1e-6 + 1e-4 * np.abs(rec["p1head"][~noisy]).max()
    assert d[noisy].max() <= 2.05e-4
    for k, v in model.bufs.items():
        if f"buf.{k}" in rec:
            assert relerr(v, rec[f"buf.{k}"]) < 1e-4, k
    with torch.no_grad():
        ev = model.forward(x, train=False)
    # after the update (noise-sign Adam steps above), eval-mode logits: 1e-3
    assert relerr(ev, rec["eval_logits"]) < 1e-3


def vae_tail_params(mode, seed):
    """Seeded UNetResNet tail parameters keyed like the reference state_dict
    (the vaeunet_amd module is used only as a CPU parameter holder)."""
    from vaeunet_amd import UNetResNet
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        m = UNetResNet(3, 1, pretrained=False, latent_injection=mode)
    seed_vae_tail(m, seed)
    return {k: v for k, v in m.state_dict().items() if not k.startswith("encoder.")}


@pytest.mark.parametrize("mode", ["all", "none", "first", "bottleneck"])
def test_vae_tail_matches_reference(mode):
    """UNetResNet after the encoder (unet_resnet.py:203-240; rows J/K/L/N) vs the
    reference's own class run in fp64 with a fixed-feature encoder double."""
    rec = load(f"vae_{mode}_256")
    B, S, seed = int(rec["B"]), int(rec["S"]), int(rec["seed"])
    st = vae_tail_params(mode, seed)
    p = {k: v.double().requires_grad_(True) for k, v in st.items()
         if "running" not in k and "num_batches" not in k}
    bufs = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in st.items()
            if "running" in k or "num_batches" in k}
    feats = [torch.from_numpy(vae_feature(sh, seed, i)).double().requires_grad_(True)
             for i, sh in enumerate(vae_feature_shapes(B, S))]
    eps = torch.from_numpy(vae_eps(B, seed)).double()
    t = torch.from_numpy(vae_target(B, S, seed)).double()
    out, mu, lv = R.unet_resnet_tail(feats, (S, S), p, bufs, eps=eps, latent_injection=mode)
    loss = R.combined_loss(out, t) + 1e-3 * R.kl_with_free_bits(mu, lv, 1e-3)
    loss.backward()
    assert relerr(out.detach(), rec["out"]) < 1e-5
    assert relerr(mu.detach(), rec["mu"]) < 1e-9
    assert relerr(lv.detach(), rec["logvar"]) < 1e-9
    assert abs(loss.item() - float(rec["loss"])) < 1e-9
    for k, gn in zip(rec["names"], rec["gnorm"]):
        g = p[str(k)].grad
        mine = float(g.norm()) if g is not None else 0.0
        assert abs(mine - gn) <= 1e-6 * max(gn, 1e-12) + 1e-12, k
    for i, f in enumerate(feats):
        mine = float(f.grad.norm()) if f.grad is not None else 0.0
        assert abs(mine - rec["fgnorm"][i]) <= 1e-6 * max(rec["fgnorm"][i], 1e-12) + 1e-12, i
    for k, v in bufs.items():
        if f"buf.{k}" in rec:
            assert relerr(v, rec[f"buf.{k}"]) < 1e-9, k
