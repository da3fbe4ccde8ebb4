"""Inference sampling path (vaeunet_amd/inference.py)
against fixtures recorded from the reference's own functions
(utils/vae_utils.py generate_predictions / encode_images, visualize_vae.py
predict_full_image / predict_with_patches / calculate_uncertainty_metrics;
oracle/gen_golden.py gen_inference) on the same UNetResNet weights, eval-mode
BatchNorm statistics and encoder test double; fp32 parity mode.
"""
import warnings

import pytest
import torch

from golden_util import (load, relerr, seed_vae_tail, seed_bn_stats, pyramid_encoder, infer_inputs,
                         INFER_SEED, INFER_GEN, INFER_PATCH)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model():
    from vaeunet_amd import UNetResNet
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        m = UNetResNet(3, 1, pretrained=False, latent_injection="all")
    seed_vae_tail(m, INFER_SEED)
    seed_bn_stats(m, INFER_SEED + 50)
    m.encoder = pyramid_encoder(INFER_SEED)
    return m.to(DEV).eval()


@pytest.fixture(scope="module")
def setup():
    return _model(), load("inference"), {k: torch.from_numpy(v) for k, v in infer_inputs().items()}


def test_encode_and_generate_predictions(setup):
    from vaeunet_amd import inference as I
    model, rec, inp = setup
    mu, lv = I.encode_images(model, inp["gen_images"].to(DEV))
    assert relerr(mu.cpu(), rec["enc_mu"]) < 1e-4
    assert relerr(lv.cpu(), rec["enc_logvar"]) < 1e-4
    pred = I.generate_predictions(model, inp["gen_images"].to(DEV), temperature=INFER_GEN["temperature"],
                                  num_samples=INFER_GEN["samples"], eps=inp["gen_eps"].to(DEV))
    assert pred.shape == rec["gen_out"].shape
    assert relerr(pred.cpu(), rec["gen_out"]) < 1e-3


def test_predict_full_image(setup):
    from vaeunet_amd import inference as I
    model, rec, inp = setup
    out = I.predict_full_image(model, inp["full_img"].to(DEV), inp["full_z"].to(DEV))
    assert out.shape == rec["full_out"].shape
    assert relerr(out.cpu(), rec["full_out"]) < 1e-4


def test_predict_with_patches(setup):
    from vaeunet_amd import inference as I
    model, rec, inp = setup
    out = I.predict_with_patches(model, inp["patch_img"].to(DEV), inp["patch_z"].to(DEV),
                                 INFER_PATCH["patch"], None, INFER_PATCH["batch"])
    assert out.shape == rec["patch_out"].shape
    assert relerr(out.cpu(), rec["patch_out"]) < 1e-4


def test_uncertainty_metrics(setup):
    from vaeunet_amd import inference as I
    _, rec, inp = setup
    got = I.calculate_uncertainty_metrics(inp["segs"].to(DEV))
    for k in ("mean", "std", "entropy", "mutual_info", "coeff_var"):
        assert got[k].shape == rec[f"unc_{k}"].shape, k
        assert relerr(got[k].cpu(), rec[f"unc_{k}"]) < 1e-5, k


def test_batched_sampling_equals_per_sample(setup):
    """segmentation_distribution decodes draws in batched passes (encoder once);
    each draw must equal the reference-style one-draw-at-a-time prediction."""
    from vaeunet_amd import inference as I
    model, _, inp = setup
    img = inp["full_img"].to(DEV)
    eps = torch.randn(5, 1, 32, generator=torch.Generator().manual_seed(3)).to(DEV)
    segs, mu, lv = I.segmentation_distribution(model, img, num_samples=5, temperature=0.8, eps=eps,
                                               sample_batch=3)
    for k in range(5):
        z = (mu + eps[k] * 0.8 * torch.exp(0.5 * lv)).view(1, -1, 1, 1)
        one = I.predict_full_image(model, img, z)
        assert relerr(segs[k:k + 1].cpu(), one.cpu()) < 1e-5, k
    pimg = inp["patch_img"].to(DEV)
    segs, mu, lv = I.segmentation_distribution(model, pimg, num_samples=2, patch_size=64, eps=eps[:2],
                                               batch_size=4)
    for k in range(2):
        z = (mu + eps[k] * torch.exp(0.5 * lv)).view(1, -1, 1, 1)
        one = I.predict_with_patches(model, pimg, z, 64, None, 4)
        assert relerr(segs[k:k + 1].cpu(), one.cpu()) < 1e-5, k
