"""Per-element parity of the BENCHMARKED bf16 GEMM kernels at production size.

One training micro-step (forward, CombinedLoss [+ 1e-3 KL], backward) of
config 2 (UNet(3,2)) and config 3 (UNetResNet(3,1), ResNet34 encoder) at
B=8, 3x512x512 under bf16 autocast, with the DEFAULT dispatch (no tuning
override), is run with ``kernels.AUDIT`` installed (tests/gemm_audit.py):
every 3x3 / 1x1 / ConvTranspose / stem / image-conv forward, input-gradient
and weight-gradient launch of the step -- the v6 full-grid persistent walk,
the v4 ping-pong tiles incl. the automatic split-K at 32x32, v7 on the
encoder levels, the halo weight gradients with their production split-K and
slab-reduce geometry, the stream / v5 short-K GEMMs, the image conv, the stem
-- is compared element by element with the fp64 contraction of the same
bf16 operands (the convolution of the bf16-rounded activations and weights),
under the bound

  |got - exp| <= 2^-8 max(|exp|, |got|) + c * sum_k |a_k b_k| (+ floor),

and must leave every element outside its output region untouched.  A second
backward accumulates into the existing .grad buffers (train.py's gradient
accumulation), so the accumulating epilogues are audited too.

Reference ops: unet/unet_parts.py:40,43 (3x3), :11,15 (attention 1x1), :76
(ConvTranspose2d); unet/unet_resnet.py:131-137 (ResNet34 encoder), :59-69
(DecoderBlock convs), :150-154 (z_initial), :93-94 (z_proj).
"""
import pytest
import torch

from gemm_audit import GemmAudit

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last
B, S = 8, 512


def _batch(classes):
    g = torch.Generator().manual_seed(1000)   # bench.py synthetic(): rank 0
    x = torch.rand(B, 3, S, S, generator=g)
    m = (torch.rand(B, 1, S, S, generator=g) < 0.0085).float()
    t = torch.cat([1 - m, m], 1) if classes == 2 else m
    return x.to(DEV).contiguous(memory_format=CL), t.to(DEV)


def _run(model, step, micro_steps=2):
    from vaeunet_amd import kernels as K
    audit = GemmAudit(strict=False)
    K.AUDIT = audit
    try:
        for _ in range(micro_steps):
            step(model)
        torch.cuda.synchronize()
    finally:
        K.AUDIT = None
    print("\n" + audit.summary())
    bad = [r for r in audit.records if r["off"] or not r["untouched"]]
    assert not bad, bad[:5]
    return audit


def _kernels(audit, op):
    return {r["kernel"] for r in audit.records if r["op"] == op}


@pytest.mark.timeout(900)
def test_unet_config2_every_gemm_per_element():
    from vaeunet_amd import UNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss
    torch.manual_seed(0)
    model = seeded_init_(UNet(3, 2), 0).to(DEV).to(memory_format=CL).train()
    x, t = _batch(2)
    crit = CombinedLoss()

    def step(m):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = crit(m(x), t)
        loss.backward()
    audit = _run(model, step)
    fwd = [r for r in audit.records if r["op"] == "fwd"]
    wg = [r for r in audit.records if r["op"] == "wgrad"]
    # 2 micro-steps x (18 fwd + 17 dgrad 3x3, 4 ConvT fwd + dgrad, 8 attention
    # 1x1 fwd + 8 dgrad) / (18 3x3 + 4 ConvT + 8 1x1 weight gradients)
    assert len(fwd) >= 2 * (18 + 17 + 8 + 16), len(fwd)
    assert len(wg) >= 2 * (18 + 4 + 8), len(wg)
    # the benchmarked kernels are the ones audited: image conv (9), v6 resident
    # weights (6), v4 ping-pong incl. split-K (4), 1x1 streams (8), halo wgrad (3)
    assert {9, 6, 4, 8} <= _kernels(audit, "fwd"), _kernels(audit, "fwd")
    assert 3 in _kernels(audit, "wgrad"), _kernels(audit, "wgrad")
    assert 1 not in _kernels(audit, "fwd") and 1 not in _kernels(audit, "wgrad"), audit.summary()
    assert any(r["acc"] for r in wg) and any(r["acc"] for r in fwd)


@pytest.mark.timeout(900)
def test_unetresnet_config3_every_gemm_per_element():
    from vaeunet_amd import UNetResNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    torch.manual_seed(0)
    model = seeded_init_(UNetResNet(3, 1, pretrained=False), 0).to(DEV).to(memory_format=CL).train()
    model.eps_override = torch.randn(B, 32, generator=torch.Generator().manual_seed(77)).to(DEV)
    x, t = _batch(1)
    crit = CombinedLoss()

    def step(m):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, mu, lv = m(x)
            loss = crit(lg, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
        loss.backward()
    audit = _run(model, step)
    # stem (10), v7 small-grid encoder levels (7), v4 / v6 decoder levels
    assert {10, 7} <= _kernels(audit, "fwd"), _kernels(audit, "fwd")
    assert 3 in _kernels(audit, "wgrad"), _kernels(audit, "wgrad")
    # no launch of a bf16 step falls to the generic register-staged kernels
    assert 1 not in _kernels(audit, "fwd") and 1 not in _kernels(audit, "wgrad"), audit.summary()
