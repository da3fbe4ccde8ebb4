"""The latent vector path (vae_engine.LATENT_VECTORS, csrc/latent.hip) against
the round-3 map path on the same model, batch and latent draw: the VAE
bottleneck heads, reparameterize, z_initial and every DecoderBlock z_proj
(unet/unet_resnet.py:140-154, 191-194, 217-229, 37-41, 93-94) computed on the
[N, L] sample vectors must give the same logits / mu / logvar, the same
gradient of every parameter and the same BatchNorm running statistics as the
1x1 conv + BatchNorm + ReLU over the broadcast maps (fp32: to summation-order
noise; bf16: within the storage rounding the map path adds), for each latent
injection mode, in train and eval mode -- with the DecoderBlock latent
shortcut (vae_engine.LATENT_SHORTCUT, csrc/zbias.hip: the z part of conv1
as a per-sample border-class bias) and without it (the vector path writing
the maps)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


def _model(inj, seed=0):
    from vaeunet_amd import UNetResNet
    from vaeunet_amd.init import seeded_init_
    torch.manual_seed(seed)
    m = seeded_init_(UNetResNet(3, 1, pretrained=False, latent_injection=inj), seed)
    return m.to(DEV).to(memory_format=CL)


def _run(model, x, t, eps, vec, bf16, train=True, steps=1, shortcut=True):
    from vaeunet_amd import vae_engine as V
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    old, old_sc = V.LATENT_VECTORS, V.LATENT_SHORTCUT
    V.LATENT_VECTORS = vec
    V.LATENT_SHORTCUT = shortcut
    try:
        model.train(train)
        model.eps_override = eps
        outs = []
        for _ in range(steps):
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                lg, mu, lv = model(x)
                loss = CombinedLoss()(lg, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
            if train:
                loss.backward()
            outs.append((lg.detach().float(), mu.detach().float(), lv.detach().float(), float(loss.detach())))
        torch.cuda.synchronize()
    finally:
        V.LATENT_VECTORS = old
        V.LATENT_SHORTCUT = old_sc
    return outs


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-20))


def _oracle64(model, x, t, eps, inj):
    """fp64 gradients of the same train-mode micro-step on the CPU oracle, and
    sigma: per BatchNorm-affine gradient, the spread ||t32 - t64|| of its
    reduction terms (dz, dz * xhat) between the fp32 and fp64 oracle -- the
    error a sum of those terms has from the fp32 per-term error alone
    (tests/test_gpu_config_parity.py; the attention psi BatchNorm(1) sums are
    ill-conditioned, sum |dz| / |sum dz| up to ~1e3-1e4)."""
    from oracle import cpu_ref as R
    st = model.state_dict()
    sampling = inj not in ("none", "inject_no_bottleneck")

    def run(dt):
        p = {k: v.detach().cpu().to(dt).requires_grad_(True) for k, v in st.items()
             if "running" not in k and "num_batches" not in k}
        b = {k: (v.detach().cpu().to(dt) if v.is_floating_point() else v.detach().cpu().clone())
             for k, v in st.items() if "running" in k or "num_batches" in k}
        R.PROBE = {}
        try:
            lg, mu, lv = R.unet_resnet_forward(x.cpu().to(dt), p, b, eps=eps.cpu().to(dt) if sampling else None,
                                               latent_injection=inj)
            loss = R.combined_loss(lg, t.cpu().to(dt)) + 1e-3 * R.kl_with_free_bits(mu, lv, 1e-3)
            loss.backward()
            terms = {}
            for pre, v in R.PROBE.items():
                if not pre.startswith("gate:"):
                    xh, y = v
                    terms[pre + "bias"] = y.grad.detach().double()
                    terms[pre + "weight"] = (y.grad * xh).detach().double()
        finally:
            R.PROBE = None
        return {k: v.grad for k, v in p.items() if v.grad is not None}, terms
    g64, t64 = run(torch.float64)
    g32, t32 = run(torch.float32)
    sigma = {k: float((t32[k] - t64[k]).norm()) for k in t64 if k in t32}
    return g64, sigma, g32


@pytest.mark.parametrize("inj", ["all", "first", "bottleneck", "none", "inject_no_bottleneck"])
@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("sc", [True, False])
def test_latent_vector_path_matches_map_path(inj, bf16, sc):
    """Both paths against the fp64 oracle (one micro-step): every parameter
    gradient of the vector path is at least as close to fp64 as the map
    path's (within a factor), forward outputs and BatchNorm running
    statistics agree; a second micro-step (gradient accumulation) agrees."""
    torch.manual_seed(1)
    B, S = 4, 128
    x = torch.rand(B, 3, S, S, device=DEV).contiguous(memory_format=CL)
    t = (torch.rand(B, 1, S, S, device=DEV) < 0.05).float()
    eps = torch.randn(B, 32, device=DEV)
    a = _model(inj)
    b = copy.deepcopy(a)
    g64, sigma, g32 = _oracle64(a, x, t, eps, inj)
    ra = _run(a, x, t, eps, True, bf16, steps=1, shortcut=sc)
    rb = _run(b, x, t, eps, False, bf16, steps=1)
    tol = 3e-2 if bf16 else 1e-4
    for (la, ma, va, lsa), (lb, mb, vb, lsb) in zip(ra, rb):
        assert _rel(la, lb) < tol, (_rel(la, lb), tol)
        assert _rel(ma, mb) < tol and _rel(va, vb) < tol
        assert abs(lsa - lsb) < (1e-2 if bf16 else 1e-5)
    pa, pb = dict(a.named_parameters()), dict(b.named_parameters())
    gmax = max(float(g.norm()) for g in g64.values())
    fac, floor = (1.5, 2e-3) if bf16 else (2.0, 1e-6)
    worst, bound = [], {}
    for k, ref in g64.items():
        ga, gb = pa[k].grad, pb[k].grad
        da = float((ga.double().cpu() - ref).norm())
        db = float((gb.double().cpu() - ref).norm())
        # the reference error is the map path's or, when larger, the fp32
        # oracle's own (CPU, same inputs): downstream of the psi BatchNorm(1)
        # sums (cancellation ~1e3) two independent fp32 noise draws differ by
        # 2x at random, and the vector path is held to the oracle as every
        # other fp32 parity test is (round 6)
        d32 = float((g32[k].double().cpu() - ref).norm()) if (not bf16 and k in g32) else 0.0
        base = fac * max(db, d32) + floor * gmax
        # the BatchNorm term spread may widen the bound, but never past half
        # the gradient's norm (an uncapped sigma passed ~1.2 |g|)
        bound[k] = max(base, min(base + fac * sigma.get(k, 0.0), 0.5 * float(ref.norm())))
        worst.append((da / bound[k], k, da, db))
    worst.sort(reverse=True)
    print(f"{inj} bf16={bf16} shortcut={sc}: worst (err / bound, name, |vec - fp64|, |map - fp64|) {worst[:3]}")
    assert worst[0][0] <= 1.0, worst[:5]
    for k in pa:
        if k not in g64:   # no gradient reaches it (z_initial without the bottleneck)
            assert pa[k].grad is None or float(pa[k].grad.abs().max()) == 0.0, k
    ba, bb = dict(a.named_buffers()), dict(b.named_buffers())
    for k in ba:
        if ba[k].is_floating_point():
            torch.testing.assert_close(ba[k], bb[k], rtol=(2e-2 if bf16 else 1e-5), atol=(2e-3 if bf16 else 1e-6))
        else:
            assert torch.equal(ba[k], bb[k]), k
    # a second micro-step accumulates into the existing .grad buffers
    ra = _run(a, x, t, eps, True, bf16, steps=1, shortcut=sc)
    rb = _run(b, x, t, eps, False, bf16, steps=1)
    assert _rel(ra[0][0], rb[0][0]) < tol
    for k in g64:
        ga, gb = pa[k].grad.double(), pb[k].grad.double()
        assert float((ga - gb).norm()) <= 3 * (bound[k] + fac * float((pb[k].grad.double().cpu() - 2 * g64[k]).norm())), k


@pytest.mark.parametrize("inj", ["all", "bottleneck"])
@pytest.mark.parametrize("sc", [True, False])
def test_latent_vector_path_eval_forward(inj, sc):
    torch.manual_seed(2)
    B, S = 3, 128
    x = torch.rand(B, 3, S, S, device=DEV).contiguous(memory_format=CL)
    t = (torch.rand(B, 1, S, S, device=DEV) < 0.05).float()
    eps = torch.randn(B, 32, device=DEV)
    a = _model(inj, 3)
    _run(a, x, t, eps, True, False, train=True)      # non-trivial running statistics
    a.zero_grad(set_to_none=True)
    b = copy.deepcopy(a)
    with torch.no_grad():
        ra = _run(a, x, t, eps, True, False, train=False, shortcut=sc)
        rb = _run(b, x, t, eps, False, False, train=False)
    for u, v in zip(ra[0][:3], rb[0][:3]):
        assert _rel(u, v) < 2e-4
