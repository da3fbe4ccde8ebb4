"""Parity at the BENCHMARKED configurations (BASELINE.json configs[1] and [2]),
round 3:

* config 2 (UNet(3,2)) and config 3 (UNetResNet(3,1), ResNet34 encoder, latent
  32, injection "all", fixed latent eps) at B=8, 3x512x512, in fp32 parity mode
  against the CPU oracle in fp32 AND fp64.  The argmax (class map) flips
  between the HIP path and the fp32 oracle are adjudicated against fp64: a
  flip is accepted only where the fp64 margin is within the fp32 reduction
  error the reference's OWN fp32 path makes at this size (measured in the same
  test as max |m_fp32_oracle - m_fp64|), times a stated factor; and the HIP
  path's margin error must not exceed that factor times the oracle's.  This
  replaces a fixed "margin > 1e-4" mask.
* config 3 under bf16 autocast (the benchmarked precision) against the fp32
  oracle, with the reference's own CPU-bf16 drift as the yardstick (as
  test_gpu_model.test_unet_config2_bf16_b8_vs_oracle does for config 2):
  logits, mu / logvar, CombinedLoss + 1e-3 * KL, per-parameter gradient norms.

Reference behaviour: unet/unet_model.py:25-36, unet/unet_resnet.py:196-240,
utils/loss.py:44-63,148-170.  The ResNet34 encoder is a restatement (timm is
absent): config-3 parity is against the oracle's restatement.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last
B, S = 8, 512

from golden_util import adjudicate_flips as _adjudicate, class_margin as margin  # noqa: E402


def _threads():
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))


def _batch(classes):
    g = torch.Generator().manual_seed(1000)   # bench.py synthetic(): rank 0
    x = torch.rand(B, 3, S, S, generator=g)
    m = (torch.rand(B, 1, S, S, generator=g) < 0.0085).float()
    t = torch.cat([1 - m, m], 1) if classes == 2 else m
    return x.contiguous(memory_format=CL), t


def _eps():
    return torch.randn(B, 32, generator=torch.Generator().manual_seed(77))


def _split(state, dtype):
    p = {k: v.clone().to(dtype) for k, v in state.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone())
            for k, v in state.items() if "running" in k or "num_batches" in k}
    return p, bufs


@pytest.mark.timeout(900)
def test_unet_config2_fp32_b8_flips_adjudicated_fp64():
    from oracle import cpu_ref as R
    from vaeunet_amd import UNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss
    from vaeunet_amd.metrics import dice_score
    _threads()
    model = seeded_init_(UNet(3, 2), 0)
    state = model.state_dict()
    x, t = _batch(2)
    with torch.no_grad():
        p32, b32 = _split(state, torch.float32)
        l32 = R.unet_forward(x, p32, b32, True).contiguous()
        p64, b64 = _split(state, torch.float64)
        l64 = R.unet_forward(x.double(), p64, b64, True).contiguous()
    loss32 = float(R.combined_loss(l32, t))
    model = model.to(DEV).to(memory_format=CL).train()
    with torch.no_grad():
        lg = model(x.to(DEV))
        loss = float(CombinedLoss()(lg, t.to(DEV)))
        ds = float(dice_score(lg, l32.to(DEV).contiguous(memory_format=CL)))
    lg = lg.float().cpu().contiguous()
    scale = float(l64.abs().max())
    assert float((lg.double() - l64).abs().max()) <= 1e-3 * scale        # north_star: logits within 1e-3
    assert abs(loss - loss32) < 1e-3                                     # Dice+BCE loss within 1e-3
    _adjudicate("config2 fp32 B=8", margin(lg).double(), margin(l32).double(), margin(l64))
    assert ds == pytest.approx(float(R.dice_score(l32, l32)), abs=1e-4)  # reference dice_score semantics


@pytest.mark.timeout(900)
def test_unetresnet_config3_fp32_b8_flips_adjudicated_fp64():
    from oracle import cpu_ref as R
    from vaeunet_amd import UNetResNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    _threads()
    model = seeded_init_(UNetResNet(3, 1, pretrained=False), 0)
    state = model.state_dict()
    x, t = _batch(1)
    eps = _eps()
    with torch.no_grad():
        p32, b32 = _split(state, torch.float32)
        l32, mu32, lv32 = R.unet_resnet_forward(x, p32, b32, eps=eps)
        p64, b64 = _split(state, torch.float64)
        l64, mu64, lv64 = R.unet_resnet_forward(x.double(), p64, b64, eps=eps.double())
    loss32 = float(R.combined_loss(l32, t) + 1e-3 * R.kl_with_free_bits(mu32, lv32, 1e-3))
    model = model.to(DEV).to(memory_format=CL).train()
    model.eps_override = eps
    with torch.no_grad():
        lg, mu, lv = model(x.to(DEV))
        loss = float(CombinedLoss()(lg, t.to(DEV)) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3))
    lg = lg.float().cpu().contiguous()
    scale = float(l64.abs().max())
    assert float((lg.double() - l64).abs().max()) <= 1e-3 * scale
    for a, ref in ((mu, mu64), (lv, lv64)):
        assert float((a.double().cpu() - ref).abs().max()) <= 1e-3 * float(ref.abs().max())
    assert abs(loss - loss32) < 1e-3
    _adjudicate("config3 fp32 B=8", lg[:, 0].double(), l32[:, 0].double(), l64[:, 0])


# bf16 tolerances (as tests/test_gpu_model.py, config 2): the reference's own
# CPU-autocast bf16 path against its fp32 path is the yardstick
BF16_VS_REF_DRIFT = 1.5
BF16_LOSS = 1e-2
BF16_GNORM = 5e-2
BF16_TOTAL = 2e-2
BF16_FLIPS = 1.5


def _drift(a, ref):
    d = (a - ref).abs()
    return d.max().item() / ref.abs().max().item(), (d.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt()).item()


def _ref_bf16_run(R, state, x, t, eps, names, probe=False):
    """The reference's own CPU-bf16 autocast step: (per-parameter gradient
    norms, logits, mu, logvar, loss, per-BatchNorm dz if probe)."""
    ref16 = R.UNetResNetRef(state)
    R.PROBE = {} if probe else None
    try:
        with torch.autocast("cpu", dtype=torch.bfloat16):
            l16, mu16, lv16 = ref16.forward(x, eps, True)
            loss16 = R.combined_loss(l16.float(), t) + 1e-3 * R.kl_with_free_bits(mu16.float(), lv16.float(), 1e-3)
        loss16.backward()
        dz = {k: v[1].grad.detach().float() for k, v in R.PROBE.items() if not k.startswith("gate:")} \
            if probe else None
    finally:
        R.PROBE = None
    g16 = np.array([float(ref16.p[k].grad.double().norm()) if ref16.p[k].grad is not None else 0.0
                    for k in names])
    ref16.vec1 = {k: ref16.p[k].grad.detach().double().reshape(-1) for k in names
                  if ref16.p[k].grad is not None and ref16.p[k].grad.dim() == 1}
    return g16, l16.detach().float().contiguous(), mu16.detach().float(), lv16.detach().float(), loss16, dz, ref16


# The reference's own bf16 drift of ONE parameter's gradient norm is not a
# stable yardstick: for the cancellation-dominated BatchNorm-affine sums
# (dgamma = sum dz * xhat over up to 524k pixels) it swings by up to 17x
# between inputs that are the same at bf16 resolution (encoder.bn1.weight:
# 6.1 % / 13.8 % / 1.6 % for the bench input and two copies perturbed by a
# relative 2^-12 / 2^-10 -- below the bf16 half-ulp, so only elements at a
# rounding boundary change -- and layer1.2.bn1.weight 3.1 / 2.2 / 27.4 %),
# because the bf16 backward is ~80 % away from the fp32 one elementwise at
# the encoder (the dz of every BatchNorm, in the reference's path as in ours:
# tools/bn_drift_probe.py, profiles/r5b_bn_drift_probe.log).  Round 5: both
# paths run on the same seven-input ensemble (the bench input and six
# copies perturbed by a relative 2^-13 ... 2^-10); a BatchNorm-affine
# gradient's drift is the ensemble MEAN of its per-channel relative error
# ||g - g32|| / ||g32|| (a sum over channels: a stable statistic, where the
# norm drift |(||g|| - ||g32||)| / ||g32|| of a vector 80 % off elementwise is
# one noise draw -- its ensemble mean still differed 2x between two paths
# whose per-channel errors agree, profiles/r5k_bn_drift_probe.log), the HIP
# path's within 1.5x the reference's + 5 %; weights (>= 2-D, well
# conditioned) compare the bench input's norm drift with the reference
# ensemble's max; and the elementwise dz drift is compared at every BatchNorm
# (HIP must not drift more than the reference's own bf16 path).
REF_PERTURB = (2.0 ** -13, 2.0 ** -12, 2.0 ** -11.5, 2.0 ** -11, 2.0 ** -10.5, 2.0 ** -10)
DZ_VS_REF = 1.05
# per-gradient norm drift cap of the config-3 bf16 test (VERDICT r5 "do this"
# 1): every BatchNorm-affine gradient's bench-input norm drift within 2x the
# reference's own bf16 ensemble max + 5 %
BF16_GNORM_VS_ENS = 2.0


class _DzRecorder:
    """Records dz = dL/d(BatchNorm output) (the ReLU mask applied) at every
    BatchNorm the engine's bn_bwd serves, keyed by the module's state_dict
    prefix (the oracle PROBE's key), as CPU fp64/fp32 tensors."""

    def __init__(self, model, dtype=torch.float32):
        from vaeunet_amd import engine as E, kernels as K
        self.E, self.K, self.dtype, self.dz = E, K, dtype, {}
        self.names = {id(mod): n + "." for n, mod in model.named_modules() if isinstance(mod, torch.nn.BatchNorm2d)}
        # the attention gates' psi BatchNorm(1) runs its backward straight
        # through kernels.bn_backward (no ReLU: dz = dbnq), keyed by its weight
        self.psi = {id(mod.weight): n + "." for n, mod in model.named_modules()
                    if isinstance(mod, torch.nn.BatchNorm2d) and n.endswith("psi.1")}

    def __enter__(self):
        E, K = self.E, self.K
        self.orig = orig = E.bn_bwd
        self.orig_k = orig_k = K.bn_backward

        def bn_backward(dy, x, coef, gamma, relu, *a, **kw):
            pre = self.psi.get(id(gamma))
            if pre is not None and not relu:
                self.dz[pre] = dy.detach().float().to(self.dtype).cpu()
            return orig_k(dy, x, coef, gamma, relu, *a, **kw)
        K.bn_backward = bn_backward

        def bn_bwd(dy, xx, coef, bn, relu, M, *a, **kw):
            pre = self.names.get(id(bn))
            if pre is not None:
                d = (dy.materialize(M) if isinstance(dy, E.PoolGrad) else dy).detach().float()
                if relu:
                    C_ = xx.shape[1]
                    d = d * ((xx.float() * coef[0].view(1, C_, 1, 1) + coef[1].view(1, C_, 1, 1)) > 0).float()
                self.dz[pre] = d.to(self.dtype).cpu()
            return orig(dy, xx, coef, bn, relu, M, *a, **kw)
        E.bn_bwd = bn_bwd
        # the attention gates' W_g / W_x BatchNorms (round 6: one paired
        # backward, no ReLU: dz = ds for both)
        self.orig_pair = orig_pair = E.bn_bwd_pair

        def bn_bwd_pair(dy, a, b, M):
            for _, _, bn, _ in (a, b):
                pre = self.names.get(id(bn))
                if pre is not None:
                    self.dz[pre] = dy.detach().float().to(self.dtype).cpu()
            return orig_pair(dy, a, b, M)
        E.bn_bwd_pair = bn_bwd_pair
        return self

    def __exit__(self, *a):
        self.E.bn_bwd = self.orig
        self.E.bn_bwd_pair = self.orig_pair
        self.K.bn_backward = self.orig_k
        return False


@pytest.mark.timeout(900)
def test_unetresnet_config3_bf16_b8_vs_oracle():
    from oracle import cpu_ref as R
    from vaeunet_amd import UNetResNet, engine as E, _lib
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    _threads()
    # diagnostics: VU_TEST_TUNE="KEY=VAL,..." (vu_gemm_set_tuning before the run)
    for kv in filter(None, os.environ.get("VU_TEST_TUNE", "").split(",")):
        key, val = kv.split("=")
        _lib.call("vu_gemm_set_tuning", int(key), int(val))
    model = seeded_init_(UNetResNet(3, 1, pretrained=False), 0)
    state = model.state_dict()
    names = [k for k, _ in model.named_parameters()]
    x, t = _batch(1)
    eps = _eps()
    ref = R.UNetResNetRef(state)
    R.PROBE = {}
    try:
        lref, muref, lvref = ref.forward(x, eps, True)
        loss_ref = R.combined_loss(lref, t) + 1e-3 * R.kl_with_free_bits(muref, lvref, 1e-3)
        loss_ref.backward()
        dz32 = {k: v[1].grad.detach().float() for k, v in R.PROBE.items() if not k.startswith("gate:")}
    finally:
        R.PROBE = None
    gref = np.array([float(ref.p[k].grad.double().norm()) if ref.p[k].grad is not None else 0.0 for k in names])
    lref, muref, lvref = lref.detach().contiguous(), muref.detach(), lvref.detach()
    g16, l16, mu16, lv16, loss16, dz16, ref16 = _ref_bf16_run(R, state, x, t, eps, names, probe=True)
    ref_max, ref_rms = _drift(l16, lref)
    ref_flips = int(((l16 > 0) != (lref > 0)).sum())
    ref_mu = max(_drift(mu16, muref)[0], _drift(lv16, lvref)[0])
    r = torch.rand(x.shape, generator=torch.Generator().manual_seed(5)) * 2 - 1
    xps = [(x * (1 + sc * r)).contiguous(memory_format=CL) for sc in REF_PERTURB]
    g16_ens, v16_ens = [g16], [ref16.vec1]
    for xp in xps:
        run = _ref_bf16_run(R, state, xp, t, eps, names)
        g16_ens.append(run[0])
        v16_ens.append(run[6].vec1)

    model = model.to(DEV).to(memory_format=CL).train()
    model.eps_override = eps
    with _DzRecorder(model) as rec:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, mu, lv = model(x.to(DEV))
            loss = CombinedLoss()(lg, t.to(DEV)) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
        loss.backward()
    dz_hip = rec.dz
    lg = lg.detach().float().cpu().contiguous()
    max_rel, rms_rel = _drift(lg, lref)
    flips = int(((lg > 0) != (lref > 0)).sum())
    mu_rel = max(_drift(mu.detach().float().cpu(), muref)[0], _drift(lv.detach().float().cpu(), lvref)[0])
    params = dict(model.named_parameters())
    gn = np.array([float(params[k].grad.double().norm()) if params[k].grad is not None else 0.0 for k in names])
    ghip_ens = [gn]
    vhip_ens = [{k: p.grad.detach().double().cpu().reshape(-1) for k, p in params.items()
                 if p.grad is not None and p.dim() == 1}]
    for xp in xps:   # the same perturbed inputs through the HIP path (fresh model, same weights)
        mp = UNetResNet(3, 1, pretrained=False)
        mp.load_state_dict(state)
        mp = mp.to(DEV).to(memory_format=CL).train()
        mp.eps_override = eps
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lp, mup, lvp = mp(xp.to(DEV))
            lossp = CombinedLoss()(lp, t.to(DEV)) + 1e-3 * kl_with_free_bits(mup, lvp, free_bits=1e-3)
        lossp.backward()
        pp = dict(mp.named_parameters())
        ghip_ens.append(np.array([float(pp[k].grad.double().norm()) if pp[k].grad is not None else 0.0
                                  for k in names]))
        vhip_ens.append({k: p.grad.detach().double().cpu().reshape(-1) for k, p in pp.items()
                         if p.grad is not None and p.dim() == 1})
        del mp, pp
    big = gref > 1e-3 * gref.max()
    grel = np.abs(gn - gref) / np.maximum(gref, 1e-30)
    grel_ens = np.max([np.abs(g - gref) / np.maximum(gref, 1e-30) for g in g16_ens], axis=0)
    mean_ref = np.mean([np.abs(g - gref) / np.maximum(gref, 1e-30) for g in g16_ens], axis=0)
    mean_hip = np.mean([np.abs(g - gref) / np.maximum(gref, 1e-30) for g in ghip_ens], axis=0)
    g32v = {k: p.grad.detach().double().reshape(-1) for k, p in ref.p.items() if p.grad is not None}

    def vrel(ens):   # ensemble mean of the per-channel relative error, per 1-D parameter
        out = np.zeros(len(names))
        for i, k in enumerate(names):
            if k in ens[0] and k in g32v:
                den = max(float(g32v[k].norm()), 1e-30)
                out[i] = np.mean([float((v[k] - g32v[k]).norm()) / den for v in ens])
        return out
    vmean_ref, vmean_hip = vrel(v16_ens), vrel(vhip_ens)
    grel16 = np.abs(g16 - gref) / np.maximum(gref, 1e-30)   # the reference's own bf16 gradient drift
    # per parameter: excess over the reference's own bf16 drift (ensemble max)
    excess = grel - BF16_VS_REF_DRIFT * grel_ens
    worst = sorted(((excess[i], names[i], grel[i], grel_ens[i]) for i in np.where(big)[0]), reverse=True)[:5]
    tot = abs(np.sqrt((gn ** 2).sum()) / np.sqrt((gref ** 2).sum()) - 1)
    npx = lg.numel()
    # elementwise dz drift at every BatchNorm: HIP vs the reference's bf16
    dzr = []
    for k, d32 in dz32.items():
        if k in dz_hip and k in dz16:
            den = float(d32.double().norm())
            if den > 0:
                dzr.append((float((dz_hip[k].double() - d32.double()).norm()) / den,
                            float((dz16[k].double() - d32.double()).norm()) / den, k))
    dz_worst = max(dzr, key=lambda v: v[0] / (DZ_VS_REF * v[1] + 0.01))
    print(f"config3 bf16 B=8 vs fp32 oracle: HIP logits max_rel {max_rel:.3e} rms_rel {rms_rel:.3e} flips "
          f"{flips}/{npx}, mu/logvar max_rel {mu_rel:.3e}; reference CPU-bf16 max_rel {ref_max:.3e} rms_rel "
          f"{ref_rms:.3e} flips {ref_flips} mu/logvar {ref_mu:.3e}; loss {loss.item():.6f} vs "
          f"{loss_ref.item():.6f}; grad-norm worst (excess, name, HIP, CPU-bf16 ensemble max) "
          f"{[(round(float(a), 4), b, round(float(c), 4), round(float(d), 4)) for a, b, c, d in worst[:3]]}; "
          f"total {tot:.2e}; dz drift at {len(dzr)} BatchNorms, HIP / CPU-bf16 max "
          f"{max(a / b for a, b, _ in dzr):.3f} (worst {dz_worst[2]}: {dz_worst[0]:.3f} vs {dz_worst[1]:.3f})")
    assert max_rel <= BF16_VS_REF_DRIFT * ref_max + 5e-3
    assert rms_rel <= BF16_VS_REF_DRIFT * ref_rms + 5e-3
    assert mu_rel <= BF16_VS_REF_DRIFT * ref_mu + 5e-3
    assert flips <= BF16_FLIPS * ref_flips + 1e-3 * npx
    assert abs(loss.item() - loss_ref.item()) < BF16_LOSS
    assert len(dzr) >= 50   # every conv BatchNorm of the encoder and the decoder blocks (53)
    for a, b, k in dzr:
        assert a <= DZ_VS_REF * b + 0.01, (k, a, b)
    # per-parameter gradient norms within 1.5x the reference's own bf16 drift
    # (max over the ensemble) + 5 %: weights (>= 2-D) and, individually, the
    # BatchNorm-affine gradients; the latter also as a group (relative L2
    # error of the concatenated BN-affine gradients within 1.5x the
    # reference's + 5 %).
    dims = {k: p.dim() for k, p in model.named_parameters()}
    wbig = [i for i in np.where(big)[0] if dims[names[i]] >= 2]
    bbig = [i for i in np.where(big)[0] if dims[names[i]] == 1]
    worst_w = max(excess[i] for i in wbig)
    assert worst_w < BF16_GNORM, [w for w in worst if dims[w[1]] >= 2]
    excess_b = vmean_hip - BF16_VS_REF_DRIFT * vmean_ref
    worst_bl = sorted(((excess_b[i], names[i], vmean_hip[i], vmean_ref[i]) for i in bbig), reverse=True)[:3]
    worst_b = worst_bl[0][0]
    for _, nm, _, _ in worst_bl:
        i = names.index(nm)
        print(f"  {nm}: per-channel error HIP {vmean_hip[i]:.4f} vs CPU-bf16 {vmean_ref[i]:.4f} (ensemble means); "
              f"norm drifts HIP {[round(float(abs(g[i] - gref[i]) / gref[i]), 4) for g in ghip_ens]} "
              f"(mean {mean_hip[i]:.4f}), CPU-bf16 {[round(float(abs(g[i] - gref[i]) / gref[i]), 4) for g in g16_ens]} "
              f"(mean {mean_ref[i]:.4f})")
    assert worst_b < BF16_GNORM, worst_bl
    # and each BatchNorm-affine gradient's own bench-input norm drift (round 4's
    # per-gradient cap, restored at 2x the reference's ensemble max + 5 %)
    capv = sorted(((grel[i] - BF16_GNORM_VS_ENS * grel_ens[i], names[i], grel[i], grel_ens[i]) for i in bbig),
                  reverse=True)
    print(f"config3 bf16: BN-affine norm drift worst (excess over {BF16_GNORM_VS_ENS}x ensemble max, name, HIP, "
          f"CPU-bf16 ensemble max) {[(round(float(a_), 4), b_, round(float(c_), 4), round(float(d_), 4)) for a_, b_, c_, d_ in capv[:3]]}")
    assert capv[0][0] <= BF16_GNORM, capv[:3]
    vecs = {k: (params[k].grad.double().cpu().reshape(-1), ref.p[k].grad.double().reshape(-1),
                ref16.p[k].grad.double().reshape(-1)) for k in (names[i] for i in bbig)}
    num = sum(float((a - r_).pow(2).sum()) for a, r_, _ in vecs.values()) ** 0.5
    num16 = sum(float((c - r_).pow(2).sum()) for _, r_, c in vecs.values()) ** 0.5
    den = sum(float(r_.pow(2).sum()) for _, r_, _ in vecs.values()) ** 0.5
    print(f"config3 bf16: BN-affine gradients, relative L2 error HIP {num / den:.3e} vs CPU-bf16 "
          f"{num16 / den:.3e}; worst weight excess {worst_w:.3e}; BN-affine ensemble-mean per-channel error worst "
          f"(excess, name, HIP, CPU-bf16) {[(round(float(a_), 4), b_, round(float(c_), 4), round(float(d_), 4)) for a_, b_, c_, d_ in worst_bl]}; "
          f"bench-input-only CPU-bf16 drift of the worst: {grel16[names.index(worst[0][1])]:.3f}")
    assert num / den <= BF16_VS_REF_DRIFT * num16 / den + BF16_GNORM
    assert tot < BF16_TOTAL


# ---------------------------------------------------------------------------
# fp32 BACKWARD parity at 512^2 (train.py:403 loss.backward()), B=2: every
# parameter gradient of the HIP fp32 path vs the fp64 oracle, judged against
# the fp32 oracle's OWN error at the same size (the reference's CPU fp32
# autograd is what a user of the reference gets):
#
#   ||g_hip - g64||  <=  GRAD_ERR_FACTOR * ( ||g32 - g64||  +  sigma_k  +  u32 * ||g64|| )
#
# sigma_k, per BatchNorm affine gradient (round 5, replaces round 4's global
# floor 1e-6 * max_k ||g64_k||): the gradient is a reduction over pixels,
# dbeta = sum_p dz_p and dgamma = sum_p dz_p * xhat_p, and its error is the
# sum of its terms' errors.  The oracle probes every BatchNorm
# (oracle/cpu_ref.PROBE) and sigma_k = || t32 - t64 ||_2 over the terms t of
# that reduction: the spread a sum of the terms has when each term carries the
# fp32 oracle's own per-term error (independent term errors add in quadrature).
# It matters where a reduction is ill-conditioned, sum |t| >> |sum t|: the
# attention psi BatchNorm(1) bias at up2 has sum |dz| / |sum dz| = 4.5e3, so
# the ~0.5 % per-pixel error the fp32 backward carries at that depth (oracle:
# 4.7e-3, HIP path: 7.4e-3 -- measured by tools/psi_probe.py,
# profiles/r5a_psi_probe.log) becomes 4-25 % on the sum, and that sum of the
# HIP path's own dbnq in fp64 reproduces the HIP gradient's error exactly (the
# reduction kernels add nothing).  u32 * ||g64||: storing the result in fp32.
# Gradients that are mathematically zero (the bias of a conv feeding a
# train-mode BatchNorm: BN(x + b) does not depend on b) are written as exact
# zeros by the HIP path for the 1x1 / ConvT convs (engine.bias_grad), where
# the reference's autograd leaves summation noise (the psi conv's bias, summed
# by its own kernel, also keeps noise): held to "both within the fp32 noise
# floor 1e-5 * max ||g||" instead, and the exact zeros are counted.
# ---------------------------------------------------------------------------
GRAD_ERR_FACTOR = 4.0
GRAD_VS_ORACLE = 1.5
SIGMA_CAP = 0.5
U32 = 2.0 ** -24
BW_B = 2


def _grad_adjudicate(tag, names, g_hip, g32, g64, sigma, dz_ok=None):
    """Every gradient k: ||g_hip - g64|| <= GRAD_VS_ORACLE * (||g32 - g64|| +
    u32 ||g64||) -- the HIP fp32 path within 1.5x the fp32 oracle's own error.
    A gradient outside it is re-judged on the term-spread bound
    GRAD_ERR_FACTOR * (||g32 - g64|| + sigma_k + u32 ||g64||) ONLY when that
    bound stays below SIGMA_CAP * ||g64|| (a sigma-dominated bound
    of ~1.2 |g| passed a 100 %-wrong gradient) AND the terms of its sum -- the
    dz of its BatchNorm, ``dz_ok[prefix]`` -- were pinned elementwise within
    DZ32_FACTOR x the fp32 oracle's own per-term error (_dz_adjudicate): such
    a gradient's error is a draw of the per-term noise over an ill-conditioned
    sum whose oracle draw was small.  Anything else is 'unpinnable' and fails."""
    gmax = max(float(g.norm()) for g in g64.values())
    rows, zero, spread, unpin = [], [], [], []
    for k in names:
        r = float(g64[k].norm())
        if r <= 1e-9 * gmax:
            zero.append(float(g_hip[k].abs().max()) == 0.0)
            assert float(g_hip[k].norm()) <= 1e-5 * gmax, (k, float(g_hip[k].norm()))
            assert float(g32[k].norm()) <= 1e-5 * gmax, (k, float(g32[k].norm()))
            continue
        d_h = float((g_hip[k] - g64[k]).norm())
        d_32 = float((g32[k] - g64[k]).norm())
        s = sigma.get(k, 0.0)
        ratio = d_h / (GRAD_VS_ORACLE * (d_32 + U32 * r))   # > 1: outside the primary bound
        rows.append((ratio, k, d_h / r, d_32 / r, s / r))
        if ratio > 1.0:
            b2 = GRAD_ERR_FACTOR * (d_32 + s + U32 * r)
            pre = k.rsplit(".", 1)[0] + "."
            if b2 > SIGMA_CAP * r or not (dz_ok or {}).get(pre, False):
                unpin.append((k, d_h / r, d_32 / r, s / r))
            else:
                spread.append((d_h / b2, k, d_h / r, d_32 / r, s / r))
    rows.sort(reverse=True)
    print(f"{tag}: {len(rows)} gradients vs fp64, {len(zero)} mathematically zero ({sum(zero)} written as exact "
          f"zeros); worst (HIP err / ({GRAD_VS_ORACLE} x fp32-oracle err), name, HIP rel, fp32-oracle rel, term "
          f"spread / |g|): {[(f'{a:.2f}', b, f'{c:.2e}', f'{d:.2e}', f'{e:.2e}') for a, b, c, d, e in rows[:5]]}; "
          f"median HIP/oracle {sorted(r[2] / max(r[3], 1e-300) for r in rows)[len(rows) // 2]:.3f}; "
          f"{len(spread)} judged on the capped term spread {[(f'{a:.2f}', b) for a, b, *_ in sorted(spread, reverse=True)[:4]]}; "
          f"unpinnable {unpin}")
    assert not unpin, unpin
    assert all(a <= 1.0 for a, *_ in spread), sorted(spread, reverse=True)[:4]
    return rows


def _bw_batch(classes):
    x, t = _batch(classes)
    return x[:BW_B].contiguous(memory_format=CL), t[:BW_B].contiguous()


def _oracle_grads(fwd, state, dtype, probe=False):
    """The oracle's gradients (fp64 copies) and loss; probe: also the terms
    of every train-mode BatchNorm's affine-gradient reductions
    (prefix+'bias': dz, prefix+'weight': dz * xhat), in fp64."""
    from oracle import cpu_ref as R
    p, bufs = _split(state, dtype)
    for v in p.values():
        v.requires_grad_(True)
    R.PROBE = {} if probe else None
    try:
        loss = fwd(p, bufs)
        loss.backward()
        terms = {}
        if probe:
            for pre, v in R.PROBE.items():
                if pre.startswith("gate:"):
                    continue
                xh, y = v
                dz = y.grad.detach().double()
                terms[pre + "bias"] = dz
                terms[pre + "weight"] = dz * xh.detach().double()
    finally:
        R.PROBE = None
    grads = {k: v.grad.detach().double() if v.grad is not None else torch.zeros_like(v, dtype=torch.float64)
             for k, v in p.items()}
    return grads, float(loss.detach()), terms


def _oracle_pair(fwd, state):
    """fp64 and fp32 oracle gradients, the per-BatchNorm term spreads sigma,
    the fp64 dz at every BatchNorm and the fp32 oracle's own error on it."""
    g64, loss64, t64 = _oracle_grads(fwd(torch.float64), state, torch.float64, probe=True)
    g32, _, t32 = _oracle_grads(fwd(torch.float32), state, torch.float32, probe=True)
    sigma = {k: float((t32[k] - t64[k]).norm()) for k in t64 if k in t32}
    dz64 = {k[:-4]: t64[k] for k in t64 if k.endswith("bias")}
    dzerr32 = {pre: float((t32[pre + "bias"] - d).norm()) for pre, d in dz64.items() if pre + "bias" in t32}
    del t32, t64
    return g32, g64, loss64, sigma, dz64, dzerr32


# dz = dL/d(BatchNorm output) at every BatchNorm the engine's backward serves,
# elementwise vs fp64: the HIP fp32 path's error within DZ32_FACTOR x the fp32
# oracle's own (VERDICT r5 "do this" 1: the error a gradient carries arrives
# with dz -- tools/psi_probe.py -- so this pins its source directly, at every
# depth, independent of how ill-conditioned the affine sums over it are)
DZ32_FACTOR = 1.5


def _dz_adjudicate(tag, dz_hip, dz64, dzerr32):
    rows = []
    for pre, d64 in dz64.items():
        if pre not in dz_hip or pre not in dzerr32:
            continue
        nrm = float(d64.norm())
        if nrm == 0:
            continue
        e_h = float((dz_hip[pre].double() - d64).norm())
        rows.append((e_h / (DZ32_FACTOR * dzerr32[pre] + U32 * nrm), pre, e_h / nrm, dzerr32[pre] / nrm))
    rows.sort(reverse=True)
    print(f"{tag}: dz at {len(rows)} BatchNorms vs fp64, worst (HIP err / ({DZ32_FACTOR} x fp32-oracle err), "
          f"name, HIP rel, fp32-oracle rel): {[(f'{a:.3f}', b, f'{c:.2e}', f'{d:.2e}') for a, b, c, d in rows[:4]]}; "
          f"median ratio HIP/oracle {sorted(r[2] / r[3] for r in rows)[len(rows) // 2]:.3f}")
    assert rows and rows[0][0] <= 1.0, rows[:4]
    return {pre: a <= 1.0 for a, pre, _, _ in rows}


@pytest.mark.timeout(900)
def test_unet_config2_fp32_backward_512_vs_fp64():
    from oracle import cpu_ref as R
    from vaeunet_amd import UNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss
    _threads()
    model = seeded_init_(UNet(3, 2), 0)
    state = model.state_dict()
    names = [k for k, _ in model.named_parameters()]
    x, t = _bw_batch(2)

    def fwd(dtype):
        return lambda p, b: R.combined_loss(R.unet_forward(x.to(dtype), p, b, True), t.to(dtype))
    g32, g64, loss64, sigma, dz64, dzerr32 = _oracle_pair(fwd, state)
    model = model.to(DEV).to(memory_format=CL).train()
    with _DzRecorder(model) as rec:
        loss = CombinedLoss()(model(x.to(DEV)), t.to(DEV))
        loss.backward()
    assert abs(float(loss.detach()) - loss64) < 1e-5
    params = dict(model.named_parameters())
    gh = {k: params[k].grad.detach().double().cpu() for k in names}
    dzrows = _dz_adjudicate("config2 fp32 backward B=2 512^2", rec.dz, dz64, dzerr32)
    assert len(dzrows) >= 30   # every conv BatchNorm + the attention gates' W_g / W_x / psi BatchNorms
    _grad_adjudicate("config2 fp32 backward B=2 512^2", names, gh, g32, g64, sigma, dzrows)


@pytest.mark.timeout(900)
def test_unetresnet_config3_fp32_backward_512_vs_fp64():
    from oracle import cpu_ref as R
    from vaeunet_amd import UNetResNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    _threads()
    model = seeded_init_(UNetResNet(3, 1, pretrained=False), 0)
    state = model.state_dict()
    names = [k for k, p in model.named_parameters()]
    x, t = _bw_batch(1)
    eps = _eps()[:BW_B]

    def fwd(dtype):
        def f(p, b):
            lg, mu, lv = R.unet_resnet_forward(x.to(dtype), p, b, eps=eps.to(dtype))
            return R.combined_loss(lg, t.to(dtype)) + 1e-3 * R.kl_with_free_bits(mu, lv, 1e-3)
        return f
    g32, g64, loss64, sigma, dz64, dzerr32 = _oracle_pair(fwd, state)
    model = model.to(DEV).to(memory_format=CL).train()
    model.eps_override = eps.to(DEV)
    with _DzRecorder(model) as rec:
        lg, mu, lv = model(x.to(DEV))
        loss = CombinedLoss()(lg, t.to(DEV)) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
        loss.backward()
    assert abs(float(loss.detach()) - loss64) < 1e-5
    dzrows = _dz_adjudicate("config3 fp32 backward B=2 512^2", rec.dz, dz64, dzerr32)
    assert len(dzrows) >= 56   # + the four decoder gates' psi BatchNorms
    params = dict(model.named_parameters())
    gh = {k: (params[k].grad.detach().double().cpu() if params[k].grad is not None
              else torch.zeros_like(params[k], dtype=torch.float64, device="cpu")) for k in names}
    _grad_adjudicate("config3 fp32 backward B=2 512^2", names, gh, g32, g64, sigma, dzrows)
