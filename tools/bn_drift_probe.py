"""Where do the config-3 bf16 encoder BatchNorm-affine gradients drift?
(VERDICT r4 'do this' 3.)  UNetResNet(3,1), B=8, 3x512x512: the gradient
arriving at every BatchNorm output (dz, after the ReLU mask) in the HIP bf16
path and in the reference's own CPU-bf16 autocast path, each against the fp32
oracle, plus the affine gradients' norm errors -- in backward order, so the
growth of the drift can be followed.  Test infrastructure (imports oracle/)."""
import os
import sys

import numpy as np
import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "tests")]
from oracle import cpu_ref as R  # noqa: E402

B, S = 8, 512


def rel(a, ref):
    return float((a.double() - ref.double()).norm() / ref.double().norm().clamp_min(1e-300))


def oracle(x, t, eps, state, autocast):
    ref = R.UNetResNetRef(state)
    R.PROBE = {}
    if autocast:
        with torch.autocast("cpu", dtype=torch.bfloat16):
            lg, mu, lv = ref.forward(x, eps, True)
            loss = R.combined_loss(lg.float(), t) + 1e-3 * R.kl_with_free_bits(mu.float(), lv.float(), 1e-3)
    else:
        lg, mu, lv = ref.forward(x, eps, True)
        loss = R.combined_loss(lg, t) + 1e-3 * R.kl_with_free_bits(mu, lv, 1e-3)
    loss.backward()
    dz = {k: v[1].grad.detach().float() for k, v in R.PROBE.items() if not k.startswith("gate:")}
    xh = {k: v[0].detach().float() for k, v in R.PROBE.items() if not k.startswith("gate:") and k in FOCUS}
    R.PROBE = None
    return dz, {k: v.grad.detach().double() for k, v in ref.p.items() if v.grad is not None}, xh


# BatchNorms whose affine-gradient drift is decomposed (dz error vs xhat error)
FOCUS = ("encoder.bn1.", "encoder.layer1.0.bn2.", "encoder.layer1.0.bn1.", "encoder.layer2.0.bn1.")


def main():
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    from vaeunet_amd import UNetResNet, engine as E
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    g = torch.Generator().manual_seed(1000)
    x = torch.rand(B, 3, S, S, generator=g)
    m = (torch.rand(B, 1, S, S, generator=g) < 0.0085).float()
    x = x.contiguous(memory_format=torch.channels_last)
    eps = torch.randn(B, 32, generator=torch.Generator().manual_seed(77))
    model = seeded_init_(UNetResNet(3, 1, pretrained=False), 0)
    state = model.state_dict()
    model = model.cuda().to(memory_format=torch.channels_last).train()
    model.eps_override = eps.cuda()
    bn_name = {id(mod): n + "." for n, mod in model.named_modules() if isinstance(mod, torch.nn.BatchNorm2d)}
    hip, order, hipx = {}, [], {}
    orig = E.bn_bwd

    def bn_bwd(dy, xx, coef, bn, relu, M, *a, **kw):
        pre = bn_name.get(id(bn))
        if pre is not None and not isinstance(dy, E.PoolGrad):
            d = dy.detach().float()
            if relu:
                C = xx.shape[1]
                d = d * ((xx.float() * coef[0].view(1, C, 1, 1) + coef[1].view(1, C, 1, 1)) > 0).float()
            hip[pre] = d.cpu()
            order.append(pre)
            if pre in FOCUS:   # HIP's xhat from its own stored BN input and statistics
                C = xx.shape[1]
                hipx[pre] = ((xx.float() - coef[2].view(1, C, 1, 1)) * coef[3].view(1, C, 1, 1)).cpu()
        return orig(dy, xx, coef, bn, relu, M, *a, **kw)
    E.bn_bwd = bn_bwd
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lg, mu, lv = model(x.cuda())
        loss = CombinedLoss()(lg, m.cuda()) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
    loss.backward()
    torch.cuda.synchronize()
    E.bn_bwd = orig
    params = {k: v.grad.detach().double().cpu() for k, v in model.named_parameters() if v.grad is not None}
    print("HIP done", flush=True)
    dz32, g32, xh32 = oracle(x, m, eps, state, False)
    print("oracle fp32 done", flush=True)
    dz16, g16, xh16 = oracle(x, m, eps, state, True)
    print("oracle CPU-bf16 done", flush=True)
    print(f"{'BatchNorm (backward order)':44s} {'dz HIP':>9s} {'dz bf16':>9s} | {'dgamma HIP':>10s} "
          f"{'CPU-bf16':>9s} | {'dbeta HIP':>9s} {'CPU-bf16':>9s}")
    for pre in order:
        if pre not in dz32:
            continue
        r = []
        for k in ("weight", "bias"):
            n = pre + k
            ref = g32[n]
            gn = float(params[n].norm()) if n in params else 0.0
            r.append((abs(gn - float(ref.norm())) / float(ref.norm()),
                      abs(float(g16[n].norm()) - float(ref.norm())) / float(ref.norm())))
        print(f"{pre:44s} {rel(hip[pre], dz32[pre]):9.2e} {rel(dz16[pre], dz32[pre]):9.2e} | "
              f"{r[0][0]:10.2e} {r[0][1]:9.2e} | {r[1][0]:9.2e} {r[1][1]:9.2e}", flush=True)
    # decomposition of the dgamma = sum dz * xhat error (per channel, norm over channels)
    print("dgamma decomposition, relative to the fp32 dgamma norm: A = HIP dz x HIP xhat, "
          "C = HIP dz x fp32 xhat, D = fp32 dz x HIP xhat, E = bf16-ref dz x bf16-ref xhat, "
          "F = bf16-ref dz x fp32 xhat; dbeta: HIP / bf16-ref")
    for pre in FOCUS:
        if pre not in hipx or pre not in xh32:
            continue
        d32, x32 = dz32[pre].double(), xh32[pre].double()
        dh, xhh = hip[pre].double(), hipx[pre].double()
        d16, x16 = dz16[pre].double(), xh16[pre].double()
        G = (d32 * x32).sum((0, 2, 3))
        nb = float(G.norm())

        def e(a, b_):
            return float(((a * b_).sum((0, 2, 3)) - G).norm()) / nb
        db = d32.sum((0, 2, 3))
        print(f"  {pre:28s} A {e(dh, xhh):.3e}  C {e(dh, x32):.3e}  D {e(d32, xhh):.3e}  E {e(d16, x16):.3e}  "
              f"F {e(d16, x32):.3e} | dbeta {float((dh.sum((0, 2, 3)) - db).norm()) / float(db.norm()):.3e} / "
              f"{float((d16.sum((0, 2, 3)) - db).norm()) / float(db.norm()):.3e}; xhat rel err HIP "
              f"{rel(xhh, x32):.2e} bf16-ref {rel(x16, x32):.2e}", flush=True)


if __name__ == "__main__":
    main()
