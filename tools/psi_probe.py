"""Where does the attention-gate psi BatchNorm(1) gradient error come from?
(VERDICT r4 'do this' 1.)  Config 2, B=2, 3x512x512, fp32: the HIP path's
gate intermediates -- the gate-output gradient dout, psi, dbnq = dL/d BN(q)
and q -- against the fp64 oracle, next to the fp32 oracle's own errors, per
gate; then the psi.1 gradients.  Test infrastructure (imports oracle/)."""
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "tests")]
from oracle import cpu_ref as R  # noqa: E402

B, S = 2, 512


def rel(a, ref):
    return float((a.double() - ref.double()).norm() / ref.double().norm())


def oracle(x, t, state, dtype):
    p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in state.items()
         if "running" not in k and "num_batches" not in k}
    b = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in state.items()
         if "running" in k or "num_batches" in k}
    R.PROBE = {}
    loss = R.combined_loss(R.unet_forward(x.to(dtype), p, b, True), t.to(dtype))
    loss.backward()
    gates = {}
    for k, v in R.PROBE.items():
        if k.startswith("gate:"):
            q, z, psi, out = v
            gates[k[5:]] = dict(q=q.detach(), psi=psi.detach(), dout=out.grad, dbnq=z.grad, dpsi=psi.grad)
    cond = R.probe_bn_conditioning()
    R.PROBE = None
    return gates, {k: v.grad.detach() for k, v in p.items()}, cond


def main():
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    from vaeunet_amd import UNet, engine as E, kernels as K
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss
    g = torch.Generator().manual_seed(1000)
    x = torch.rand(8, 3, S, S, generator=g)
    m = (torch.rand(8, 1, S, S, generator=g) < 0.0085).float()
    t = torch.cat([1 - m, m], 1)
    x, t = x[:B].contiguous(), t[:B].contiguous()
    model = seeded_init_(UNet(3, 2), 0)
    state = model.state_dict()
    model = model.cuda().to(memory_format=torch.channels_last).train()
    names = {id(getattr(model, u).attention): f"{u}.attention." for u in ("up1", "up2", "up3", "up4")}
    hip = {}
    cur = {}
    orig_bwd, orig_bnb = E.attention_bwd, K.bn_backward

    def bwd(M, att, saved, dout, dg_out, dg_acc):
        pre = names[id(att)]
        cur["pre"] = pre
        hip[pre] = dict(dout=dout.detach().double().cpu(), q=saved[6].double().cpu(), psi=saved[8].double().cpu())
        r = orig_bwd(M, att, saved, dout, dg_out, dg_acc)
        cur["pre"] = None
        return r

    def bnb(dy, xx, coef, *a, **kw):
        if cur.get("pre") and dy.shape[1] == 1:
            hip[cur["pre"]]["dbnq"] = dy.detach().double().cpu()
        return orig_bnb(dy, xx, coef, *a, **kw)
    E.attention_bwd, K.bn_backward = bwd, bnb
    loss = CombinedLoss()(model(x.cuda()), t.cuda())
    loss.backward()
    torch.cuda.synchronize()
    E.attention_bwd, K.bn_backward = orig_bwd, orig_bnb
    params = dict(model.named_parameters())
    print("HIP done", flush=True)
    o64, g64, cond = oracle(x, t, state, torch.float64)
    print("oracle fp64 done", flush=True)
    o32, g32, _ = oracle(x, t, state, torch.float32)
    print("oracle fp32 done", flush=True)
    for pre in ("up1.attention.", "up2.attention.", "up3.attention.", "up4.attention."):
        row = []
        for k in ("dout", "q", "psi", "dbnq"):
            row.append(f"{k}: HIP {rel(hip[pre][k], o64[pre][k]):.2e} fp32 {rel(o32[pre][k], o64[pre][k]):.2e}")
        print(pre, " | ".join(row))
        for k in ("psi.1.bias", "psi.1.weight", "psi.0.weight"):
            n = pre + k
            r = float(g64[n].double().norm())
            c = float(cond[n].norm()) / r if n in cond else float("nan")
            print(f"   {n}: HIP {rel(params[n].grad.cpu(), g64[n]):.3e} fp32 {rel(g32[n], g64[n]):.3e} "
                  f"cond(S/|g|) {c:.3e}")
        # the psi.1 gradients recomputed in fp64 from the HIP path's own dbnq / the fp64 dbnq
        d = hip[pre]["dbnq"]
        print(f"   sum(dbnq_HIP) in fp64 vs fp64 oracle: {float(d.sum() - o64[pre]['dbnq'].sum()) / float(o64[pre]['dbnq'].sum()):.3e}")


if __name__ == "__main__":
    main()
