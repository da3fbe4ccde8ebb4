"""Which torch (non-library) device ops a training step launches, and from
where: aten::fill_ / copy_ / zero_ / cat ... counted per Python call site in
vaeunet_amd/ (torch.profiler with stacks, one eager step after warm-up).
A tuning aid: every such op is a launch the step could fold into its own kernels.

usage: python tools/torch_op_census.py [--model unet|vae]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vae")
    args = ap.parse_args()
    from bench import synthetic
    from vaeunet_amd import UNet, UNetResNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    from vaeunet_amd.optim import FusedAdamW, clip_grad_norm_
    dev = torch.device("cuda")
    vae = args.model == "vae"
    model = UNetResNet(3, 1, pretrained=False) if vae else UNet(3, 2)
    model = seeded_init_(model, 0).to(dev).to(memory_format=torch.channels_last).train()
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    crit = CombinedLoss()
    x, t = synthetic(8, 512, 1 if vae else 2, 0, dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if vae:
                lg, mu, lv = model(x)
                loss = crit(lg, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
            else:
                loss = crit(model(x), t)
        loss.backward()
        clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    sites = collections.Counter()
    ops = collections.Counter()
    for ev in prof.events():
        name = ev.name
        if not name.startswith("aten::") or name in ("aten::empty", "aten::empty_like", "aten::empty_strided",
                                                      "aten::view", "aten::as_strided", "aten::reshape",
                                                      "aten::permute", "aten::t", "aten::transpose",
                                                      "aten::detach", "aten::alias", "aten::select",
                                                      "aten::slice", "aten::unsqueeze", "aten::squeeze",
                                                      "aten::expand", "aten::lift_fresh", "aten::_local_scalar_dense",
                                                      "aten::item", "aten::resolve_conj", "aten::resolve_neg",
                                                      "aten::result_type", "aten::is_nonzero", "aten::contiguous",
                                                      "aten::set_", "aten::unbind", "aten::split", "aten::chunk",
                                                      "aten::narrow", "aten::to", "aten::_to_copy", "aten::flatten",
                                                      "aten::unflatten", "aten::_reshape_alias", "aten::numpy_T",
                                                      "aten::empty_like", "aten::zeros_like", "aten::zeros",
                                                      "aten::ones_like", "aten::full", "aten::full_like",
                                                      "aten::new_empty", "aten::new_empty_strided"):
            continue
        # only leaf-ish device ops that launch kernels
        if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::") and \
                ev.cpu_parent.name not in ("aten::zeros", "aten::zeros_like", "aten::to", "aten::_to_copy",
                                           "aten::contiguous", "aten::full", "aten::full_like", "aten::ones_like"):
            continue
        frames = [f for f in (ev.stack or []) if "vaeunet_amd" in f or "bench.py" in f]
        site = frames[0] if frames else "(no package frame)"
        sites[(name, site)] += 1
        ops[name] += 1
    print("ops:", dict(ops.most_common()))
    for (name, site), n in sites.most_common(60):
        print(f"{n:4d}  {name:28s} {site}")


if __name__ == "__main__":
    main()
