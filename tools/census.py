"""Per-call-site GPU time of one training step: every C-ABI launch of the
engine is bracketed by HIP events (on the launch stream) and attributed to
its engine call site and, for the GEMMs, to its shape and algorithmic HBM
bytes.  A tuning aid, not part of the product.

usage: python tools/census.py [--model unet|vae] [--steps 2] [--top 60] [--engine-flag M.NAME=V] [--tune K=V]
"""
import argparse
import collections
import ctypes as C
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import _lib, kernels as K  # noqa: E402

RECS = []
ON = [False]
_orig = _lib.call
ENGINE = ("engine.py", "vae_engine.py", "unet_parts.py", "unet_resnet.py", "loss.py", "optim.py", "functional.py")


def _site():
    for f in reversed(traceback.extract_stack()[:-3]):
        if f.filename.endswith(ENGINE):
            return f"{os.path.basename(f.filename)}:{f.name}:{f.lineno}"
    return "?"


def _shape(name, args):
    try:
        if name == "vu_gemm_fwd":
            a = args[0]._obj
            g = a.a
            M = g.N * g.H * g.W
            K_ = g.R * g.S * g.C
            b = M * g.C * 2 + M * a.ncol * 2 + a.ncol * K_ * 2
            kid = _lib.query("vu_gemm_fwd_kernel", args[0], args[1])
            return f"fwd R{g.R}x{g.S} s{g.sy} C{g.C} {g.H}x{g.W} N{a.ncol} om{a.out_mode} k{kid}", b, 2 * M * K_ * a.ncol
        if name == "vu_gemm_wgrad":
            w = args[0]._obj
            M = w.p.N * w.p.H * w.p.W
            b = M * (w.p.C + w.q.C) * 2
            return f"wgrad R{w.q.R} {w.q.H}x{w.q.W} ni{w.ni} nj{w.nj} s{w.splits}", b, 2 * M * w.ni * w.nj
        # BatchNorm streams: (x, xs, y, ys, P, C, ...) -> bytes per launch (bf16/fp32 by dtype)
        nbytes = {"vu_bn_apply": 2, "vu_bn_bwd_reduce": 2, "vu_bn_bwd_apply": 3}
        if name in nbytes:
            iv = [int(getattr(a, "value", a) or 0) for a in (args[4], args[5], args[-2])]
            P, Cc, dt = iv
            esz = 2 if dt == _lib.BF16 else 4
            return f"P{P} C{Cc}", nbytes[name] * P * Cc * esz, 0
    except Exception:  # noqa: BLE001
        pass
    return "", 0, 0


def tcall(name, *args):
    if not ON[0]:
        return _orig(name, *args)
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    rc = _orig(name, *args)
    e.record()
    shp, b, fl = _shape(name, args)
    RECS.append((name, _site(), shp, b, fl, s, e))
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="unet")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--top", type=int, default=70)
    ap.add_argument("--engine-flag", action="append", default=[], metavar="MODULE.NAME=VAL",
                    help="set a vaeunet_amd module switch first (as bench.py), e.g. vae_engine.LATENT_SHORTCUT=0")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VAL")
    args = ap.parse_args()
    import importlib
    for kv in args.engine_flag:
        name, val = kv.split("=")
        modname, name = name.rsplit(".", 1) if "." in name else ("engine", name)
        mod = importlib.import_module("vaeunet_amd." + modname)
        old = getattr(mod, name)
        setattr(mod, name, bool(int(val)) if isinstance(old, bool) else type(old)(int(val)))
    for kv in args.tune:
        key, val = kv.split("=")
        _lib.call("vu_gemm_set_tuning", int(key), int(val))
    _lib.call = tcall
    for m in ("kernels", "loss", "optim", "metrics", "fp8"):
        mod = importlib.import_module("vaeunet_amd." + m)
        if hasattr(mod, "call"):
            mod.call = tcall
    dev = torch.device("cuda")
    from vaeunet_amd import UNet, UNetResNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    from vaeunet_amd.optim import FusedAdamW, clip_grad_norm_
    vae = args.model == "vae"
    model = (UNetResNet(3, 1, pretrained=False) if vae else UNet(3, 2))
    model = seeded_init_(model, 0).to(dev).to(memory_format=torch.channels_last).train()
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    crit = CombinedLoss()
    from bench import synthetic
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

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ON[0] = True
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ON[0] = False
    agg = collections.OrderedDict()
    tot = 0.0
    for name, site, shp, b, fl, s, e in RECS:
        ms = s.elapsed_time(e)
        tot += ms
        d = agg.setdefault((name, site, shp), [0, 0.0, b, fl])
        d[0] += 1
        d[1] += ms
    n = args.steps
    print(f"# {len(RECS) // n} launches/step, {tot / n:.3f} ms/step inside events")
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    for (name, site, shp), (cnt, ms, b, fl) in rows[:args.top]:
        us = ms / cnt * 1e3
        extra = ""
        if b:
            extra = f" {b / (us * 1e-6) / 1e9:7.0f}GB/s {fl / (us * 1e-6) / 1e12:6.0f}TF"
        print(f"{ms / n:7.3f} ms/step {cnt // n:3d}x {us:8.1f}us  {name[:22]:22s} {site[:44]:44s} {shp}{extra}")
    by = collections.defaultdict(float)
    for (name, _, _), (cnt, ms, b, fl) in agg.items():
        by[name] += ms / n
    print("# by entry point")
    for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f"{v:7.3f} ms/step  {k}")


if __name__ == "__main__":
    main()
