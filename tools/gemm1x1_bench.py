"""Per-call timing of the short-K GEMMs of UNet(3,2) at 3x512x512 B=8 (attention
1x1 fwd / input-grad, ConvTranspose fwd / input-grad) through the C-ABI, with
an optional check against torch fp32 ops on the GPU.
usage: python tools/gemm1x1_bench.py [--check] [--reps N] [--tune KEY=VAL,...]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import kernels as K  # noqa: E402
from vaeunet_amd import _lib  # noqa: E402
from vaeunet_amd.engine import w1x1_fwd, w1x1_dgrad, wT_fwd, wT_dgrad  # noqa: E402

B = 8
# (level, channels of g/x (= in//2), spatial of the skip)
LEVELS = [("up1", 512, 64), ("up2", 256, 128), ("up3", 128, 256), ("up4", 64, 512)]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def err(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tune", default="", help="KEY=VAL,... for vu_gemm_set_tuning")
    args = ap.parse_args()
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _lib.call("vu_gemm_set_tuning", int(k), int(v))
    dev = torch.device("cuda")
    torch.manual_seed(0)
    d = _lib.BF16
    tot = 0.0
    for name, C, S in LEVELS:
        Fi = C // 2
        x = torch.randn(B, C, S, S, device=dev).bfloat16().contiguous(memory_format=K.CL)
        w = (torch.randn(Fi, C, 1, 1, device=dev) / C ** 0.5)
        b = torch.randn(Fi, device=dev)
        u = K.empty_act(B, Fi, S, S, torch.bfloat16, dev)
        wf = w1x1_fwd(w, d)
        ms = timeit(lambda: K.gemm_fwd(K.gather1x1([x]), wf, Fi, u, d, bias=b, stats=True), args.reps)
        byts = B * S * S * (C + Fi) * 2
        fl = 2.0 * B * S * S * C * Fi
        line = f"{name} attn fwd  {C:4d}->{Fi:4d} @{S:3d}: {ms * 1e3:7.1f}us {byts / ms / 1e9:5.2f}TB/s {fl / ms / 1e9:6.0f}TF"
        if args.check:
            line += f" err {err(u, F.conv2d(x.float(), w.bfloat16().float(), b)):.1e}"
        tot += ms
        print(line, flush=True)
        du = torch.randn(B, Fi, S, S, device=dev).bfloat16().contiguous(memory_format=K.CL)
        dx = torch.randn(B, C, S, S, device=dev).bfloat16().contiguous(memory_format=K.CL)
        dx0 = dx.clone()
        wd = w1x1_dgrad(w, d)
        K.gemm_fwd(K.gather1x1([du]), wd, C, dx, d, accumulate=True)
        if args.check:
            ref = dx0.float() + torch.nn.grad.conv2d_input(dx.shape, w.bfloat16().float(), du.float())
            e1 = err(dx, ref)
        ms = timeit(lambda: K.gemm_fwd(K.gather1x1([du]), wd, C, dx, d, accumulate=True), args.reps)
        byts = B * S * S * (Fi + 2 * C) * 2
        line = f"{name} attn dgrad {Fi:4d}->{C:4d} @{S:3d}: {ms * 1e3:7.1f}us {byts / ms / 1e9:5.2f}TB/s {fl / ms / 1e9:6.0f}TF"
        if args.check:
            line += f" err {e1:.1e}"
        tot += ms
        print(line, flush=True)
        # ConvTranspose2d(2C -> C, 2, 2): x1 [B, 2C, S/2, S/2] -> u [B, C, S, S]
        ci, co, h = 2 * C, C, S // 2
        x1 = torch.randn(B, ci, h, h, device=dev).bfloat16().contiguous(memory_format=K.CL)
        wt = torch.randn(ci, co, 2, 2, device=dev) / ci ** 0.5
        bt = torch.randn(co, device=dev)
        uo = K.empty_act(B, co, S, S, torch.bfloat16, dev)
        wtf = wT_fwd(wt, d)
        fn = lambda: K.gemm_fwd(K.gather1x1([x1]), wtf, 4 * co, uo, d, bias=bt, convT=(S, S, 0, 0, co))  # noqa
        ms = timeit(fn, args.reps)
        byts = B * (h * h * ci + S * S * co) * 2
        fl = 2.0 * B * h * h * ci * 4 * co
        line = f"{name} convT fwd {ci:4d}->{co:4d} @{S:3d}: {ms * 1e3:7.1f}us {byts / ms / 1e9:5.2f}TB/s {fl / ms / 1e9:6.0f}TF"
        if args.check:
            line += f" err {err(uo, F.conv_transpose2d(x1.float(), wt.bfloat16().float(), bt, stride=2)):.1e}"
        tot += ms
        print(line, flush=True)
        duo = torch.randn(B, co, S, S, device=dev).bfloat16().contiguous(memory_format=K.CL)
        dx1 = K.empty_act(B, ci, h, h, torch.bfloat16, dev)
        wtd = wT_dgrad(wt, d)
        fn = lambda: K.gemm_fwd(K.gather_convT(duo, B, h, h), wtd, ci, dx1, d)  # noqa
        ms = timeit(fn, args.reps)
        line = f"{name} convT dgrad {co:4d}->{ci:4d} @{S:3d}: {ms * 1e3:7.1f}us {byts / ms / 1e9:5.2f}TB/s {fl / ms / 1e9:6.0f}TF"
        if args.check:
            ref = torch.nn.grad.conv2d_weight  # placeholder to keep flake quiet
            xr = x1.float().requires_grad_(True)
            yr = F.conv_transpose2d(xr, wt.bfloat16().float(), None, stride=2)
            yr.backward(duo.float())
            line += f" err {err(dx1, xr.grad):.1e}"
        tot += ms
        print(line, flush=True)
        # ConvTranspose2d weight gradient: x1^T x gather(du) (split-K slabs + reduce)
        gw = torch.empty(ci, co, 2, 2, device=dev)
        from vaeunet_amd.engine import convT_layout
        fn = lambda: K.gemm_wgrad(K.gather1x1([x1]), K.gather_convT(duo, B, h, h), ci, 4 * co, gw,  # noqa: E731
                                  convT_layout(gw), d, False)
        ms = timeit(fn, args.reps)
        line = f"{name} convT wgrad {ci:4d}x{4 * co:4d} @{h:3d}: {ms * 1e3:7.1f}us {byts / ms / 1e9:5.2f}TB/s {fl / ms / 1e9:6.0f}TF"
        tot += ms
        print(line, flush=True)
    print(f"TOTAL {tot:.3f} ms")


if __name__ == "__main__":
    main()
