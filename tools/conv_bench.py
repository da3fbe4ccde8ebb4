"""Per-layer timing of the 3x3 implicit-GEMM kernels at the UNet(3,2)
3x512x512 B=8 shapes (fwd, input-grad, weight-grad), through the C-ABI.
Optionally checks each result against torch fp32 conv2d on the GPU and times
MIOpen's bf16 conv for comparison.

usage: python tools/conv_bench.py [--check] [--miopen] [--only fwd,dgrad,wgrad] [--reps N]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import kernels as K  # noqa: E402
from vaeunet_amd import _lib  # noqa: E402
from vaeunet_amd.engine import w3x3_fwd, w3x3_dgrad, conv_layout  # noqa: E402

B = 8
# (name, cin sources, cout, H) for the 3x3 convs of UNet(3,2) (inc.0 excluded)
LAYERS = [
    ("inc.2", [64], 64, 512), ("down1.1", [64], 128, 256), ("down1.2", [128], 128, 256),
    ("down2.1", [128], 256, 128), ("down2.2", [256], 256, 128),
    ("down3.1", [256], 512, 64), ("down3.2", [512], 512, 64),
    ("down4.1", [512], 1024, 32), ("down4.2", [1024], 1024, 32),
    ("up1.1", [512, 512], 512, 64), ("up1.2", [512], 512, 64),
    ("up2.1", [256, 256], 256, 128), ("up2.2", [256], 256, 128),
    ("up3.1", [128, 128], 128, 256), ("up3.2", [128], 128, 256),
    ("up4.1", [64, 64], 64, 512), ("up4.2", [64], 64, 512),
]


def timeit(fn, reps):
    """GPU time per call: the calls are captured in one HIP graph and replayed
    (timed eagerly, the Python + ctypes enqueue -- the statistics buffers'
    allocation included -- inflated the shorter launches).  Note: with
    statistics every captured call allocates fresh partial buffers, and the
    replay then shows inter-kernel gaps the training step does not have
    (down3.2: kernel durations equal under rocprofv3, graph time +17 us);
    compare kernel durations (rocprofv3 --kernel-trace) for the epilogue cost."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--miopen", action="store_true")
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--layers", default="")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tune", default="", help="KEY=VAL,... for vu_gemm_set_tuning (include/vaeunet.h)")
    args = ap.parse_args()
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _lib.call("vu_gemm_set_tuning", int(k), int(v))
    kinds = args.only.split(",")
    dev = torch.device("cuda")
    torch.manual_seed(0)
    d = _lib.BF16
    tot = {k: [0.0, 0.0] for k in kinds}
    for name, cins, co, H in LAYERS:
        if args.layers and name not in args.layers.split(","):
            continue
        srcs = [torch.randn(B, c, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=K.CL)
                for c in cins]
        ci = sum(cins)
        conv = torch.nn.Conv2d(ci, co, 3, padding=1, bias=False).to(dev)
        w = conv.weight
        dy = torch.randn(B, co, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=K.CL)
        fl = 2.0 * B * H * H * co * 9 * ci
        line = f"{name:8s} {ci:5d}->{co:5d} @{H:3d}"
        for kind in kinds:
            if kind in ("fwd", "fwdnostats"):
                y = K.empty_act(B, co, H, H, torch.bfloat16, dev)
                wf = w3x3_fwd(w, d)
                st = kind == "fwd"
                fn = lambda: K.gemm_fwd(K.gather3x3(srcs), wf, co, y, d, stats=st)  # noqa: E731
            elif kind == "dgrad":
                dx = K.empty_act(B, ci, H, H, torch.bfloat16, dev)
                wd = w3x3_dgrad(w, d)
                fn = lambda: K.gemm_fwd(K.gather3x3([dy]), wd, ci, dx, d, kind="dgrad")  # noqa: E731
            else:
                g = torch.empty_like(w)
                fn = lambda: K.gemm_wgrad(K.gather1x1([dy]), K.gather3x3(srcs), co, 9 * ci, g,  # noqa: E731
                                          conv_layout(g), d, False)
            ms = timeit(fn, args.reps)
            tot[kind][0] += fl
            tot[kind][1] += ms
            line += f" | {kind} {ms * 1e3:7.1f}us {fl / ms / 1e9:6.0f}TF"
            if args.check:
                xs = torch.cat([s.float() for s in srcs], 1)
                if kind == "fwd":
                    ref = F.conv2d(xs, w.bfloat16().float(), padding=1)
                    out = y.float()
                elif kind == "dgrad":
                    ref = torch.nn.grad.conv2d_input(xs.shape, w.bfloat16().float(), dy.float(), padding=1)
                    out = dx.float()
                else:
                    ref = torch.nn.grad.conv2d_weight(xs, w.shape, dy.float(), padding=1)
                    out = g
                err = ((out - ref).abs().max() / ref.abs().max()).item()
                line += f" err {err:.1e}"
                if err > 2e-2:
                    line += " !!!"
            if args.miopen and kind == "fwd":
                xc = torch.cat(srcs, 1).contiguous(memory_format=K.CL)
                wb = w.bfloat16().contiguous(memory_format=K.CL)
                ms2 = timeit(lambda: F.conv2d(xc, wb, padding=1), args.reps)
                line += f" [miopen {fl / ms2 / 1e9:5.0f}TF]"
        print(line, flush=True)
    for k, (f, t) in tot.items():
        if t:
            print(f"TOTAL {k}: {t:.3f} ms, {f / t / 1e9:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
