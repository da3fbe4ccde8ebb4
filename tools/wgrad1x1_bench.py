"""Per-call timing of the 1x1 weight gradients of the attention gates of
UNet(3,2) at 3x512x512 B=8 (W_g / W_x: dy [B,F_int,H,W] x x [B,C,H,W]) through
vu_gemm_wgrad + vu_slab_reduce, for the dispatcher's split count and forced
ones; reports the HBM rate of the operand streams.
usage: python tools/wgrad1x1_bench.py [--splits 64,128,256,512]"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import kernels as K  # noqa: E402
from vaeunet_amd import _lib  # noqa: E402

B = 8
LEVELS = [("up1", 512, 64), ("up2", 256, 128), ("up3", 128, 256), ("up4", 64, 512)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def run(gp, gq, ni, nj, splits, slab):
    M = gp.N * gp.H * gp.W
    w = K.VuGemmWgrad()
    w.p, w.q, w.ni, w.nj = gp, gq, ni, nj
    mps = ((-(-M // splits)) + 63) // 64 * 64
    w.splits, w.m_per_split = -(-M // mps), mps
    w.out = slab.data_ptr()
    _lib.call("vu_gemm_wgrad", C.byref(w), _lib.BF16, K.stream())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", default="64,128,256,512,1024")
    ap.add_argument("--convt", action="store_true", help="the ConvTranspose(2,2) weight gradients instead")
    args = ap.parse_args()
    dev = torch.device("cuda")
    if args.convt:
        # up1..up4: ConvT(cin -> cin/2) on an h x h input, dW[ci][(a,b,co)] = sum x1 * dU
        for name, cin, h in [("up1", 1024, 32), ("up2", 512, 64), ("up3", 256, 128), ("up4", 128, 256)]:
            cu = cin // 2
            x1 = torch.randn(B, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=K.CL)
            du = torch.randn(B, cu, 2 * h, 2 * h, device=dev).to(torch.bfloat16).contiguous(memory_format=K.CL)
            g = torch.empty(cin, cu, 2, 2, device=dev)
            fl = 2.0 * B * h * h * cin * 4 * cu
            from vaeunet_amd.engine import convT_layout
            ms = timeit(lambda: K.gemm_wgrad(K.gather1x1([x1]), K.gather_convT(du, B, h, h, 0, 0), cin, 4 * cu, g,
                                             convT_layout(g), _lib.BF16, False))
            line = f"{name} {cin:4d}x{4 * cu:4d} M={B * h * h:7d} | dispatch {ms * 1e3:7.1f}us {fl / ms / 1e9:5.0f}TF"
            slab = torch.empty(max(int(v) for v in args.splits.split(",")), cin, 4 * cu, device=dev)
            for s in [int(v) for v in args.splits.split(",")]:
                ms = timeit(lambda: run(K.gather1x1([x1]), K.gather_convT(du, B, h, h, 0, 0), cin, 4 * cu, s, slab))
                line += f" | s{s} {ms * 1e3:6.1f}us"
            print(line, flush=True)
        return
    for name, c, h in LEVELS:
        fi = c // 2
        dy = torch.randn(B, fi, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=K.CL)
        x = torch.randn(B, c, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=K.CL)
        g = torch.empty(fi, c, 1, 1, device=dev)
        byts = dy.numel() * 2 + x.numel() * 2
        ms = timeit(lambda: K.gemm_wgrad(K.gather1x1([dy]), K.gather1x1([x]), fi, c, g, (c, 0, 1), _lib.BF16, False))
        line = f"{name} {fi:4d}x{c:4d} @{h:3d} | dispatch {ms * 1e3:7.1f}us {byts / ms / 1e6:6.0f}GB/s"
        slab = torch.empty(1024, fi, c, device=dev)
        for s in [int(v) for v in args.splits.split(",")]:
            ms = timeit(lambda: run(K.gather1x1([dy]), K.gather1x1([x]), fi, c, s, slab))
            line += f" | s{s} {ms * 1e3:6.1f}us"
        print(line, flush=True)


if __name__ == "__main__":
    main()
