"""Per-call timing of the BatchNorm / channel reductions at the UNet(3,2) B=8
layer shapes (vu_bn_finalize, vu_bn_bwd_reduce + apply, vu_chan_sum).
usage: python tools/red_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import kernels as K  # noqa: E402

SHAPES = [(8, 64, 512, 512), (8, 128, 256, 256), (8, 256, 128, 128), (8, 512, 64, 64), (8, 1024, 32, 32),
          (8, 32, 512, 512)]


def timeit(fn, reps=20):
    """GPU time per call: `reps` calls captured in one HIP graph (the tiny
    finalize launches would otherwise measure the host enqueue)."""
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
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = torch.device("cuda")
    tot = 0.0
    for N, C, H, W in SHAPES:
        x = K.empty_act(N, C, H, W, torch.bfloat16, dev).normal_()
        dy = K.empty_act(N, C, H, W, torch.bfloat16, dev).normal_()
        dx = torch.empty_like(x)
        tiles = N * H * W // 128
        st = K.Stats(torch.rand(tiles, C, device=dev) * 128, torch.rand(tiles, C, device=dev) * 128, tiles, 128,
                     N * H * W)
        g, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.int64, device=dev)
        coef = K.bn_finalize(st, C, g, b, rm, rv, nbt, 0.1, 1e-5)
        t_fin = timeit(lambda: K.bn_finalize(st, C, g, b, rm, rv, nbt, 0.1, 1e-5))
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        t_bwd = timeit(lambda: K.bn_backward(dy, x, coef, g, True, dg, db, False, dx, 1))
        out = torch.zeros(C, device=dev)
        t_sum = timeit(lambda: K.chan_sum(x, out, False, 1))
        tot += t_fin + t_bwd + t_sum
        print(f"{N}x{C}x{H}x{W}: finalize {t_fin:6.1f}us  bwd(reduce+apply) {t_bwd:6.1f}us  chan_sum {t_sum:6.1f}us",
              flush=True)
    print(f"TOTAL {tot:.1f} us")


if __name__ == "__main__":
    main()
