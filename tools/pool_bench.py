"""Per-call timing of the Down max-pool with its producing BatchNorm fused
(vu_bn_apply_maxpool2) against vu_bn_apply + vu_maxpool2_fwd, and of the
backward pair (vu_maxpool2_bwd + BN backward), at the UNet(3,2) B=8 encoder
shapes.  usage: python tools/pool_bench.py"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import kernels as K  # noqa: E402
from vaeunet_amd import _lib  # noqa: E402

SHAPES = [(8, 64, 512, 512), (8, 128, 256, 256), (8, 256, 128, 128), (8, 512, 64, 64)]


def timeit(fn, reps=10):
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
    argparse.ArgumentParser().parse_args()
    dev = torch.device("cuda")
    d = _lib.BF16
    for N, C, H, W in SHAPES:
        y = K.empty_act(N, C, H, W, torch.bfloat16, dev).normal_()
        coef = torch.stack([torch.rand(C) + 0.5, torch.randn(C) * 0.3, torch.randn(C) * 0.1,
                            torch.rand(C) + 0.5]).to(dev)
        a, p = torch.empty_like(y), K.empty_act(N, C, H // 2, W // 2, y.dtype, dev)
        dp, add = torch.randn_like(p), torch.randn_like(y)
        dx, out = torch.empty_like(y), torch.empty_like(y)
        gamma, dg, db = torch.ones(C, device=dev), torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        t_ff = timeit(lambda: K.bn_apply_maxpool(y, a, p, coef, True, d))
        t_fu = timeit(lambda: (K.bn_apply(y, a, coef, True, d), K.maxpool_fwd(a, d)))
        t_bu = timeit(lambda: (K.maxpool_bwd(a, dp, dx, add, d),
                               K.bn_backward(dx, y, coef, gamma, True, dg, db, False, out, d)))
        line = (f"{N}x{C}x{H}x{W}: fwd fused {t_ff:6.1f} / apply+pool {t_fu:6.1f} us | bwd pool+reduce+apply "
                f"{t_bu:6.1f} us")
        print(line, flush=True)


if __name__ == "__main__":
    main()
