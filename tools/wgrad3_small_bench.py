"""Per-call timing of the small-grid 3x3 weight gradients (ResNet34 encoder of
UNetResNet at B=8, 3x512^2 input: 64..512 channels at 128^2..16^2) through
vu_gemm_wgrad + vu_slab_reduce: the dispatcher's split count and forced ones
(the fp32 split slabs are ni x nj x 4 bytes each, so for these small pixel
counts their traffic rivals the operands').
usage: python tools/wgrad3_small_bench.py [--splits 1,2,4,8,16]"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import kernels as K  # noqa: E402
from vaeunet_amd import _lib  # noqa: E402
from vaeunet_amd.engine import conv_layout  # noqa: E402

B = 8
LAYERS = [("layer1", 64, 128), ("layer2", 128, 64), ("layer3", 256, 32), ("layer4", 512, 16)]


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


def forced(gp, gq, ni, nj, grad, splits):
    M = gp.N * gp.H * gp.W
    bi, bj = C.c_int(0), C.c_int(0)
    w = K.VuGemmWgrad()
    w.p, w.q, w.ni, w.nj = gp, gq, ni, nj
    kind = K.query("vu_gemm_wgrad_tile", C.byref(w), _lib.BF16, C.byref(bi), C.byref(bj))
    gran = 128 if kind == 3 else 64
    mps = ((-(-M // splits)) + gran - 1) // gran * gran
    w.splits, w.m_per_split = -(-M // mps), mps
    slab = torch.empty((w.splits, ni, nj), dtype=torch.float32, device=grad.device)
    w.out = slab.data_ptr()
    s_i, s_tap, s_c = conv_layout(grad)

    def fn():
        _lib.call("vu_gemm_wgrad", C.byref(w), _lib.BF16, K.stream())
        _lib.call("vu_slab_reduce", K.ptr(slab), w.splits, ni, nj, gq.C, gq.C, s_i, s_tap, s_c, K.ptr(grad), 0,
                  K.stream())
    return fn, kind, w.splits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", default="1,2,4,8,16,32")
    args = ap.parse_args()
    dev = torch.device("cuda")
    for name, c, h in LAYERS:
        x = torch.randn(B, c, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=K.CL)
        dy = torch.randn(B, c, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=K.CL)
        g = torch.empty(c, c, 3, 3, device=dev)
        fl = 2.0 * B * h * h * c * 9 * c
        ms = timeit(lambda: K.gemm_wgrad(K.gather1x1([dy]), K.gather3x3([x]), c, 9 * c, g, conv_layout(g),
                                         _lib.BF16, False))
        ref = g.clone()
        line = f"{name} {c:4d}@{h:3d} | dispatch {ms * 1e3:6.1f}us {fl / ms / 1e9:5.0f}TF"
        for s in map(int, args.splits.split(",")):
            fn, kind, sp = forced(K.gather1x1([dy]), K.gather3x3([x]), c, 9 * c, g, s)
            t = timeit(fn)
            err = ((g - ref).abs().max() / ref.abs().max()).item()
            line += f" | s{sp} k{kind} {t * 1e3:6.1f}us" + (" !!!" if err > 1e-3 else "")
        print(line, flush=True)


if __name__ == "__main__":
    main()
