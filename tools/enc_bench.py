"""Per-layer timing of the small-grid 3x3 convolutions (the ResNet34 encoder of
UNetResNet and the UNet(3,2) bottleneck, B=8, 3x512^2 input) through the
C-ABI: forward and input gradient.

usage: python tools/enc_bench.py [--tune KEY=VAL,...] [--phases]
--phases: one forward per layer on the small-grid kernel's timing mode
(VU_TUNE_V7_XM = 5): the share of each phase of its waves' cycles
(also times the UNet(3,2) small-grid layers: down4 and up1 at B=8)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import kernels as K  # noqa: E402
from vaeunet_amd import _lib  # noqa: E402
from vaeunet_amd.engine import w3x3_fwd, w3x3_dgrad  # noqa: E402

B = 8
LAYERS = [("layer1", 64, 64, 128), ("layer2", 128, 128, 64), ("layer3", 256, 256, 32), ("layer4", 512, 512, 16),
          # UNet(3,2) small grids: down4 conv1 / conv2, up1 conv2
          ("unet.down4a", 512, 1024, 32), ("unet.down4b", 1024, 1024, 32), ("unet.up1b", 512, 512, 64),
          # UNetResNet decoder block 1 (32^2): the conv1 input gradient (512 -> 832 padded concat channels)
          ("dec1.conv1_dgrad", 512, 832, 32)]


def timeit(fn, reps=20):
    """GPU time per call: the calls are captured in one HIP graph and replayed
    (timed eagerly, the Python + ctypes enqueue of a ~10 us kernel is the
    bottleneck, not the kernel)."""
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
    ap.add_argument("--tune", default="")
    ap.add_argument("--wsplit", type=int, default=0, help="cap on the weight-gradient split-K ways (A/B)")
    ap.add_argument("--phases", action="store_true")
    args = ap.parse_args()
    if args.phases:
        return phases()
    K.WGRAD_SPLIT_CAP = args.wsplit
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _lib.call("vu_gemm_set_tuning", int(k), int(v))
    dev = torch.device("cuda")
    d = _lib.BF16
    tot = 0.0
    for name, ci, co, S in LAYERS:
        x = K.empty_act(B, ci, S, S, torch.bfloat16, dev).normal_()
        w = torch.randn(co, ci, 3, 3, device=dev) / (3 * ci ** 0.5)
        y = K.empty_act(B, co, S, S, torch.bfloat16, dev)
        fl = 2.0 * B * S * S * co * ci * 9
        import ctypes as C
        a = _lib.VuGemmFwd()
        a.a = K.gather3x3([x])
        a.b = w3x3_fwd(w, d).data_ptr()
        a.ldb = 9 * ci
        a.ncol = co
        a.out = y.data_ptr()
        a.out_stride = K.pstride(y)
        a.out_mode = 0
        diag = (K.query("vu_gemm_fwd_row_tile", C.byref(a), d), K.query("vu_gemm_fwd_workspace_bytes", C.byref(a), d),
                "kernel", K.query("vu_gemm_fwd_kernel", C.byref(a), d))
        tf = timeit(lambda: K.gemm_fwd(K.gather3x3([x]), w3x3_fwd(w, d), co, y, d, stats=True))
        dx = K.empty_act(B, ci, S, S, torch.bfloat16, dev)
        tb = timeit(lambda: K.gemm_fwd(K.gather3x3([y]), w3x3_dgrad(w, d), ci, dx, d, kind="dgrad"))
        gw = torch.zeros(co, ci, 3, 3, device=dev)
        from vaeunet_amd.engine import conv_layout
        tw = timeit(lambda: K.gemm_wgrad(K.gather1x1([y]), K.gather3x3([x]), co, 9 * ci, gw, conv_layout(gw), d,
                                         False))
        tot += tf + tb + tw
        print(f"{name} {ci}->{co} @{S:3d} | fwd {tf * 1e3:7.1f}us {fl / tf / 1e9:6.0f}TF | "
              f"dgrad {tb * 1e3:7.1f}us {fl / tb / 1e9:6.0f}TF | wgrad+reduce {tw * 1e3:7.1f}us "
              f"{fl / tw / 1e9:6.0f}TF | row_tile,ws {diag}", flush=True)
    print(f"TOTAL {tot:.3f} ms")


def phases():
    import ctypes as C
    import numpy as np
    dev, d = torch.device("cuda"), _lib.BF16
    lib = _lib.lib()
    names = ("prologue", "reads+DMA wait", "barrier 1", "MFMA issue", "barrier 2", "epilogue")
    for name, ci, co, S in LAYERS[:4] + LAYERS[5:6]:
        x = K.empty_act(B, ci, S, S, torch.bfloat16, dev).normal_()
        w = torch.randn(co, ci, 3, 3, device=dev) / (3 * ci ** 0.5)
        y = K.empty_act(B, co, S, S, torch.bfloat16, dev)
        a = _lib.VuGemmFwd()
        a.a = K.gather3x3([x])
        a.b = w3x3_fwd(w, d).data_ptr()
        a.ldb, a.ncol, a.out, a.out_stride, a.out_mode = 9 * ci, co, y.data_ptr(), K.pstride(y), 0
        kern = K.query("vu_gemm_fwd_kernel", C.byref(a), d)
        if kern != 7:
            print(f"{name}: kernel {kern}, not the small-grid kernel (7)")
            continue
        _lib.call("vu_gemm_set_tuning", 33, 1)   # VU_TUNE_UNSAFE: experiment modes allowed
        _lib.call("vu_gemm_set_tuning", 18, 5)   # VU_TUNE_V7_XM
        try:
            for _ in range(3):
                K.gemm_fwd(K.gather3x3([x]), w3x3_fwd(w, d), co, y, d, stats=True)
            torch.cuda.synchronize()
            buf = (C.c_ulonglong * (64 * 64))()
            _lib.call("vu_sg_debug_read", buf, 64 * 64)
        finally:
            _lib.call("vu_gemm_set_tuning", 18, 0)
        v = np.frombuffer(buf, dtype=np.uint64).reshape(64, 8, 8).astype(np.float64)
        tot = v[:, :, :6].sum(-1)
        ok = tot > 0
        if not ok.any():
            print(f"{name}: no counters (split-K launch: the timing mode is unsplit only)")
            continue
        share = (v[:, :, :6][ok] / tot[ok][:, None]).mean(0)
        steps = v[:, :, 6][ok].mean()
        print(f"{name} {ci}->{co} @{S}: kernel {kern}, {steps:.0f} steps, {tot[ok].mean():.0f} cycles/wave: " +
              ", ".join(f"{n} {100 * f:.1f}%" for n, f in zip(names, share)) +
              f" | per step {(v[:, :, 1:5].sum(-1)[ok] / np.maximum(v[:, :, 6][ok], 1)).mean():.0f} cycles", flush=True)


if __name__ == "__main__":
    main()
