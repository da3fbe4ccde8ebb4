"""Where does the HIP fp32 (parity-mode) path's excess error come from?

VERDICT r5 "do this" 1: profiles/r5a_psi_probe.log shows the HIP fp32
forward at 1.6-2.1x the fp32 oracle's error at every attention gate.  This
probe isolates single ops on random operands and reports, for each, the
relative error against an fp64 evaluation of the same operands -- the HIP
kernel's and torch CPU fp32's (the oracle's arithmetic: oneDNN / ATen) --
and their ratio:

  conv3x3 forward / input gradient / weight gradient at K = 9*Cin from 72 to
  9216 (the generic parity-mode GEMM, fp32 MFMA 16x16x4), conv + train-mode
  BatchNorm + ReLU (the statistics epilogue, fp64 finalize, apply pass).

A ratio that grows with K points at the summation order; a constant one at
the per-operation rounding of the MFMA.  Test infrastructure only (imports
nothing from oracle/); run on the GPU box:
    python tools/fp32_err_probe.py > gpurun_out/fp32_err_probe.log
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CL = torch.channels_last


def rel(a, ref):
    a = a.double().cpu()
    return float((a - ref).norm() / ref.norm().clamp_min(1e-300))


def rel_max(a, ref):
    a = a.double().cpu()
    return float((a - ref).abs().max() / ref.abs().max().clamp_min(1e-300))


def line(name, hip, cpu, extra=""):
    r = hip[0] / max(cpu[0], 1e-300)
    print(f"{name:44s} rms HIP {hip[0]:.3e} CPU32 {cpu[0]:.3e} ratio {r:5.2f} | "
          f"max HIP {hip[1]:.3e} CPU32 {cpu[1]:.3e} {extra}", flush=True)
    return r


def conv_cases(dev, seed, mfma_only=False):
    from vaeunet_amd import ops  # noqa: F401 (registers vaeunet::*)
    g = torch.Generator().manual_seed(seed)
    cases = [(2, 8, 64, 128), (2, 64, 64, 128), (2, 128, 64, 128), (2, 256, 256, 64), (2, 512, 512, 32),
             (2, 1024, 512, 32)]
    for N, ci, co, H in cases:
        x = torch.randn(N, ci, H, H, generator=g)
        w = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
        dy = torch.randn(N, co, H, H, generator=g)
        x64, w64, dy64 = x.double(), w.double(), dy.double()
        xd = x.to(dev).contiguous(memory_format=CL)
        wd = w.to(dev)
        dyd = dy.to(dev).contiguous(memory_format=CL)
        tag = f"{N}x{ci}->{co}@{H}^2 K={9 * ci}"
        # forward
        y64 = F.conv2d(x64, w64, padding=1)
        yh = torch.ops.vaeunet.conv3x3_fwd(xd, wd, None)
        yc = F.conv2d(x, w, padding=1)
        line("fwd   " + tag, (rel(yh, y64), rel_max(yh, y64)), (rel(yc, y64), rel_max(yc, y64)))
        # input gradient
        dx64 = torch.nn.grad.conv2d_input(x.shape, w64, dy64, padding=1)
        dxh = torch.ops.vaeunet.conv3x3_dgrad(dyd, wd)
        dxc = torch.nn.grad.conv2d_input(x.shape, w, dy, padding=1)
        line("dgrad " + tag, (rel(dxh, dx64), rel_max(dxh, dx64)), (rel(dxc, dx64), rel_max(dxc, dx64)))
        # weight gradient (K = N*H*W pixels)
        dw64 = torch.nn.grad.conv2d_weight(x64, w.shape, dy64, padding=1)
        dwh = torch.ops.vaeunet.conv3x3_wgrad(xd, dyd)
        dwc = torch.nn.grad.conv2d_weight(x, w.shape, dy, padding=1)
        line("wgrad " + tag + f" P={N * H * H}", (rel(dwh, dw64), rel_max(dwh, dw64)),
             (rel(dwc, dw64), rel_max(dwc, dw64)))
        torch.cuda.synchronize()


def matmul_cases(dev, seed):
    """A plain [M, K] x [K, N] contraction through the 1x1 path of the same
    generic kernel is not exposed as an op; torch's own GPU fp32 matmul
    (hipBLASLt, fp32 MFMA) is printed instead as a second GPU data point."""
    g = torch.Generator().manual_seed(seed)
    torch.backends.cuda.matmul.allow_tf32 = False
    for K in (64, 576, 2304, 9216):
        a = torch.randn(4096, K, generator=g)
        b = torch.randn(K, 256, generator=g) / K ** 0.5
        r64 = a.double() @ b.double()
        rg = (a.to(dev) @ b.to(dev))
        rc = a @ b
        line(f"torch.cuda matmul fp32 K={K}", (rel(rg, r64), rel_max(rg, r64)), (rel(rc, r64), rel_max(rc, r64)))


def fma_chain_reference(seed):
    """What a strict sequential fp32 FMA chain gives on the same data (numpy,
    in the CPU): the floor a VALU FMA kernel would have."""
    import numpy as np
    g = np.random.default_rng(seed)
    for K in (576, 2304, 9216):
        a = g.standard_normal((256, K)).astype(np.float32)
        b = (g.standard_normal((K, 64)) / K ** 0.5).astype(np.float32)
        r64 = a.astype(np.float64) @ b.astype(np.float64)
        acc = np.zeros((256, 64), np.float32)
        for k in range(K):
            acc = (acc.astype(np.float64) + np.outer(a[:, k], b[k]).astype(np.float64)).astype(np.float32)
        seq = float(np.linalg.norm(acc - r64) / np.linalg.norm(r64))
        blas = float(np.linalg.norm((a @ b).astype(np.float64) - r64) / np.linalg.norm(r64))
        print(f"numpy K={K:5d}: sequential fp32 FMA chain rms {seq:.3e}   numpy BLAS fp32 {blas:.3e} "
              f"ratio {seq / blas:5.2f}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-chain", action="store_true")
    args = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    t0 = time.time()
    if not args.no_chain:
        fma_chain_reference(args.seed)
    if torch.cuda.is_available():
        dev = torch.device("cuda")
        conv_cases(dev, args.seed)
        matmul_cases(dev, args.seed)
    print(f"done {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
