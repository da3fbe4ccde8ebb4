"""Times the latent-shortcut kernels (csrc/zbias.hip) on the config-3
DecoderBlock shapes (UNetResNet at 256^2: conv1 co 512/256/128/64 at
32/64/128/256, L = 32), alone and per job, so rocprofv3 --kernel-trace
--stats separates them.  usage: python tools/zbias_bench.py [--n 8] [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = ((512, 32, 768 - 512), (256, 64, 640 - 256), (128, 128, 320 - 128), (64, 256, 192 - 64))  # co, H, lead


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--L", type=int, default=32)
    ap.add_argument("--debug", default="0", help="comma list of vu_zbias_set_debug modes to time "
                    "(1 skip staging, 2 skip the table / dW loop, 4 skip R, 8 skip dc; results wrong)")
    args = ap.parse_args()
    from vaeunet_amd import _lib, kernels as K
    N, L, dev = args.n, args.L, "cuda"
    g = torch.Generator().manual_seed(3)
    keep, jobs = [], []
    for co, H, lead in SHAPES:
        w = (torch.randn(co, lead + L, 3, 3, generator=g) / 30).to(dev)
        act = torch.rand(N, L, generator=g).to(dev)
        table = torch.empty((N, 9, co), device=dev)
        dy = torch.randn(N, co, H, H, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dw = torch.zeros_like(w)
        part = torch.empty(N * 32 * L, device=dev)
        rs = torch.empty(K.query("vu_zbias_rs_floats", N, co, H, H), device=dev)
        keep += [w, act, table, dy, dw, part, rs]
        j = _lib.VuZbJob()
        j.w = w.data_ptr()
        j.ws_co, j.ws_ci, j.ws_ky, j.ws_kx = w.stride()
        j.cz0, j.L, j.co, j.H, j.W = lead, L, co, H, H
        j.act, j.table = act.data_ptr(), table.data_ptr()
        j.dy, j.dy_stride = dy.data_ptr(), K.pstride(dy)
        j.rs, j.part, j.dw, j.grad_acc = rs.data_ptr(), part.data_ptr(), dw.data_ptr(), 0
        jobs.append(j)
    arr = (_lib.VuZbJob * len(jobs))(*jobs)
    st = K.stream()
    for mode in (int(m) for m in args.debug.split(",")):
        _lib.lib().vu_zbias_set_debug(mode)
        print(f"debug mode {mode}", flush=True)
        run(args, N, jobs, st)
    _lib.lib().vu_zbias_set_debug(0)
    del arr


def run(args, N, jobs, st):
    from vaeunet_amd import _lib, kernels as K
    for tag, sub in (("all", list(range(len(jobs)))),) + tuple((f"co{SHAPES[i][0]}", [i]) for i in range(len(jobs))):
        a = (_lib.VuZbJob * len(sub))(*[jobs[i] for i in sub])
        for _ in range(3):
            K.call("vu_zbias_fwd", a, len(sub), N, st)
            K.call("vu_zbias_bwd", a, len(sub), N, 1, st)
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        for _ in range(args.reps):
            K.call("vu_zbias_fwd", a, len(sub), N, st)
        e1.record()
        for _ in range(args.reps):
            K.call("vu_zbias_bwd", a, len(sub), N, 1, st)
        e2.record()
        torch.cuda.synchronize()
        dyb = sum(N * SHAPES[i][0] * SHAPES[i][1] ** 2 * 2 for i in sub)
        tb = e1.elapsed_time(e2) * 1e3 / args.reps
        print(f"{tag:6s} N={N}: fwd {e0.elapsed_time(e1) * 1e3 / args.reps:7.1f} us  bwd {tb:7.1f} us "
              f"(dy {dyb / 1e6:.1f} MB -> {dyb / tb / 1e3:.0f} GB/s over the whole backward)", flush=True)


if __name__ == "__main__":
    main()
