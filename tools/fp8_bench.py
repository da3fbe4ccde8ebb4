"""BASELINE.json configs[4]: fp8 (e4m3) NHWC implicit-GEMM 3x3 conv forward on
the gfx950 f8f6f4 MFMA at 3x1024x1024 -- every 3x3 conv of UNet(3,2) except
inc.0 at the 1024^2 layer shapes (1,472.5 GFLOP/img of 3x3
forward), timed per layer with HIP events, against the bf16 halo kernels on
the same shapes; error vs the unquantised fp32 conv reported per layer.

--double: the DoubleConv blocks instead (conv -> BN -> ReLU, twice, train-mode
BatchNorm), timed end to end INCLUDING every activation quantisation: the
delayed-scaling fp8 path (fp8.double_conv_forward: one-pass input quantise,
BN1 apply fused with the e4m3 quantise), the just-in-time fp8 path and the
chained fp8 block (e4m3 in from the producing block, BN2 apply fused with
the e4m3 quantise of the output: the steady state of consecutive fp8
blocks), the same chained block just in time (the input quantised by the
producer with its exact amax, the output's exact amax from conv2's min / max
epilogue: no history, no calibration pass) against the bf16 engine path (engine.double_conv_fwd) on the same
module.

usage: python tools/fp8_bench.py [--batch 2] [--reps 20] [--layers inc.2,...] [--double] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import _lib, fp8  # noqa: E402
from vaeunet_amd import kernels as K  # noqa: E402
from vaeunet_amd.engine import w3x3_fwd  # noqa: E402

PEAK_FP8, PEAK_BF16 = 5000.0, 2500.0
# (name, cin sources, cout, H) of the DoubleConv blocks of UNet(3,2) at 1024^2
# (inc: 3 input channels, not an fp8 shape; its conv2 is inc.2 above)
BLOCKS = [
    ("down1", [64], 128, 512), ("down2", [128], 256, 256), ("down3", [256], 512, 128),
    ("down4", [512], 1024, 64), ("up1", [512, 512], 512, 128), ("up2", [256, 256], 256, 256),
    ("up3", [128, 128], 128, 512), ("up4", [64, 64], 64, 1024),
]


def double_main(args):
    from vaeunet_amd import DoubleConv
    from vaeunet_amd import engine as E
    dev = torch.device("cuda")
    B = args.batch
    rows, tot = [], {"bf16": 0.0, "fp8": 0.0, "fp8_jit": 0.0, "fp8_chain": 0.0, "fp8_jit_chain": 0.0, "fl": 0.0}
    for name, cins, co, H in BLOCKS:
        if args.layers and name not in args.layers.split(","):
            continue
        ci = sum(cins)
        mod = DoubleConv(ci, co).to(dev).train()
        srcs = [torch.randn(B, c, H, H, device=dev).relu().to(torch.bfloat16).contiguous(memory_format=K.CL)
                for c in cins]
        fl = 2.0 * B * H * H * co * 9 * (ci + co)
        M = E.Mode(_lib.BF16, dev)

        def bf16():
            E.double_conv_fwd(M, mod.double_conv, srcs)
        msb = timeit(bf16, args.reps)
        ms8 = timeit(lambda: fp8.double_conv_forward(mod, srcs, delayed=True), args.reps)
        msj = timeit(lambda: fp8.double_conv_forward(mod, srcs, delayed=False), args.reps)
        # chained: input already e4m3 (quantised by the producing block), output e4m3
        xq = fp8.double_conv_forward(mod, srcs, delayed=True)  # (warm the scales)
        dsq = fp8.DelayedScale(dev)
        fp8.calibrate(srcs[0], None, False, dsq)
        qin = [fp8.bn_apply_quant(t, None, False, dsq)[0] for t in srcs]
        qdq = fp8.bn_apply_quant(srcs[0], None, False, dsq)[1]
        del xq
        msc = timeit(lambda: fp8.double_conv_forward(mod, None, delayed=True, x_q=(qin, qdq), out_fp8=True), args.reps)
        # chained just in time: the producer's e4m3 output (exact just-in-time
        # scale) in, e4m3 out with the exact scale of relu(BN2(y2)) from conv2's
        # min / max epilogue -- every call self-contained, no history
        dsj = fp8.DelayedScale(dev)
        for t in srcs:
            fp8.calibrate(t, None, False, dsj)
        qj = []
        for t in srcs:
            q_, jdq = fp8.bn_apply_quant(t, None, False, dsj)
            qj.append(q_)
        msjc = timeit(lambda: fp8.double_conv_forward(mod, None, x_q=(qj, jdq), out_fp8=True), args.reps)
        with torch.no_grad():
            yb = E.double_conv_fwd(M, mod.double_conv, srcs)[0].float()
            y8 = fp8.double_conv_forward(mod, srcs, delayed=True).float()
        row = {"block": name, "cin": ci, "cout": co, "hw": H, "bf16_us": round(msb * 1e3, 1),
               "fp8_us": round(ms8 * 1e3, 1), "fp8_jit_us": round(msj * 1e3, 1),
               "fp8_chain_us": round(msc * 1e3, 1), "fp8_jit_chain_us": round(msjc * 1e3, 1),
               "speedup": round(msb / ms8, 3), "speedup_jit": round(msb / msj, 3),
               "speedup_chain": round(msb / msc, 3), "speedup_jit_chain": round(msb / msjc, 3),
               "rel_err_vs_bf16": round(((y8 - yb).abs().max() / yb.abs().max()).item(), 4)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        tot["bf16"] += msb
        tot["fp8"] += ms8
        tot["fp8_jit"] += msj
        tot["fp8_chain"] += msc
        tot["fp8_jit_chain"] += msjc
        tot["fl"] += fl
        del srcs, mod
        torch.cuda.empty_cache()
    summ = {"batch": B, "image": "3x1024x1024", "blocks": len(rows), "bf16_ms": round(tot["bf16"], 3),
            "fp8_ms": round(tot["fp8"], 3), "fp8_jit_ms": round(tot["fp8_jit"], 3),
            "fp8_chain_ms": round(tot["fp8_chain"], 3),
            "speedup": round(tot["bf16"] / tot["fp8"], 3), "speedup_jit": round(tot["bf16"] / tot["fp8_jit"], 3),
            "speedup_chain": round(tot["bf16"] / tot["fp8_chain"], 3),
            "fp8_jit_chain_ms": round(tot["fp8_jit_chain"], 3),
            "speedup_jit_chain": round(tot["bf16"] / tot["fp8_jit_chain"], 3),
            "fp8_block_tflops": round(tot["fl"] / tot["fp8"] / 1e9, 1)}
    print("SUMMARY " + json.dumps(summ), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"blocks": rows, "summary": summ}, f, indent=1)
# (name, cin sources, cout, H) of the 3x3 convs of UNet(3,2) at 1024^2 (inc.0 excluded)
LAYERS = [
    ("inc.2", [64], 64, 1024), ("down1.1", [64], 128, 512), ("down1.2", [128], 128, 512),
    ("down2.1", [128], 256, 256), ("down2.2", [256], 256, 256),
    ("down3.1", [256], 512, 128), ("down3.2", [512], 512, 128),
    ("down4.1", [512], 1024, 64), ("down4.2", [1024], 1024, 64),
    ("up1.1", [512, 512], 512, 128), ("up1.2", [512], 512, 128),
    ("up2.1", [256, 256], 256, 256), ("up2.2", [256], 256, 256),
    ("up3.1", [128, 128], 128, 512), ("up3.2", [128], 128, 512),
    ("up4.1", [64, 64], 64, 1024), ("up4.2", [64], 64, 1024),
]


GRAPH = False  # --graph: time one captured HIP graph of `reps` calls (GPU time, no Python enqueue)


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if GRAPH:
        # the training step replays as one graph: time the blocks the same way
        # (eagerly, the just-in-time path's extra launches are Python-bound at
        # the 64^2-128^2 blocks; a delayed call's host slot counter freezes in
        # the capture, which changes values, not the kernels timed)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--layers", default="")
    ap.add_argument("--no-bf16", action="store_true")
    ap.add_argument("--json", default="")
    ap.add_argument("--double", action="store_true", help="time whole DoubleConv blocks (see above)")
    ap.add_argument("--tune", default="", help="KEY=VAL,... vu_gemm_set_tuning before the run (A/B)")
    ap.add_argument("--jit-two-pass", action="store_true",
                    help="just-in-time path as in round 5 (fp8.JIT_MINMAX = False: BN1 apply to bf16, amax + "
                         "quantise passes) instead of the min/max-epilogue scale")
    ap.add_argument("--graph", action="store_true", help="time graph replays (GPU time) instead of eager calls")
    args = ap.parse_args()
    global GRAPH
    GRAPH = args.graph
    if args.jit_two_pass:
        fp8.JIT_MINMAX = False
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _lib.call("vu_gemm_set_tuning", int(k), int(v))
    torch.manual_seed(0)
    if args.double:
        return double_main(args)
    dev = torch.device("cuda")
    B = args.batch
    rows = []
    tot = {"fp8": [0.0, 0.0], "bf16": [0.0, 0.0], "quant": [0.0, 0.0]}
    for name, cins, co, H in LAYERS:
        if args.layers and name not in args.layers.split(","):
            continue
        # post-ReLU-like activations (non-negative, half zeros)
        srcs = [torch.randn(B, c, H, H, device=dev).relu().to(torch.bfloat16).contiguous(memory_format=K.CL)
                for c in cins]
        ci = sum(cins)
        w = torch.nn.Conv2d(ci, co, 3, padding=1, bias=False).to(dev).weight.detach()
        fl = 2.0 * B * H * H * co * 9 * ci
        am = fp8.amax(srcs)
        qs, dq = [], None
        for t in srcs:
            q, dq = fp8.quantize(t, am)
            qs.append(q)
        wq, ws = fp8.quantize_weight(w)
        y8 = K.empty_act(B, co, H, H, torch.bfloat16, dev)
        ms8 = timeit(lambda: fp8.conv3x3(qs, dq, wq, ws, co, out=y8, stats=True), args.reps)

        def quant():
            a = fp8.amax(srcs)
            for t in srcs:
                fp8.quantize(t, a)
        msq = timeit(quant, args.reps)
        row = {"layer": name, "cin": ci, "cout": co, "hw": H, "fp8_us": round(ms8 * 1e3, 1),
               "fp8_tflops": round(fl / ms8 / 1e9, 1), "fp8_frac": round(fl / ms8 / 1e9 / PEAK_FP8, 4),
               "quant_us": round(msq * 1e3, 1)}
        tot["fp8"][0] += fl
        tot["fp8"][1] += ms8
        tot["quant"][1] += msq
        if not args.no_bf16:
            yb = K.empty_act(B, co, H, H, torch.bfloat16, dev)
            wb = w3x3_fwd(w, _lib.BF16)
            msb = timeit(lambda: K.gemm_fwd(K.gather3x3(srcs), wb, co, yb, _lib.BF16, stats=True), args.reps)
            row.update(bf16_us=round(msb * 1e3, 1), bf16_tflops=round(fl / msb / 1e9, 1),
                       speedup=round(msb / ms8, 2))
            tot["bf16"][0] += fl
            tot["bf16"][1] += msb
        # error vs the unquantised conv of the same bf16 input, one image (reported)
        x32 = torch.cat([s_[:1].float() for s_ in srcs], 1)
        ref = F.conv2d(x32, w, padding=1)
        err = (y8[:1].float() - ref).abs()
        row["rel_err_max"] = round((err.max() / ref.abs().max()).item(), 5)
        row["rel_err_rms"] = round((err.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt()).item(), 5)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del srcs, qs, y8
        torch.cuda.empty_cache()
    f8 = tot["fp8"]
    summ = {"batch": B, "image": "3x1024x1024", "layers": len(rows),
            "fp8_ms": round(f8[1], 3),
            "fp8_tflops": round(f8[0] / f8[1] / 1e9, 1) if f8[1] else None,
            "fp8_frac_of_5pf": round(f8[0] / f8[1] / 1e9 / PEAK_FP8, 4) if f8[1] else None,
            "quant_ms": round(tot["quant"][1], 3),
            "conv_img_per_s": round(B / (f8[1] * 1e-3), 2) if f8[1] else None}
    if tot["bf16"][1]:
        summ.update(bf16_ms=round(tot["bf16"][1], 3),
                    bf16_tflops=round(tot["bf16"][0] / tot["bf16"][1] / 1e9, 1),
                    speedup=round(tot["bf16"][1] / f8[1], 3))
    print("SUMMARY " + json.dumps(summ), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"layers": rows, "summary": summ}, f, indent=1)


if __name__ == "__main__":
    main()
