"""Host-side cost of one training step: wall time of the step's Python +
launch path with the GPU kept busy (no sync inside the timed steps) vs the
GPU time of the same steps.  A step is launch-bound when the two meet.

usage: python tools/host_overhead.py [--model unet|vae] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="unet")
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    from bench import synthetic
    from vaeunet_amd import UNet, UNetResNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    from vaeunet_amd.optim import FusedAdamW, clip_grad_norm_
    dev = torch.device("cuda")
    vae = args.model == "vae"
    model = UNetResNet(3, 1, pretrained=False) if vae else UNet(3, 2)
    model = seeded_init_(model, 0).to(dev).to(memory_format=torch.channels_last).train()
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    crit = CombinedLoss()
    x, t = synthetic(8, 512, 1 if vae else 2, 0, dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if vae:
                lg, mu, lv = model(x)
                loss = crit(lg, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
            else:
                loss = crit(model(x), t)
        loss.backward()
        clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    def step_split(acc):
        t0 = time.perf_counter()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if vae:
                lg, mu, lv = model(x)
                t1 = time.perf_counter()
                loss = crit(lg, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
            else:
                lg = model(x)
                t1 = time.perf_counter()
                loss = crit(lg, t)
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        t4 = time.perf_counter()
        for k, v in zip(("forward", "loss", "backward", "clip+optim"), (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            acc[k] = acc.get(k, 0.0) + v

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    acc = {}
    for _ in range(args.steps):
        step_split(acc)
    torch.cuda.synchronize()
    print(" ".join(f"{k} {1e3 * v / args.steps:.2f}" for k, v in acc.items()), "ms/step host")
    # host time per step: enqueue K steps back to back, time the Python side
    # (the queue never drains as long as the GPU is the slower side)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t1 = time.perf_counter()
    e.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    gpu = s.elapsed_time(e) / args.steps
    print(f"{args.model}: host enqueue {1e3 * (t1 - t0) / args.steps:.2f} ms/step, "
          f"wall {1e3 * (t2 - t0) / args.steps:.2f} ms/step, GPU events {gpu:.2f} ms/step")


if __name__ == "__main__":
    main()
