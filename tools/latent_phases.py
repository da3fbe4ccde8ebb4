"""Phase timing of vu_latent_bwd (diagnostics): one VAE-U-Net train step at
B=8, 512^2 with vae_engine.LATENT_TIMING set; prints the time between the
kernel's phase-boundary timestamps (100 MHz real-time counter).

usage: python tools/latent_phases.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vaeunet_amd import UNetResNet, vae_engine as V  # noqa: E402
from vaeunet_amd.init import seeded_init_  # noqa: E402
from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits  # noqa: E402

NAMES = ["start", "job table", "phase 1 (split sums)", "phase 2 (BN bwd)", "phase 3a/3b (dW, dz partials)",
         "dz / reparameterize", "pooled -> LDS", "heads dW, db, dpooled"]


def main():
    dev = torch.device("cuda")
    m = seeded_init_(UNetResNet(3, 1, pretrained=False), 0).to(dev).to(memory_format=torch.channels_last)
    x = torch.rand(8, 3, 512, 512, device=dev).contiguous(memory_format=torch.channels_last)
    t = (torch.rand(8, 1, 512, 512, device=dev) < 0.05).float()
    ts = torch.zeros(16, dtype=torch.int64, device=dev)
    for it in range(4):
        V.LATENT_TIMING = ts if it == 3 else None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, mu, lv = m(x)
            loss = CombinedLoss()(lg, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
        loss.backward()
        m.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    v = ts.cpu().tolist()
    for k in range(1, 8):
        print(f"{NAMES[k]:34s} {(v[k] - v[k - 1]) / 100.0:8.2f} us")
    print(f"{'total':34s} {(v[7] - v[0]) / 100.0:8.2f} us")


if __name__ == "__main__":
    main()
