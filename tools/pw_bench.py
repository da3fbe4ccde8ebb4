"""Cold-cache timing of vu_pointwise_fwd (OutConv 64 -> 2 at 8x512x512, bf16): a 512 MB
write between timed calls evicts the input from the L2s / Infinity Cache.
usage: python tools/pw_bench.py"""
import os, sys, torch
sys.path.insert(0, os.getcwd())
from vaeunet_amd import kernels as K
from vaeunet_amd._lib import call, ptr, stream
dev = torch.device("cuda")
x = K.empty_act(8, 64, 512, 512, torch.bfloat16, dev).normal_()
y = torch.empty((8 * 512 * 512, 2), dtype=torch.float32, device=dev)
w = torch.randn(2, 64, device=dev); b = torch.randn(2, device=dev)
P = 8 * 512 * 512
def f():
    call("vu_pointwise_fwd", ptr(x), 64, P, 64, 2, ptr(w), ptr(b), ptr(y), 2, 1, stream())
for _ in range(3): f()
torch.cuda.synchronize()
# flush caches between timed calls with a 512 MB write
junk = torch.empty(512 * 1024 * 1024 // 4, device=dev)
ts = []
for _ in range(10):
    junk.fill_(1.0)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(); f(); e.record(); torch.cuda.synchronize()
    ts.append(s.elapsed_time(e) * 1e3)
ts.sort()
print(f"median {ts[5]:.1f} us  min {ts[0]:.1f} us", flush=True)
