"""Host CPU probe for the cpu_baseline leg: affinity, cgroup quota, and the
time of one CPU conv at several thread counts (prints as it goes)."""
import os
import time

import torch
import torch.nn.functional as F

aff = len(os.sched_getaffinity(0))
print("affinity", aff, "cpu_count", os.cpu_count(), "OMP", os.environ.get("OMP_NUM_THREADS"), flush=True)
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us"):
    try:
        print(p, open(p).read().strip(), flush=True)
    except OSError:
        pass
x = torch.randn(8, 64, 256, 256).contiguous(memory_format=torch.channels_last)
w = torch.randn(64, 64, 3, 3).contiguous(memory_format=torch.channels_last)
for t in (8, 16, 32, 64, 128, aff):
    torch.set_num_threads(t)
    F.conv2d(x, w, padding=1)
    t0 = time.perf_counter()
    for _ in range(3):
        F.conv2d(x, w, padding=1)
    dt = (time.perf_counter() - t0) / 3
    print(f"threads {t:4d}: conv 8x64x256^2 3x3 {dt * 1e3:8.1f} ms  ({2 * 8 * 256 * 256 * 64 * 576 / dt / 1e12:.2f} TFLOP/s)",
          flush=True)
