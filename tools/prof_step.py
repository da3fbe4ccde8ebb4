"""Per-launch listing of one training step from a rocprofv3 rocpd .db
(kernel, workgroups, duration, LDS, VGPRs). Step boundary = the AdamW kernel.
usage: python tools/prof_step.py run_results.db [step_index]"""
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
k = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(c.execute("select name, grid_x, workgroup_x, duration, lds_size, vgpr_count, accum_vgpr_count "
                      "from kernels order by start"))
idx = [i for i, r in enumerate(rows) if "mt_adamw" in r[0]]
s0, s1 = idx[k - 1] + 1, idx[k] + 1
tot = 0
for n, gx, wx, d, lds, v, a in rows[s0:s1]:
    n = re.sub(r"\(anonymous namespace\)::|void |at::native::", "", n)
    n = n.split("(")[0]
    tot += d
    print(f"{n[:58]:58s} wg={gx // max(wx, 1):8d} {d / 1000:8.1f}us lds={lds:6d} v={v} a={a}")
print(f"# step total {tot / 1e6:.3f} ms, {s1 - s0} launches")
