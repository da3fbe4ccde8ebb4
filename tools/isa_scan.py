"""Scan the gfx950 ISA of the HIP kernels for serialised memory round trips.

Two patterns cost a full memory latency each time they occur and are easy to
introduce from C++ without noticing:

  * ``load -> s_waitcnt vmcnt(0) -> load -> vmcnt(0) ...`` (3+ in a row): a
    guarded load (``if (p < P) v = x[p]``) lands in a basic block of its own
    and is waited for before the next one issues, or a load sits behind a
    store it may alias;
  * ``store -> s_waitcnt vmcnt(0) -> store``: a guarded store whose value is
    computed inside the branch from a load; the wait after the branch also
    waits for the previous STORE (vmcnt counts both).

usage: python tools/isa_scan.py [file.hip ...]   (default: every csrc/*.hip)
Prints one line per kernel with either pattern: the source, the number of
load chains / serialised stores, and the demangled kernel name.  Round 4's
fixes of the hits (DESIGN.md §4.2 "Serialised loads in the small streams")
are measured in profiles/r4ai_*, r4ak_*, r4al_*, r4ao_*, r4ap_*.
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def classify(line):
    if "global_load" in line and "lds" not in line:
        return "L"
    if "s_waitcnt vmcnt(0)" in line:
        return "Z"
    if "global_store" in line:
        return "S"
    return ""


def scan(src, out):
    asm = os.path.join(out, os.path.basename(src) + ".s")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S", src,
                    "-o", asm], check=True, stderr=subprocess.DEVNULL)
    text = open(asm).read()
    hits = []
    for m in re.finditer(r"^(_Z\w+):", text, re.M):
        end = text.find(".Lfunc_end", m.end())
        if end < 0:
            continue
        seq = "".join(classify(l) for l in text[m.end():end].splitlines())
        loads = len(re.findall(r"(?:L+Z){3,}", seq))
        stores = len(re.findall(r"S+Z(?=S)", seq))
        if loads or stores:
            name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
            hits.append((os.path.basename(src), loads, stores, name))
    return hits


def main(argv):
    srcs = argv or sorted(glob.glob(os.path.join(ROOT, "vaeunet_amd", "csrc", "*.hip")))
    with tempfile.TemporaryDirectory() as out:
        for src in srcs:
            for f, loads, stores, name in scan(src, out):
                print(f"{f:18s} load-chains {loads}  serial-stores {stores}  {name[:110]}")


if __name__ == "__main__":
    main(sys.argv[1:])
