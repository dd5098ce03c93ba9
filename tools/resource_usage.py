#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy table of the codec library.

    python tools/resource_usage.py [substring ...]

Compiles openfl_amd/csrc/eden_kernels.hip with -Rpass-analysis=kernel-resource-usage
(into /tmp, the in-tree library is untouched) and prints one line per kernel
whose mangled name contains any of the given substrings (all kernels if none).
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "openfl_amd", "csrc", "eden_kernels.hip")
KEYS = ("TotalSGPRs", "VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "Occupancy [waves/SIMD]",
        "LDS Size [bytes/block]")


def main():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++20", "-O3", "-fPIC", "-shared",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.dirname(SRC),
           "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/ofl_resource_usage.so", SRC]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = {}, None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        for k in KEYS:
            m = re.search(r"remark:\s+" + re.escape(k) + r": (\d+)", line)
            if m and cur:
                rows[cur][k] = int(m.group(1))
    subs = sys.argv[1:]
    print(f"{'kernel':44s} " + " ".join(f"{k.split()[0][:8]:>8s}" for k in KEYS))
    for name, r in rows.items():
        if subs and not any(s in name for s in subs):
            continue
        print(f"{name[:44]:44s} " + " ".join(f"{r.get(k, -1):8d}" for k in KEYS))


if __name__ == "__main__":
    main()
