#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy summary of one HIP source file,
from the compiler's kernel-resource-usage remarks (gfx950):

    python tools/kernel_resources.py fdtd3d_amd/csrc/yee3d_tb.hip [name-filter]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I",
           os.path.join(ROOT, "fdtd3d_amd", "csrc"), "-c", src, "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            name = txt.split(":", 1)[1].strip()
            dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            dem = re.sub(r"\(.*", "", dem.replace("(anonymous namespace)::", "")).replace("void ", "")
            cur = {"name": dem}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    print("| kernel | VGPRs | AGPRs | SGPRs | scratch B | LDS B | occupancy (waves/SIMD) |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for r in rows:
        if filt not in r["name"]:
            continue
        print("| `%s` | %s | %s | %s | %s | %s | %s |" % (r["name"], r.get("VGPRs", ""), r.get("AGPRs", ""),
                                                     r.get("SGPRs", ""), r.get("ScratchSize [bytes/lane]", ""),
                                                     r.get("LDS Size [bytes/block]", ""), r.get("Occupancy [waves/SIMD]", "")))


if __name__ == "__main__":
    main()
