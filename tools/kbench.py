#!/usr/bin/env python3
"""Kernel micro-benchmark: interleaved rounds of the 3D update variants on one
GPU in ONE process (cdna_hip_programming.md section 5.4 rule 24), printing the
median and min ms/step and the effective HBM bandwidth of each variant.

    python tools/kbench.py --size 1024 1024 1024 --rounds 5 --steps 10
"""

import argparse
import ctypes
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, nargs=3, default=[1024, 1024, 1024])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--variants", default="split-scalar,split-v4,fused-scalar,fused-v4-r7,fused-v4-r3")
    ap.add_argument("--xchunks", default="32")
    a = ap.parse_args()
    import torch
    from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
    from fdtd3d_amd.ops import make_ops
    from fdtd3d_amd.ops import hip_ops

    lib = hip_ops.load_library()
    size = tuple(a.size)
    cells = size[0] * size[1] * size[2]
    results = {}
    schemes = {}
    for v in a.variants.split(","):
        for xc in [int(x) for x in a.xchunks.split(",")]:
            fused = v.startswith("fused")
            vec4 = "v4" in v
            cfg = SchemeConfig(scheme="3d", size=size, time_steps=0, scene="vacuum", dtype="f32", use_fused=fused)
            key = "%s/xc%d" % (v, xc)
            schemes[key] = (cfg, vec4, xc, v)
    for r in range(a.rounds):
        for key, (cfg, vec4, xc, v) in schemes.items():
            if "r3" in v:
                lib.fdtd_set_fused_rows(3)
            else:
                lib.fdtd_set_fused_rows(7)
            ops = make_ops("hip", None, "cuda:0", torch.float32, xchunk=xc, vec4=vec4)
            s = YeeScheme(cfg, ops)
            s.init_scheme()
            s.init_grids()
            for _ in range(2):
                s.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                s.step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps
            results.setdefault(key, []).append(dt)
            del s, ops
            torch.cuda.empty_cache()
    for key, ts in results.items():
        fused = key.startswith("fused")
        bpc = 48 if fused else 72
        med = statistics.median(ts)
        print("%-22s median %.3f ms  min %.3f ms  %.1f kMcells/s  %.2f TB/s(algorithmic)" % (
            key, med * 1e3, min(ts) * 1e3, cells / med / 1e9, cells * bpc / med / 1e12))


if __name__ == "__main__":
    main()
