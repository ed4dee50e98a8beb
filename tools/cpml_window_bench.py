#!/usr/bin/env python3
"""Micro-benchmark of the fp32 CPML split kernels (csrc/yee3d_cpml.hip) on
the windows a 512^3 CPML hybrid shell launches: x / y / z slabs of the T=5
shell (32 cells deep, PML 10 inside them), the PML-free inner box, and the
whole grid.  CUDA-event timing, median of rounds; GB/s counts 36 bytes per
cell and half step (3 source + 3 destination reads, 3 writes; psi extra).

    python tools/cpml_window_bench.py [--n 512] [--depth 32]
    FDTD3D_HIP_LIB=/path/to/other/libfdtd3d_hip.so python tools/cpml_window_bench.py   # A/B
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme  # noqa: E402
from fdtd3d_amd.ops import make_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--depth", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    n, d = a.n, a.depth
    cfg = SchemeConfig(scheme="3d", size=(n, n, n), dtype="f32", scene="vacuum", use_pml=True, pml_type="cpml",
                       hybrid_block=1, time_steps=1)
    s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32))
    s.init_scheme()
    s.init_grids()
    s.randomize_fields(seed=1)
    F = s.F[0]
    wins = {
        "x-slab": ((0, 0, 0), (d, n, n)),
        "y-slab": ((d, 0, 0), (n - d, d, n)),
        "z-slab": ((d, d, 0), (n - d, n - d, d)),
        "inner": ((d, d, d), (n - d, n - d, n - d)),
        "pml-free": ((12, 12, 12), (n - 12, n - 12, n - 12)),
        "whole": ((0, 0, 0), (n, n, n)),
    }
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for _ in range(a.rounds):
        for name, w in wins.items():
            for kind in ("E", "H"):
                comps = s.e_comps if kind == "E" else s.h_comps
                boxes = {c: s.local_box(c, w) for c in comps}
                tab = s.cpml.kernel_table(kind, 0)
                s.ops.curl_update_cpml(kind, boxes, F, F, s.cb, tab)
                ev0.record()
                for _ in range(5):
                    s.ops.curl_update_cpml(kind, boxes, F, F, s.cb, tab)
                ev1.record()
                torch.cuda.synchronize()
                res.setdefault((name, kind), []).append(ev0.elapsed_time(ev1) / 5)
    for (name, kind), v in res.items():
        w = wins[name]
        cells = 1
        for k in range(3):
            cells *= w[1][k] - w[0][k]
        ms = statistics.median(v)
        print("%-9s %s %-30s %8.1f us  %7.0f Mcells/s  %6.2f TB/s" % (name, kind, w, ms * 1e3, cells / ms / 1e3,
                                                                     36 * cells / ms / 1e9), flush=True)


if __name__ == "__main__":
    main()
