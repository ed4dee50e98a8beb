#!/usr/bin/env python3
"""Micro-benchmark of the multi-row blocked kernel's variants (csrc/tb3d_mr.h):
plain and TF/SF (TfsfSets), on the core box
of a 512^3 CPML + TF/SF run; CUDA-event timing, median of rounds.

    python tools/mr_bench.py [--n 512] [--T 5]
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
    ap.add_argument("--T", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--margin", type=int, default=16, help="core box margin to each face")
    a = ap.parse_args()
    n, T = a.n, a.T
    cfg = SchemeConfig(scheme="3d", size=(n, n, n), dtype="f32", scene="vacuum", use_pml=True, pml_type="cpml",
                       use_tfsf=True, hybrid_block=1, time_steps=1)
    s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32))
    s.init_scheme()
    s.init_grids()
    s.randomize_fields(seed=1)
    F = s.F[0]
    G = {c: torch.zeros_like(F[c]) for c in s.comps}
    alloc = s.domain.allocated_global()
    upd = {c: s.local_box(c, alloc) for c in s.comps}
    m = a.margin
    core = ((m, m, m), (n - m, n - m, n - m))
    g = s._tfsf_pass(0, T)
    inner = ((40, 40, 40), (n - 40, n - 40, n - 40))  # no TF/SF target within its cone
    cases = [("plain", {}, core), ("tfsf", {"tfsf": g}, core), ("plain-in", {}, inner), ("tfsf-in", {"tfsf": g}, inner)]
    res = {c[0]: [] for c in cases}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for name, kw, box in cases:
            s.ops.tb_step(F, G, upd, box, s.cb, T, None, **kw)
            ev0.record()
            for _ in range(3):
                s.ops.tb_step(F, G, upd, box, s.cb, T, None, **kw)
            ev1.record()
            torch.cuda.synchronize()
            res[name].append(ev0.elapsed_time(ev1) / 3)
    for name, _, box in cases:
        cells = 1
        for d in range(3):
            cells *= box[1][d] - box[0][d]
        ms = statistics.median(res[name])
        print("T%d %-10s box %s  %8.3f ms  %9.1f Mcell-steps/s" % (T, name, box, ms, cells * T / ms / 1e3),
              flush=True)


if __name__ == "__main__":
    main()
