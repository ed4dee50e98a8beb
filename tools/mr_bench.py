#!/usr/bin/env python3
"""Micro-benchmark of the multi-row blocked kernel's feature variants
(yee3d_tb.hip k_tb3d_mr): plain / TF-SF / CPML / sparse per-cell, full grid
and thin shell windows, one process, CUDA-event timing (median of rounds).

    python tools/mr_bench.py [--n 512]
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
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    n = a.n
    cfg = SchemeConfig(scheme="3d", size=(n, n, n), dtype="f32", scene="vacuum", use_pml=True, pml_type="cpml",
                       use_tfsf=True, hybrid_block=1, time_steps=1)
    s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32))
    s.init_scheme()
    s.init_grids()
    F = s.F[0]
    G = {c: torch.zeros_like(F[c]) for c in s.comps}
    alloc = s.domain.allocated_global()
    upd = {c: s.local_box(c, alloc) for c in s.comps}
    whole = ((0, 0, 0), (n, n, n))
    t = 21
    wins = {"whole": whole, "xwin": ((0, 0, 0), (t, n, n)), "ywin": ((t, 0, 0), (n - t, t, n)),
            "zwin": ((t, t, 0), (n - t, n - t, t)), "core": ((16, 16, 16), (n - 16, n - 16, n - 16))}
    g = s._tfsf_pass(0, 5)
    cp = s.cpml.host_table(0)
    cases = []
    for T in (1, 4):
        for name, box in wins.items():
            if T == 4 and name != "core" and name != "whole":
                continue
            cases.append(("T%d plain %s" % (T, name), T, box, None, None))
            cases.append(("T%d tfsf  %s" % (T, name), T, box, g, None))
            if T == 1:
                cases.append(("T1 cpml  %s" % name, 1, box, None, cp))
                cases.append(("T1 cp+tf %s" % name, 1, box, g, cp))
    res = {c[0]: [] for c in cases}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(a.rounds):
        for name, T, box, tf, cpd in cases:
            kw = {}
            if tf is not None:
                kw["tfsf"] = tf
            if cpd is not None:
                kw["cpml"] = cpd
            s.ops.tb_step(F, G, upd, box, s.cb, T, None, **kw)
            ev0.record()
            for _ in range(3):
                s.ops.tb_step(F, G, upd, box, s.cb, T, None, **kw)
            ev1.record()
            torch.cuda.synchronize()
            res[name].append(ev0.elapsed_time(ev1) / 3)
    for name, T, box, tf, cpd in cases:
        cells = 1
        for d in range(3):
            cells *= box[1][d] - box[0][d]
        ms = statistics.median(res[name])
        print("%-22s %8.3f ms  %9.1f Mcell-steps/s" % (name, ms, cells * T / ms / 1e3))


if __name__ == "__main__":
    main()
