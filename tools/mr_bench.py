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
    ap.add_argument("--only", default="", help="run only the cases whose name contains this")
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
    cls = {"core": 0, "xwin": 1, "ywin": 2, "zwin": 4}
    for T in (1, 4):
        cases.append(("T%d plain core" % T, T, wins["core"], None, None, 0))
        cases.append(("T%d tfsf  core" % T, T, wins["core"], g, None, 0))
        for name in ("core", "xwin", "ywin", "zwin"):
            cases.append(("T%d cpml  %s" % (T, name), T, wins[name], None, cp, 7))
            if T > 1 and name != "core":
                cases.append(("T%d cpml  %s class %d" % (T, name, cls[name]), T, wins[name], None, cp, cls[name]))
        cases.append(("T%d cp+tf xwin" % T, T, wins["xwin"], g, cp, 1 if T > 1 else 7))
    if a.only:
        cases = [c for c in cases if a.only in c[0]]
    res = {c[0]: [] for c in cases}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(a.rounds):
        for name, T, box, tf, cpd, cax in cases:
            kw = {"cpml_axes": cax} if cpd is not None else {}
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
    for name, T, box, tf, cpd, cax in cases:
        cells = 1
        for d in range(3):
            cells *= box[1][d] - box[0][d]
        ms = statistics.median(res[name])
        print("%-22s %8.3f ms  %9.1f Mcell-steps/s" % (name, ms, cells * T / ms / 1e3))


if __name__ == "__main__":
    main()
