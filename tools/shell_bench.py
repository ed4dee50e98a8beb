#!/usr/bin/env python3
"""Micro-benchmark of the hybrid pass's stepped shell (512^3 CPML + TF/SF by
default): per shell window, the split CPML E / H kernels against the plain
split kernels on the same boxes, plus one whole shell step.  One process,
CUDA-event timing, median of rounds.

    python tools/shell_bench.py [--n 512] [--pml cpml|upml]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme  # noqa: E402
from fdtd3d_amd.ops import make_ops  # noqa: E402


def vol(b):
    v = 1
    for d in range(3):
        v *= max(0, b[1][d] - b[0][d])
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--pml", default="cpml")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    n = a.n
    cfg = SchemeConfig(scheme="3d", size=(n, n, n), dtype="f32", scene="vacuum", use_pml=True, pml_type=a.pml,
                       use_tfsf=True, time_steps=8)
    s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32))
    s.init_scheme()
    s.init_grids()
    s.randomize_fields() if hasattr(s, "randomize_fields") else None
    hp = s.hybrid
    assert hp is not None, "hybrid pass not selected"
    wins = hp["shell"]
    F = s.F[0]
    cases = []
    for i, w in enumerate(wins):
        for kind in ("E", "H"):
            comps = s.e_comps if kind == "E" else s.h_comps
            boxes = {c: s.local_box(c, w) for c in comps}
            if s.use_cpml:
                cases.append(("win%d %s cpml" % (i, kind), w,
                              lambda k=kind, b=boxes: s.ops.curl_update_cpml(k, b, F, F, s.cb,
                                                                             s.cpml.kernel_table(k, 0))))
            cases.append(("win%d %s plain" % (i, kind), w, lambda k=kind, b=boxes: s.ops.curl_update(k, b, F, F, s.cb)))
    cases.append(("shell step", None, lambda: s.step(wins)))
    cases.append(("core pass", None, lambda: [s.ops.tb_step(s.F[0], s.F_alt[0], hp["upd"], ob, s.cb, hp["T"], None)
                                             for ob in hp["core"]]))
    res = {c[0]: [] for c in cases}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for name, w, fn in cases:
            fn()
            ev0.record()
            for _ in range(3):
                fn()
            ev1.record()
            torch.cuda.synchronize()
            res[name].append(ev0.elapsed_time(ev1) / 3)
    print("T=%d core %s, %d shell windows, shell cells %d" % (hp["T"], hp["core"], len(wins),
                                                              sum(vol(w) for w in wins)))
    for name, w, fn in cases:
        ms = statistics.median(res[name])
        extra = ""
        if w is not None:
            extra = "  %s  %7.1f Mcells/s" % (w, vol(w) / ms / 1e3)
        print("%-18s %8.4f ms%s" % (name, ms, extra))


if __name__ == "__main__":
    main()
