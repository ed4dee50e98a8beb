#!/usr/bin/env python3
"""Per-window timing of the stepped shell's split CPML kernels
(yee3d_cpml.hip k_update_{e,h}3d_cpml_v4) against the plain float4 split
kernels on the same windows and on the whole grid: 512^3 CPML + TF/SF hybrid
plan (GPU; CUDA events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme  # noqa: E402
from fdtd3d_amd.ops import make_ops  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    cfg = SchemeConfig(scheme="3d", size=(n, n, n), dtype="f32", pml_size=(10, 10, 10), time_steps=10,
                       scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, use_fused=True)
    s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32))
    s.init_scheme()
    s.init_grids()
    s.randomize_fields(seed=1)
    hp = s.hybrid
    assert hp is not None and not hp.get("v2")
    F = s.F[0]
    ops = s.ops
    print("T %d, core %s, %d shell windows" % (hp["T"], hp["core"], len(hp["shells"][0])))
    tot_c = tot_p = 0.0
    for w in hp["shells"][0]:
        cells = 1
        for d in range(3):
            cells *= w[1][d] - w[0][d]
        row = []
        for kind in ("E", "H"):
            comps = s.e_comps if kind == "E" else s.h_comps
            boxes = {c: s.local_box(c, w) for c in comps}
            tab = s.cpml.kernel_table(kind, 0)
            mc = timeit(lambda: ops.curl_update_cpml(kind, boxes, F, F, s.cb, tab))
            mp = timeit(lambda: ops.curl_update(kind, boxes, F, F, s.cb))
            tot_c += mc
            tot_p += mp
            row.append("%s cpml %.4f plain %.4f ms" % (kind, mc, mp))
        print("window %s %9d cells: %s" % (w, cells, "; ".join(row)))
    print("shell step: cpml kernels %.4f ms, plain kernels on the same windows %.4f ms" % (tot_c, tot_p))
    whole = ((0, 0, 0), (n, n, n))
    for kind in ("E", "H"):
        comps = s.e_comps if kind == "E" else s.h_comps
        boxes = {c: s.local_box(c, whole) for c in comps}
        tab = s.cpml.kernel_table(kind, 0)
        mc = timeit(lambda: ops.curl_update_cpml(kind, boxes, F, F, s.cb, tab))
        mp = timeit(lambda: ops.curl_update(kind, boxes, F, F, s.cb))
        print("whole grid %s: cpml %.4f ms (%.0f Gcells/s), plain %.4f ms (%.0f Gcells/s)" % (
            kind, mc, n ** 3 / mc / 1e6, mp, n ** 3 / mp / 1e6))


if __name__ == "__main__":
    main()
