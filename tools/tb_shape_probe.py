#!/usr/bin/env python3
"""Rate of the fp32 multi-row blocked kernel on one output box inside arrays
of different shapes (the decomposed interior's array carries ghost planes /
rows around the owned cells): which of array shape, box offset and box size
costs what.  Fields are zeros (timing only).

    python tools/tb_shape_probe.py --T 4 --case 256,512,1024:0,0,0:256,512,1024 ...
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=4)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--case", action="append", required=True,
                    help="array nx,ny,nz : box lo x,y,z : box size x,y,z")
    a = ap.parse_args()
    import torch
    from fdtd3d_amd.ops import make_ops
    from fdtd3d_amd.ops.coef import Coef
    ops = make_ops("hip", None, "cuda:0", torch.float32)
    comps = ("Ex", "Ey", "Ez", "Hx", "Hy", "Hz")
    for case in a.case:
        sh, lo, sz = [tuple(int(v) for v in p.split(",")) for p in case.split(":")]
        fin = {c: torch.zeros(sh, device="cuda:0") for c in comps}
        fout = {c: torch.zeros(sh, device="cuda:0") for c in comps}
        upd = {c: ((0, 0, 0), sh) for c in comps}
        ob = (lo, tuple(lo[d] + sz[d] for d in range(3)))
        cb = {c: Coef(scalar=0.5) for c in comps}
        for _ in range(2):
            ops.tb_step(fin, fout, upd, ob, cb, a.T)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(a.reps):
            ops.tb_step(fin, fout, upd, ob, cb, a.T) if r % 2 == 0 else ops.tb_step(fout, fin, upd, ob, cb, a.T)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        cells = sz[0] * sz[1] * sz[2]
        print("array %s box lo %s size %s: %.3f ms per pass, %.0f Mcells/s" % (sh, lo, sz, ms, cells * a.T / ms / 1e3),
              flush=True)
        del fin, fout
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
