#!/usr/bin/env python3
"""Debug the fused single-step shell kernel against its torch reference:
per case and component the max error and where it sits (GPU)."""
import dataclasses
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fdtd3d_amd.models.blocking import _cut_pieces, _merge_pieces  # noqa: E402
from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme  # noqa: E402
from fdtd3d_amd.ops import make_ops  # noqa: E402
from fdtd3d_amd.parallel.domain import box_subtract  # noqa: E402


def mk(cfg, be, dev, dt):
    s = YeeScheme(cfg, make_ops(be, None, dev, dt))
    s.init_scheme()
    s.init_grids()
    return s


def case(name, size, pml_type, pml, mode, steps=3):
    cfg = SchemeConfig(scheme="3d", size=size, time_steps=3, dtype="f32", scene="vacuum", use_pml=pml is not None,
                       pml_type=pml_type, pml_size=pml or (0, 0, 0), hybrid_block=1)
    s = mk(cfg, "hip", "cuda:0", torch.float32)
    s.randomize_fields(seed=11)
    s.advance(steps)
    torch.cuda.synchronize()
    alloc = ((0, 0, 0), tuple(s.domain.shape))
    if s.use_cpml:
        cuts = s._cpml_cuts()
    else:
        cuts = [None, None, None]
    if mode == "all":
        boxes = [alloc]
    elif mode == "plainall":
        boxes = [alloc]
        cuts = [None, None, None]
    else:
        K = ((14, 13, 15), (size[0] - 12, size[1] - 14, size[2] - 13))
        boxes = [b for b in box_subtract(alloc, K) if all(b[1][d] > b[0][d] for d in range(3))]
    pieces = _merge_pieces([pc for b in boxes for pc in _cut_pieces(b, cuts)])
    upd = {c: s.local_box(c, s.domain.allocated_global()) for c in s.comps}
    ref = mk(dataclasses.replace(cfg, dtype="f64"), "torch", "cpu", torch.float64)
    fin = {c: s.F[0][c].double().cpu() for c in s.comps}
    if s.use_cpml:
        for c in s.comps:
            for a, b in zip(ref.cpml.slabs[c], s.cpml.slabs[c]):
                a.psi[0].copy_(b.psi[0].double().cpu())
    out_r = {c: torch.full_like(fin[c], 7.0) for c in s.comps}
    cp_r = (ref.cpml, 0) if s.use_cpml else None
    ref.ops.shell_step(fin, out_r, upd, [b for b, _ in pieces], [a for _, a in pieces], ref.cb, None, cpml=cp_r)
    out = {c: torch.full_like(s.F[0][c], 7.0) for c in s.comps}
    cp = s.cpml.host_table(0) if s.use_cpml else None
    ax = [a for _, a in pieces] if s.use_cpml else [0] * len(pieces)
    s.ops.shell_step(s.F[0], out, upd, [b for b, _ in pieces], ax, s.cb, None, cpml=cp)
    torch.cuda.synchronize()
    print("== %s pieces %d classes %s" % (name, len(pieces), sorted(set(a for _, a in pieces))))
    for c in s.comps:
        scale = max(float(fin[o].abs().max()) for o in s.comps if o[0] == c[0])
        d = (out[c].double().cpu() - out_r[c]).abs()
        e = float(d.max())
        idx = tuple(int(v) for v in (d == d.max()).nonzero()[0]) if e > 0 else None
        bad = int((d > 2e-5 * scale).sum())
        print("  %s err %.3g rel %.3g bad %d at %s" % (c, e, e / scale, bad, idx))


if __name__ == "__main__" and len(sys.argv) == 1:
    case("plain-all", (40, 36, 48), None, None, "plainall")
    case("plain-thinz", (44, 40, 28), None, None, "plainall")
    case("cpml-all", (40, 36, 48), "cpml", (5, 5, 5), "all")
    case("cpml-shell", (64, 60, 72), "cpml", (6, 6, 6), "shell")


def hybrid_case(T=4, tfsf=True, size=(80, 72, 96)):
    base = dict(scheme="3d", size=size, dtype="f32", pml_size=(5, 5, 5), tfsf_size=(8, 8, 8))
    cfg = SchemeConfig(time_steps=2 * T + 1, **base, scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=tfsf,
                       hybrid_shell="single-pass")
    runs = {}
    for name, hb, be, dev, dt in (("hy", T, "hip", "cuda:0", torch.float32), ("st", 1, "hip", "cuda:0", torch.float32),
                                  ("ref", 1, "torch", "cpu", torch.float64), ("refhy", T, "torch", "cpu", torch.float64)):
        c2 = dataclasses.replace(cfg, hybrid_block=hb, dtype="f32" if dt == torch.float32 else "f64")
        s = mk(c2, be, dev, dt)
        s.randomize_fields(seed=5)
        s.perform_steps()
        if dev != "cpu":
            torch.cuda.synchronize()
        runs[name] = s
    print("== hybrid T=%d tfsf=%s v2=%s" % (T, tfsf, runs["hy"].hybrid.get("v2")))
    for a, b in (("hy", "st"), ("hy", "ref"), ("st", "ref"), ("refhy", "ref"), ("hy", "refhy")):
        out = []
        for c in runs["ref"].comps:
            x, y = runs[a].F[0][c].double().cpu(), runs[b].F[0][c].double().cpu()
            d = (x - y).abs()
            scale = max(float(runs["ref"].F[0][o].abs().max()) for o in runs["ref"].comps if o[0] == c[0])
            e = float(d.max())
            idx = tuple(int(v) for v in (d == d.max()).nonzero()[0]) if e > 0 else None
            out.append("%s %.2g@%s n%d" % (c, e / scale, idx, int((d > 1e-4 * scale).sum())))
        print("  %s vs %s: %s" % (a, b, "; ".join(out)))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "hybrid":
    hybrid_case(4, True)
    hybrid_case(3, False)


def pass_case(T=3, size=(80, 72, 96)):
    """One hybrid pass, step by step: the HIP shell step against the torch
    shell step on the SAME input, then the core."""
    cfg = SchemeConfig(scheme="3d", size=size, dtype="f32", pml_size=(5, 5, 5), time_steps=T, scene="vacuum",
                       use_pml=True, pml_type="cpml", hybrid_block=T)
    s = mk(cfg, "hip", "cuda:0", torch.float32)
    s.randomize_fields(seed=5)
    ref = mk(dataclasses.replace(cfg, dtype="f64"), "torch", "cpu", torch.float64)
    hp = s.hybrid
    print("== pass T=%d v2=%s core %s" % (T, hp.get("v2"), hp["core"]))
    P, Q, Z = s.F[0], s.F_alt[0], s.F_3[0]
    cur = P
    for st in range(1, T + 1):
        out = Q if st % 2 == 1 else Z
        pieces = hp["windows"][st - 1]
        fin = {c: cur[c].double().cpu() for c in s.comps}
        for c in s.comps:
            for a, b in zip(ref.cpml.slabs[c], s.cpml.slabs[c]):
                a.psi[0].copy_(b.psi[0].double().cpu())
        out_r = {c: out[c].double().cpu() for c in s.comps}
        ref.ops.shell_step(fin, out_r, hp["upd"], [b for b, _ in pieces], [a for _, a in pieces], ref.cb, None,
                           cpml=(ref.cpml, 0))
        s.ops.shell_step(cur, out, hp["upd"], [b for b, _ in pieces], [a for _, a in pieces], s.cb, None,
                         cpml=s.cpml.host_table(0))
        s.cpml.flip(0)
        torch.cuda.synchronize()
        msg = []
        for c in s.comps:
            d = (out[c].double().cpu() - out_r[c]).abs()
            scale = max(float(fin[o].abs().max()) for o in s.comps if o[0] == c[0])
            bad = d > 1e-5 * scale
            if bool(bad.any()):
                nz = bad.nonzero()
                msg.append("%s n%d x[%d,%d] y[%d,%d] z[%d,%d]" % (c, nz.shape[0], int(nz[:, 0].min()), int(nz[:, 0].max()),
                                                                int(nz[:, 1].min()), int(nz[:, 1].max()),
                                                                int(nz[:, 2].min()), int(nz[:, 2].max())))
        for c in s.comps:
            for q, (a, b) in enumerate(zip(ref.cpml.slabs[c], s.cpml.slabs[c])):
                d = (b.psi[0].double().cpu() - a.psi_alt[0]).abs()
                sc = float(a.psi_alt[0].abs().max()) + 1e-30
                if float(d.max()) > 1e-5 * sc:
                    nz = (d > 1e-5 * sc).nonzero()
                    g = [tuple(int(v) + a.lbox[0][k] for k, v in enumerate(nz[i])) for i in range(min(4, nz.shape[0]))]
                    msg.append("psi %s#%d ax%d n%d/%d lbox %s first global %s hip %.3g ref %.3g" % (
                        c, q, a.axis, nz.shape[0], d.numel(), a.lbox, g, float(b.psi[0][tuple(nz[0])]),
                        float(a.psi_alt[0][tuple(nz[0])])))
                    for k in range(3):
                        u, cnt = torch.unique(nz[:, k] + a.lbox[0][k], return_counts=True)
                        msg.append("   ax%d: %s" % (k, " ".join("%d:%d" % (int(x), int(y)) for x, y in zip(u, cnt))))
                    hz = (b.psi[0].double().cpu()[tuple(nz.t())] == 0).sum()
                    msg.append("   hip zero at %d of the bad cells; upd box %s" % (int(hz), hp["upd"][c]))
        print("  step %d pieces %d:\n%s" % (st, len(pieces), "\n".join(msg) or "ok"))
        if msg:
            for b, a in pieces:
                print("     piece", b, a)
            break
        cur = out


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pass":
    pass_case(3)


def passes_case(T=3, size=(80, 72, 96), npass=3):
    """Whole hybrid passes, HIP against the torch oracle from the SAME state
    (fields and psi copied before every pass): fields and psi after it."""
    cfg = SchemeConfig(scheme="3d", size=size, dtype="f32", pml_size=(5, 5, 5), time_steps=T, scene="vacuum",
                       use_pml=True, pml_type="cpml", hybrid_block=T, hybrid_shell="single-pass")
    s = mk(cfg, "hip", "cuda:0", torch.float32)
    s.randomize_fields(seed=5)
    r = mk(dataclasses.replace(cfg, dtype="f64"), "torch", "cpu", torch.float64)
    print("== passes T=%d v2 hip=%s torch=%s" % (T, s.hybrid.get("v2"), r.hybrid.get("v2")))
    for n in range(npass):
        for c in s.comps:
            r.F[0][c].copy_(s.F[0][c].double().cpu())
            for a, b in zip(r.cpml.slabs[c], s.cpml.slabs[c]):
                a.psi[0].copy_(b.psi[0].double().cpu())
        s.advance(T)
        r.advance(T)
        torch.cuda.synchronize()
        msg = []
        for c in s.comps:
            d = (s.F[0][c].double().cpu() - r.F[0][c]).abs()
            scale = max(float(r.F[0][o].abs().max()) for o in s.comps if o[0] == c[0])
            bad = d > 1e-5 * scale
            if bool(bad.any()):
                nz = bad.nonzero()
                msg.append("%s n%d x[%d,%d] y[%d,%d] z[%d,%d]" % (c, nz.shape[0], int(nz[:, 0].min()), int(nz[:, 0].max()),
                                                                int(nz[:, 1].min()), int(nz[:, 1].max()),
                                                                int(nz[:, 2].min()), int(nz[:, 2].max())))
            for q, (a, b) in enumerate(zip(r.cpml.slabs[c], s.cpml.slabs[c])):
                d = (b.psi[0].double().cpu() - a.psi[0]).abs()
                sc = float(a.psi[0].abs().max()) + 1e-30
                if float(d.max()) > 1e-5 * sc:
                    nz = (d > 1e-5 * sc).nonzero()
                    msg.append("psi %s#%d ax%d n%d lbox %s first %s" % (c, q, a.axis, nz.shape[0], a.lbox,
                                                                     tuple(int(v) for v in nz[0])))
        print("  pass %d: %s" % (n, "; ".join(msg) or "ok"))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "passes":
    passes_case(3)
    passes_case(1)
    passes_case(2)
