#!/usr/bin/env python3
"""Debug: one single-step CPML pass of the multi-row kernel (cpml=...) vs one
stepped step (yee3d_cpml.hip kernels) from random fields; prints the largest
field / psi differences and where they are.  Then the same over shrinking
shell windows (hybrid v2) vs the stepped run."""
import dataclasses
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme  # noqa: E402
from fdtd3d_amd.ops import make_ops  # noqa: E402


def mk(cfg):
    s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32))
    s.init_scheme()
    s.init_grids()
    s.randomize_fields(seed=5)
    return s


def where(d):
    i = int(d.abs().argmax())
    return tuple(int(v) for v in torch.unravel_index(torch.tensor(i), d.shape))


cfg = SchemeConfig(scheme="3d", size=(80, 72, 96), dtype="f32", pml_size=(5, 5, 5), scene="vacuum", use_pml=True,
                   pml_type="cpml", hybrid_block=1, time_steps=1)
a = mk(cfg)
b = mk(cfg)
b.F_alt = [{c: torch.zeros_like(b.F[0][c]) for c in b.comps}]
a.step()
alloc = b.domain.allocated_global()
upd = {c: b.local_box(c, alloc) for c in b.comps}
b.ops.tb_step(b.F[0], b.F_alt[0], upd, ((0, 0, 0), cfg.size), b.cb, 1, None, cpml=b.cpml.host_table(0))
torch.cuda.synchronize()
for c in a.comps:
    d = (a.F[0][c] - b.F_alt[0][c]).double().cpu()
    print("field", c, "max err %.3e" % float(d.abs().max()), "at", where(d), "scale %.3e" % float(a.F[0][c].abs().max()))
for c in a.comps:
    for sa, sb in zip(a.cpml.slabs[c], b.cpml.slabs[c]):
        d = (sa.psi[0] - sb.psi[0]).double().cpu()
        print("psi", c, "src", sa.src, "axis", sa.axis, "side", sa.side, "lbox", sa.lbox, "max err %.3e" % float(d.abs().max()),
              "at", where(d), "scale %.3e" % float(sa.psi[0].abs().max()))
print("---- details")
for c in ("Hy", "Hz", "Ey"):
    d = (a.F[0][c] - b.F_alt[0][c]).double().cpu()
    d[35:46, 31:42, 43:54] = 0  # source neighbourhood
    print("field", c, "err excl. source %.3e at" % float(d.abs().max()), where(d))
    for x in range(0, 6):
        print("   x=%d max err %.3e" % (x, float(d[x].abs().max())))
sa = [s_ for s_ in a.cpml.slabs["Hy"] if s_.axis == 0 and s_.side == 0][0]
sb = [s_ for s_ in b.cpml.slabs["Hy"] if s_.axis == 0 and s_.side == 0][0]
for x in range(sa.psi[0].shape[0]):
    d = (sa.psi[0][x] - sb.psi[0][x]).double().cpu()
    print("Hy psi_x plane", x, "err %.3e" % float(d.abs().max()), "a %.3e b %.3e" % (float(sa.psi[0][x].abs().max()), float(sb.psi[0][x].abs().max())))
print("profiles Hy x:", a.cpml.kernel_table("H", 0)[2][3 * 1 + 0][:6], a.cpml.kernel_table("H", 0)[2][3 * 1 + 1][:6])
