"""Convolutional PML (CPML, Roden & Gedney) as additive slab corrections.

The reference only has a UPML in D/B form that touches every cell of the grid
(three sweeps per component, ``Scheme3D.cpp:266-416``).  CPML keeps the
interior update untouched: the main Yee kernel runs over the whole domain and,
inside each absorbing slab, a correction kernel updates the convolution
auxiliaries and adds them:

    psi   = b[n] * psi + c[n] * dS          (dS: the curl difference along the slab axis)
    F    += Cb * sign * ((1/kappa[n] - 1) * dS + psi)

so auxiliary memory and traffic scale with the slab volume only.  Profiles
(polynomial grading order ``m``, target reflection ``R``; kappa and the
complex-frequency-shift alpha from ``--cpml-kappa-max`` / ``--cpml-alpha-max``)
are evaluated at each component's own staggered position.
"""

from __future__ import annotations

import math
from typing import Dict, List, Tuple

import torch

from ..layout.yee import MIN_COORD_FP
from ..parallel.domain import box_empty, box_intersect
from ..utils.constants import EPS0, MU0

GRADING_ORDER = 4
REFLECTION = 1e-8


class CPMLSlab:
    """psi auxiliary of one (component, curl term, side) slab."""

    def __init__(self, comp, src, axis, sign, side, gbox, lbox, b, c, kinv_m1, planes, device, dtype):
        self.comp, self.src, self.axis, self.sign, self.side = comp, src, axis, sign, side
        self.gbox = gbox
        self.lbox = lbox  # local box of psi storage
        shape = tuple(lbox[1][d] - lbox[0][d] for d in range(3))
        self.psi = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(planes)]
        self.b, self.c, self.kinv_m1 = b, c, kinv_m1


class CPML:
    def __init__(self, scheme):
        self.s = scheme
        cfg = scheme.cfg
        lay = scheme.layout
        dom = scheme.domain
        dt, dx = scheme.dt, scheme.dx
        self.slabs: Dict[str, List[CPMLSlab]] = {c: [] for c in scheme.comps}
        kmax = getattr(cfg, "cpml_kappa_max", 1.0)
        amax = getattr(cfg, "cpml_alpha_max", 0.0)
        for c in scheme.comps:
            glo, ghi = lay.global_range(c)
            for (src, axis, sign) in lay.curl_terms(c):
                P = lay.pml_size[axis]
                if P <= 0 or not lay.active(axis):
                    continue
                N = cfg.size[axis]
                d = P * dx
                sig_max = -(GRADING_ORDER + 1) * math.log(REFLECTION) / (2 * math.sqrt(MU0 / EPS0) * d)
                m = MIN_COORD_FP[c][axis]
                for side in (0, 1):
                    lo, hi = list(glo), list(ghi)
                    if side == 0:
                        hi[axis] = min(hi[axis], int(math.ceil(P - m)))
                    else:
                        lo[axis] = max(lo[axis], int(math.floor(N - P - m)) + 1)
                    g = (tuple(lo), tuple(hi))
                    g = box_intersect(g, dom.allocated_global())
                    if box_empty(g):
                        continue
                    lb = dom.to_local(g)
                    n_loc = dom.shape[axis]
                    idx = torch.arange(n_loc, dtype=torch.float64) + dom.origin[axis] + m
                    if side == 0:
                        depth = (P - idx) / P
                    else:
                        depth = (idx - (N - P)) / P
                    depth = depth.clamp(0.0, 1.0)
                    sig = sig_max * depth ** GRADING_ORDER
                    kap = 1.0 + (kmax - 1.0) * depth ** GRADING_ORDER
                    alp = amax * (1.0 - depth)
                    bcoef = torch.exp(-(sig / kap + alp) * dt / EPS0)
                    denom = sig * kap + kap * kap * alp
                    ccoef = torch.where(denom > 0, sig / torch.where(denom > 0, denom, torch.ones_like(denom)) * (bcoef - 1.0),
                                        torch.zeros_like(sig))
                    kinv = 1.0 / kap - 1.0
                    dev, dt_ = scheme.device, scheme.dtype
                    self.slabs[c].append(CPMLSlab(c, src, axis, sign, side, g, lb, bcoef.to(dev, dt_),
                                                  ccoef.to(dev, dt_), kinv.to(dev, dt_), scheme.planes, dev, dt_))

    def apply(self, kind: str, p: int, boxes) -> None:
        s = self.s
        F = s.F[p]
        for c, box in boxes.items():
            if box_empty(box):
                continue
            for sl in self.slabs[c]:
                b = box_intersect(box, sl.lbox)
                if box_empty(b):
                    continue
                s.ops.cpml_apply(kind, F[c], F[sl.src], sl.axis, sl.sign, sl.psi[p], sl.lbox, b, sl.b, sl.c,
                                 sl.kinv_m1, s.cb[c])

    def state_tensors(self, p: int) -> List[torch.Tensor]:
        return [sl.psi[p] for c in self.slabs for sl in self.slabs[c]]
