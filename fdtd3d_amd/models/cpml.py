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
                    # psi storage: the slab's range along the axis x the full
                    # local extents of the other two (layout of yee3d_cpml.hip)
                    lb0 = dom.to_local(g)
                    plo, phi = [0, 0, 0], list(dom.shape)
                    plo[axis], phi[axis] = lb0[0][axis], lb0[1][axis]
                    if axis == 2 and dom.shape[2] % 4 == 0:
                        # z slabs padded to whole float4 groups; the padding
                        # cells have c = 0 and 1/kappa - 1 = 0, so their psi
                        # stays 0 and adds nothing
                        plo[2] = plo[2] & ~3
                        phi[2] = min(dom.shape[2], (phi[2] + 3) & ~3)
                    lb = (tuple(plo), tuple(phi))
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

    def kernel_table(self, kind: str, p: int):
        """Term table of the fused CPML kernels (yee3d_cpml.hip) for the
        components of ``kind`` and plane ``p``: per (component, axis) the low /
        high psi slabs, their ranges along the axis, and one b / c / (1/kappa-1)
        profile that selects the side's values inside each slab and the
        identity (1, 0, 0) elsewhere."""
        key = (kind, p)
        cache = getattr(self, "_tables", None)
        if cache is None:
            cache = self._tables = {}
        if key in cache:
            return cache[key]
        s = self.s
        comps = s.e_comps if kind == "E" else s.h_comps
        ptrs, ints, keep = [], [], []
        for c in comps:
            for a in range(3):
                sl = [x for x in self.slabs[c] if x.axis == a]
                psi = [None, None]
                rng = [(0, 0), (0, 0)]
                n = s.domain.shape[a]
                b = torch.ones(n, dtype=s.dtype, device=s.device)
                cc = torch.zeros(n, dtype=s.dtype, device=s.device)
                kk = torch.zeros(n, dtype=s.dtype, device=s.device)
                for x in sl:
                    lo, hi = x.lbox[0][a], x.lbox[1][a]
                    psi[x.side] = x.psi[p]
                    rng[x.side] = (lo, hi)
                    b[lo:hi] = x.b[lo:hi]
                    cc[lo:hi] = x.c[lo:hi]
                    kk[lo:hi] = x.kinv_m1[lo:hi]
                keep += [b, cc, kk]
                ptrs += [None if psi[0] is None else psi[0].data_ptr(), None if psi[1] is None else psi[1].data_ptr(),
                         b.data_ptr(), cc.data_ptr(), kk.data_ptr()]
                ints += [rng[0][0], rng[0][1], rng[1][0], rng[1][1]]
        cache[key] = (ptrs, ints, keep)
        return cache[key]

    def apply(self, kind: str, p: int, boxes) -> None:
        s = self.s
        F = s.F[p]
        items = []
        for c, box in boxes.items():
            if box_empty(box):
                continue
            for sl in self.slabs[c]:
                b = box_intersect(box, sl.lbox)
                if box_empty(b):
                    continue
                items.append((F[c], F[sl.src], sl.axis, sl.sign, sl.psi[p], sl.lbox, b, sl.b, sl.c, sl.kinv_m1,
                              s.cb[c]))
        if len(items) > 1 and hasattr(s.ops, "cpml_apply_many"):
            # one launch per group of slabs that update disjoint cells (2D hybrid
            # shell graphs: a step costs its launches): the slabs of one
            # component overlap in the corners, where two axes' psi both add
            # to a cell -- those go to different groups (launches in order)
            groups = []
            for it in items:
                for g in groups:
                    if all(it[0].data_ptr() != o[0].data_ptr() or box_empty(box_intersect(it[6], o[6])) for o in g):
                        g.append(it)
                        break
                else:
                    groups.append([it])
            for g in groups:
                s.ops.cpml_apply_many(kind, g)
            return
        for it in items:
            s.ops.cpml_apply(kind, *it)

    def state_tensors(self, p: int) -> List[torch.Tensor]:
        return [sl.psi[p] for c in self.slabs for sl in self.slabs[c]]

    def state_boxes(self, p: int):
        """(global slab box, local index of psi[0, 0, 0]) per :meth:`state_tensors`
        entry: the unpadded global box is the same on every rank, so the
        two ends of a halo message clip it identically."""
        return [(sl.gbox, sl.lbox[0]) for c in self.slabs for sl in self.slabs[c]]
