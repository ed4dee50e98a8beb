"""Near-to-far-field transform: scattered power diagram.

Same observable as the reference's ``Scheme3D::Pointing_scat / Pointing_inc``
(``Scheme3D.cpp:2263-2307, 4093-4509``): on a closed box surface the
tangential fields define equivalent currents ``J = n x H`` and
``M = -n x E``; their radiation vectors

    N = sum_faces sum_cells J exp(i k r_hat . r') dS,   L = (same with M)

give the far-field power per unit solid angle, normalised by the incident
plane-wave intensity ``1/eta0``:

    P(theta, phi) = k^2 / (8 pi eta0) (|L_phi + eta0 N_theta|^2 + |L_theta - eta0 N_phi|^2) * eta0.

Differences from the reference, all deliberate:

* every angle of the diagram is evaluated at once: the face sums are complex
  matrix-vector products ``exp(i k r_hat(phi) . r') @ J`` (torch on the
  solver's device);
* the box is set by ``--ntff-size{x,y,z}`` (the reference hard-codes 13 cells,
  ``Scheme3D.h:231-232``, and ignores the option);
* real-valued runs are handled as complex fields with zero imaginary part
  (the reference only builds 3D with complex values).

Tangential fields are brought to the face-cell centres by averaging the two
(H) or four (E) nearest Yee samples.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..layout.yee import MIN_COORD_FP
from ..utils.constants import EPS0, MU0, PI

ETA0 = math.sqrt(MU0 / EPS0)


def _sample_plan(comp: str, axis: int, x0: float, lo: Sequence[float], hi: Sequence[float]):
    """Per axis (first index, count, offsets): averaging the Yee samples at
    ``first + offset`` (0 or 0 and 1) gives ``comp`` at the face-cell
    centres of the face ``axis = x0`` spanning ``[lo, hi)`` along the two
    other axes (centres at lo+0.5 ...)."""
    m = MIN_COORD_FP[comp]
    idx_sets = []
    for a in range(3):
        if a == axis:
            targets = [float(x0)]
        else:
            n = int(round(hi[a] - lo[a]))
            targets = [lo[a] + 0.5 + t for t in range(n)]
        first = targets[0] - m[a]
        if abs(first - round(first)) < 1e-9:
            offs = [0]
            base = int(round(first))
        else:
            offs = [0, 1]
            base = int(math.floor(first))
        idx_sets.append((base, len(targets), offs))
    return idx_sets


def _plan_box(idx_sets):
    """Global index box the samples of a plan read."""
    return (tuple(b for b, _, _ in idx_sets), tuple(b + n + max(o) for b, n, o in idx_sets))


def _sample_from(Fb: torch.Tensor, origin: Sequence[int], idx_sets, axis: int) -> torch.Tensor:
    """Face-centre values from ``Fb``, the global box starting at ``origin``.
    Returns a 2D tensor (other axes in increasing order)."""
    acc = None
    cnt = 0
    for ox in idx_sets[0][2]:
        for oy in idx_sets[1][2]:
            for oz in idx_sets[2][2]:
                o = (ox, oy, oz)
                sl = tuple(slice(idx_sets[a][0] - origin[a] + o[a], idx_sets[a][0] - origin[a] + o[a] + idx_sets[a][1])
                           for a in range(3))
                v = Fb[sl]
                acc = v if acc is None else acc + v
                cnt += 1
    return (acc / cnt).squeeze(axis)


def _sample(F: torch.Tensor, comp: str, axis: int, x0: float, lo: Sequence[float], hi: Sequence[float]):
    """Face-centre values of ``comp`` from the full global array ``F``."""
    return _sample_from(F, (0, 0, 0), _sample_plan(comp, axis, x0, lo, hi), axis)


def _faces(size, ntff):
    """(axis, x0, sign, lo, hi) of the six faces of the NTFF box."""
    L = [float(ntff[a]) for a in range(3)]
    R = [float(size[a] - ntff[a]) for a in range(3)]
    return [(axis, x0, s, L, R) for axis in range(3) for x0, s in ((L[axis], -1.0), (R[axis], 1.0))]


def ntff_requests(size, ntff) -> List[Tuple[str, Tuple]]:
    """Every (component, global index box) the diagram reads: two-cell-thick
    slabs around the six faces -- all a decomposed run has to gather (instead
    of the whole grid)."""
    req = []
    for axis, x0, _, lo, hi in _faces(size, ntff):
        for a in range(3):
            if a == axis:
                continue
            for comp in ("H" + "xyz"[a], "E" + "xyz"[a]):
                req.append((comp, _plan_box(_sample_plan(comp, axis, x0, lo, hi))))
    return req


def ntff_power(fields_re: Optional[Dict[str, torch.Tensor]], fields_im: Optional[Dict[str, torch.Tensor]], size, ntff,
               dx: float, wavelength: float, theta: float, phis: torch.Tensor, boxes=None) -> torch.Tensor:
    """Normalised scattered power for every angle in ``phis`` (radians) at
    polar angle ``theta``.  ``fields_*`` are full global grids, or (``boxes``
    given) dicts (component, box) -> the gathered ``ntff_requests`` slabs."""
    dev = (fields_re["Ex"] if boxes is None else next(iter(fields_re.values()))).device
    cdt = torch.complex128
    k = 2 * PI / wavelength
    L = [float(ntff[a]) for a in range(3)]
    R = [float(size[a] - ntff[a]) for a in range(3)]
    center = size[0] / 2.0  # the reference measures r' from Nx/2 on every axis (Scheme3D.cpp:4098)
    phis = phis.to(dev, torch.float64)
    st, ct = math.sin(theta), math.cos(theta)
    rhat = torch.stack([st * torch.cos(phis), st * torch.sin(phis), torch.full_like(phis, ct)], dim=1)  # (A, 3)

    def face(comp, axis, x0, lo, hi):
        plan = _sample_plan(comp, axis, x0, lo, hi)
        pb = _plan_box(plan)
        if boxes is None:
            # slice the (thin) slab the face reads before any conversion: a
            # whole-grid .to(float64) per face and component would dominate
            sl = tuple(slice(pb[0][a], pb[1][a]) for a in range(3))
            get = lambda f: f[comp][sl]
        else:
            get = lambda f: f[(comp, pb)]
        origin = pb[0]
        re = _sample_from(get(fields_re).to(torch.float64), origin, plan, axis)
        im = (_sample_from(get(fields_im).to(torch.float64), origin, plan, axis) if fields_im is not None
              else torch.zeros_like(re))
        return torch.complex(re, im)

    Nvec = torch.zeros(phis.numel(), 3, dtype=cdt, device=dev)
    Lvec = torch.zeros(phis.numel(), 3, dtype=cdt, device=dev)
    for axis in range(3):
        for x0, s in ((L[axis], -1.0), (R[axis], 1.0)):
            others = [a for a in range(3) if a != axis]
            lo = [L[a] for a in range(3)]
            hi = [R[a] for a in range(3)]
            Ht, Et = {}, {}
            for a in others:
                Ht[a] = face("H" + "xyz"[a], axis, x0, lo, hi)
                Et[a] = face("E" + "xyz"[a], axis, x0, lo, hi)
            # n = s e_axis;  J = n x H ; M = -n x E
            a1, a2 = others  # cyclic order check: e_axis x e_a1 = +/- e_a2
            cyc = 1.0 if (a1 - axis) % 3 == 1 else -1.0
            J = {a2: s * cyc * Ht[a1], a1: -s * cyc * Ht[a2]}
            M = {a2: -s * cyc * Et[a1], a1: s * cyc * Et[a2]}
            # The phase exp(-i k r_hat . r') of a face-cell centre r' factors
            # over the face's two axes: exp(-i k rh[axis] x0') exp(-i k rh[a1]
            # u') exp(-i k rh[a2] v').  So each face sum is one batched GEMM
            # over v (face values x v-phases) and a weighted sum over u --
            # U V A complex multiply-adds on the BLAS path and (U + V) A
            # exponentials, instead of U V A exponentials.  (Fields carry
            # exp(-i w t): source sin + i cos = i exp(-i w t).)
            nu, nv = int(round(hi[a1] - lo[a1])), int(round(hi[a2] - lo[a2]))
            u = (torch.arange(nu, device=dev, dtype=torch.float64) + lo[a1] + 0.5 - center) * dx
            v = (torch.arange(nv, device=dev, dtype=torch.float64) + lo[a2] + 0.5 - center) * dx
            eu = torch.exp(-1j * k * torch.outer(rhat[:, a1], u).to(cdt))          # (A, U)
            ev = torch.exp(-1j * k * torch.outer(rhat[:, a2], v).to(cdt))          # (A, V)
            e0 = torch.exp(-1j * k * (rhat[:, axis] * ((x0 - center) * dx)).to(cdt)) * (dx * dx)  # (A,)
            keys = [(Nvec, ca, val) for ca, val in J.items()] + [(Lvec, ca, val) for ca, val in M.items()]
            vals = torch.stack([kv[2] for kv in keys])                              # (C, U, V)
            t1 = torch.matmul(vals, ev.transpose(0, 1))                             # (C, U, A)
            sums = (t1 * eu.transpose(0, 1).unsqueeze(0)).sum(dim=1) * e0           # (C, A)
            for (acc, ca, _), sm in zip(keys, sums):
                acc[:, ca] += sm
    cp, sp = torch.cos(phis).to(cdt), torch.sin(phis).to(cdt)
    N_th = Nvec[:, 0] * ct * cp + Nvec[:, 1] * ct * sp - Nvec[:, 2] * st
    N_ph = -Nvec[:, 0] * sp + Nvec[:, 1] * cp
    L_th = Lvec[:, 0] * ct * cp + Lvec[:, 1] * ct * sp - Lvec[:, 2] * st
    L_ph = -Lvec[:, 0] * sp + Lvec[:, 1] * cp
    p = (k * k) / (8 * PI * ETA0) * ((L_ph + ETA0 * N_th).abs() ** 2 + (L_th - ETA0 * N_ph).abs() ** 2)
    return (p / (1.0 / ETA0)).real if torch.is_complex(p) else p / (1.0 / ETA0)


def reference_angles() -> torch.Tensor:
    """phi in [0, 2 pi + pi/180] with step pi/90 (Scheme3D.cpp:2283)."""
    out = []
    a = 0.0
    while a <= 2 * PI + PI / 180:
        out.append(a)
        a += PI / 90
    return torch.tensor(out, dtype=torch.float64)


def ntff_report(scheme, t: int, out=None) -> Optional[torch.Tensor]:
    """Evaluate the diagram for the scheme's current fields (gathering a
    decomposed run on rank 0) and print the reference's report lines."""
    import sys
    from ..parallel.halo import gather_box
    out = out or sys.stdout
    comps = ("Ex", "Ey", "Ez", "Hx", "Hy", "Hz")
    phis = reference_angles()
    if scheme.halo is not None:
        # decomposed: gather only the face slabs the diagram reads on rank 0
        req = ntff_requests(scheme.cfg.size, scheme.cfg.ntff_size)
        re = {key: gather_box(scheme, key[0], key[1], 0) for key in req}
        im = {key: gather_box(scheme, key[0], key[1], 1) for key in req} if scheme.planes == 2 else None
        if any(v is None for v in re.values()):
            return None
        p = ntff_power(re, im, scheme.cfg.size, scheme.cfg.ntff_size, scheme.dx, scheme.wavelength,
                       scheme.layout.theta, phis, boxes=True)
    else:
        re = {c: scheme.owned_field(c, 0) for c in comps}
        im = {c: scheme.owned_field(c, 1) for c in comps} if scheme.planes == 2 else None
        p = ntff_power(re, im, scheme.cfg.size, scheme.cfg.ntff_size, scheme.dx, scheme.wavelength,
                       scheme.layout.theta, phis)
    for a, v in zip(phis.tolist(), p.cpu().tolist()):
        out.write("=== t=%u, inc angle=%f; angle %f === %.17g \n" % (t, scheme.layout.phi, a, v))
    return p
