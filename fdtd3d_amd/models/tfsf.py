"""Total-field / scattered-field plane-wave injection.

Reference behaviour (``Scheme3D.cpp:25-208``, ``YeeGridLayout.cpp:327-845``):
an auxiliary 1D FDTD line carries the incident wave (hard
``sin(2 pi f dt t)`` source at index 0, numerical phase velocity matched to the
3D grid through ``relPhaseVelocity``).  Every field cell whose curl stencil
straddles the TF/SF box face gets its straddling neighbour corrected by the
incident field interpolated on the line at that neighbour's position:

* E cells outside a low face (LEFT/DOWN/BACK) see ``S_hi -= inc``; outside a
  high face ``S_lo -= inc``;
* H cells on a low face see ``S_lo += inc``; on a high face ``S_hi += inc``.

Because the update is linear, the correction is equivalent to adding
``coef * inc`` to the updated cell, with ``coef = Cb * (-/+ sign_of_term) *
projection``.  This module turns the reference's per-cell FP predicates into
static *correction tables* (local flat offset, line index, interpolation
weights, coefficient) once at init; each step a tiny kernel applies them, so
the stencil kernels stay branch-free.  Tables are split into layers with
unique target cells so application is deterministic without atomics.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..layout.yee import MIN_COORD_FP, YeeLayout
from ..ops.coef import Coef
from ..ops.torch_ops import TfsfTable

# (component, direction) -> per-axis open intervals (ref, off_lo, ref, off_hi);
# the third entry is flagged when it comes from the reference's "is3Dim" clause.
# Directions: L/R (x), D/U (y), B/F (z).
_I = lambda a, b, c, d: (a, b, c, d)
TFSF_PREDICATES = {
    ("Ex", "D"): (_I("L", -.5, "R", .5), _I("L", -1, "L", 0), _I("L", 0, "R", 0)),
    ("Ex", "U"): (_I("L", -.5, "R", .5), _I("R", 0, "R", 1), _I("L", 0, "R", 0)),
    ("Ex", "B"): (_I("L", -.5, "R", .5), _I("L", 0, "R", 0), _I("L", -1, "L", 0)),
    ("Ex", "F"): (_I("L", -.5, "R", .5), _I("L", 0, "R", 0), _I("R", 0, "R", 1)),
    ("Ey", "L"): (_I("L", -1, "L", 0), _I("L", -.5, "R", .5), _I("L", 0, "R", 0)),
    ("Ey", "R"): (_I("R", 0, "R", 1), _I("L", -.5, "R", .5), _I("L", 0, "R", 0)),
    ("Ey", "B"): (_I("L", 0, "R", 0), _I("L", -.5, "R", .5), _I("L", -1, "L", 0)),
    ("Ey", "F"): (_I("L", 0, "R", 0), _I("L", -.5, "R", .5), _I("R", 0, "R", 1)),
    ("Ez", "L"): (_I("L", -1, "L", 0), _I("L", 0, "R", 0), _I("L", -.5, "R", .5)),
    ("Ez", "R"): (_I("R", 0, "R", 1), _I("L", 0, "R", 0), _I("L", -.5, "R", .5)),
    ("Ez", "D"): (_I("L", 0, "R", 0), _I("L", -1, "L", 0), _I("L", -.5, "R", .5)),
    ("Ez", "U"): (_I("L", 0, "R", 0), _I("R", 0, "R", 1), _I("L", -.5, "R", .5)),
    ("Hx", "D"): (_I("L", 0, "R", 0), _I("L", -.5, "L", .5), _I("L", -.5, "R", .5)),
    ("Hx", "U"): (_I("L", 0, "R", 0), _I("R", -.5, "R", .5), _I("L", -.5, "R", .5)),
    ("Hx", "B"): (_I("L", 0, "R", 0), _I("L", -.5, "R", .5), _I("L", -.5, "L", .5)),
    ("Hx", "F"): (_I("L", 0, "R", 0), _I("L", -.5, "R", .5), _I("R", -.5, "R", .5)),
    ("Hy", "L"): (_I("L", -.5, "L", .5), _I("L", 0, "R", 0), _I("L", -.5, "R", .5)),
    ("Hy", "R"): (_I("R", -.5, "R", .5), _I("L", 0, "R", 0), _I("L", -.5, "R", .5)),
    ("Hy", "B"): (_I("L", -.5, "R", .5), _I("L", 0, "R", 0), _I("L", -.5, "L", .5)),
    ("Hy", "F"): (_I("L", -.5, "R", .5), _I("L", 0, "R", 0), _I("R", -.5, "R", .5)),
    ("Hz", "L"): (_I("L", -.5, "L", .5), _I("L", -.5, "R", .5), _I("L", 0, "R", 0)),
    ("Hz", "R"): (_I("R", -.5, "R", .5), _I("L", -.5, "R", .5), _I("L", 0, "R", 0)),
    ("Hz", "D"): (_I("L", -.5, "R", .5), _I("L", -.5, "L", .5), _I("L", 0, "R", 0)),
    ("Hz", "U"): (_I("L", -.5, "R", .5), _I("R", -.5, "R", .5), _I("L", 0, "R", 0)),
}
DIR_AXIS = {"L": 0, "R": 0, "D": 1, "U": 1, "B": 2, "F": 2}
DIR_LOW = {"L": True, "D": True, "B": True, "R": False, "U": False, "F": False}


def incident_line_length(size: Sequence[int], scheme: str) -> int:
    """Length of the auxiliary line (Scheme3D.h:216-217: 100*(Nx+Ny+Nz);
    SchemeTMz.h:186: 100*(Nx+Ny))."""
    if scheme == "3d":
        return 100 * (size[0] + size[1] + size[2])
    return 100 * (size[0] + size[1])


def _axis_mask(coords: np.ndarray, iv, L, R) -> np.ndarray:
    ra, oa, rb, ob = iv
    lo = (L if ra == "L" else R) + oa
    hi = (L if rb == "L" else R) + ob
    return (coords > lo) & (coords < hi)


def build_tfsf_tables(layout: YeeLayout, comps: Sequence[str], origin: Sequence[int], shape: Sequence[int],
                      boxes: Dict[str, Tuple], coefs: Dict[str, Coef], device, dtype,
                      line_len: int) -> Dict[str, List[TfsfTable]]:
    """Correction tables for each component, restricted to cells of ``boxes``
    (local computation boxes) of the local array ``shape`` at ``origin``.

    ``coefs[comp]`` is the coefficient multiplying the curl in the update that
    receives the correction (Cb for the plain update, CbD for the UPML D/B
    update)."""
    L, R = layout.tfsf_borders()
    zero = layout.zero_inc_coord_fp()
    dirv = layout.incident_direction()
    is3 = layout.scheme == "3d"
    out: Dict[str, List[TfsfTable]] = {}
    for comp in comps:
        kind = "E" if comp[0] == "E" else "H"
        box = boxes[comp]
        if any(box[1][d] <= box[0][d] for d in range(3)):
            out[comp] = []
            continue
        # local index ranges of the box -> global FP coordinates of comp
        rng = [np.arange(box[0][d], box[1][d]) for d in range(3)]
        m = MIN_COORD_FP[comp]
        entries = []  # (flat_local_offsets, i0, w0, w1, coef)
        for (s, axis, sign) in layout.curl_terms(comp):
            for dname in ("LRDUBF"):
                if DIR_AXIS[dname] != axis or (comp, dname) not in TFSF_PREDICATES:
                    continue
                pred = TFSF_PREDICATES[(comp, dname)]
                masks = []
                for d in range(3):
                    g = rng[d] + origin[d] + m[d]
                    if not layout.active(d):
                        masks.append(np.ones_like(g, dtype=bool))
                        continue
                    if d == 2 and not is3:
                        masks.append(np.ones_like(g, dtype=bool))
                        continue
                    masks.append(_axis_mask(g, pred[d], L[d], R[d]))
                if not (masks[0].any() and masks[1].any() and masks[2].any()):
                    continue
                ii, jj, kk = np.meshgrid(rng[0][masks[0]], rng[1][masks[1]], rng[2][masks[2]], indexing="ij")
                ii, jj, kk = ii.ravel(), jj.ravel(), kk.ravel()
                low = DIR_LOW[dname]
                # neighbour whose incident value is used
                if kind == "E":
                    nb_off = 0 if low else -1
                else:
                    nb_off = 0 if low else +1
                nidx = [ii.copy(), jj.copy(), kk.copy()]
                nidx[axis] = nidx[axis] + nb_off
                ms = MIN_COORD_FP[s]
                pos = [nidx[d] + origin[d] + ms[d] for d in range(3)]
                dd = sum((pos[d] - zero[d]) * dirv[d] for d in range(3) if layout.active(d) or d < 2)
                if kind == "H":
                    dd = dd - 0.0  # H cells read the E line: approximateIncidentWaveE (offset 0)
                else:
                    dd = dd - 0.5  # E cells read the H line: approximateIncidentWaveH (offset 0.5)
                i0 = np.floor(dd).astype(np.int64)  # d > 0 inside the grid: truncation == floor
                w1 = dd - i0
                w0 = 1.0 - w1
                if (i0 < 0).any() or (i0 + 1 >= line_len).any():
                    raise ValueError("TF/SF box does not fit the incident line")
                proj = layout.incident_projection(s)
                tsign = -sign if low else sign
                lidx = torch.as_tensor(np.stack([ii, jj, kk], axis=1), device=device)
                cval = coefs[comp].at_many(lidx).cpu().numpy() * tsign * proj
                flat = (ii * shape[1] + jj) * shape[2] + kk
                entries.append((flat, i0, w0, w1, cval, np.stack([ii, jj, kk], axis=1)))
        out[comp] = _layer(entries, device, dtype)
    return out


def _layer(entries, device, dtype) -> List[TfsfTable]:
    if not entries:
        return []
    flat = np.concatenate([e[0] for e in entries])
    i0 = np.concatenate([e[1] for e in entries])
    w0 = np.concatenate([e[2] for e in entries])
    w1 = np.concatenate([e[3] for e in entries])
    cv = np.concatenate([e[4] for e in entries])
    ijk = np.concatenate([e[5] for e in entries])
    order = np.argsort(flat, kind="stable")
    flat, i0, w0, w1, cv, ijk = flat[order], i0[order], w0[order], w1[order], cv[order], ijk[order]
    # rank of each entry among equal targets -> layer id
    first = np.r_[True, flat[1:] != flat[:-1]]
    grp = np.cumsum(first) - 1
    starts = np.flatnonzero(first)
    rank = np.arange(flat.size) - starts[grp]
    layers = []
    for r in range(int(rank.max()) + 1):
        sel = rank == r
        tab = TfsfTable(torch.as_tensor(flat[sel], device=device),
                                torch.as_tensor(i0[sel], device=device),
                                torch.as_tensor(w0[sel], device=device, dtype=dtype),
                                torch.as_tensor(w1[sel], device=device, dtype=dtype),
                                torch.as_tensor(cv[sel], device=device, dtype=dtype),
                                torch.as_tensor(ijk[sel].astype(np.int32), device=device))
        # host-side bounds of the table (checked by the HIP op without a device sync)
        tab.max_off = int(flat[sel].max()) if sel.any() else -1
        tab.max_inc = int(i0[sel].max()) + 1 if sel.any() else -1
        layers.append(tab)
    return layers
