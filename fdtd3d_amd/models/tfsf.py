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
                if layout.incident_projection(s) == 0.0:
                    continue  # the incident wave has no such component: nothing to correct
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
        if sel.any():  # targets' bounding box (lets the op skip the per-entry box test)
            v = ijk[sel].reshape(-1, 3)
            tab.bbox = (tuple(int(x) for x in v.min(0)), tuple(int(x) + 1 for x in v.max(0)))
        layers.append(tab)
    return layers


class TfsfSets:
    """TF/SF corrections in the form the blocked kernels apply them
    (``csrc/yee3d_tb.hip`` TfDev): one *set* per (component, face) -- the box
    of target cells the reference's border tests select
    (``YeeGridLayout.cpp:327-809``), one cell thick across the face -- and,
    per set, the incident-line interpolation (index ``i0``, weights ``w0``,
    ``w1``) and ``sign * projection`` factor at every index along the table
    axis ``va``.  Valid when the incident direction lies along x or y (the
    reference default theta = 90, phi = 0 is +x): the incident value of a
    target then depends on that one index.  Each blocked pass turns the
    entries into per-level g values (``k_tfsf_pass``) that the kernel adds to
    the target's curl, so ``E += Cb * (curl + g)`` equals the table path's
    ``E += Cb * curl; E += Cb * g``."""

    MAX_SETS = 24
    INTS_PER_SET = 10

    def __init__(self):
        self.sets: List[dict] = []
        self.i0 = self.w0 = self.w1 = self.c = None
        self.n_e = self.n_h = 0
        self.xpl = [[-1, -1], [-1, -1]]
        self.dev = None  # int32 device block (TfDev)

    @property
    def ld(self) -> int:
        return self.n_e + self.n_h

    def struct_ints(self) -> np.ndarray:
        v = [len(self.sets), self.ld, self.xpl[0][0], self.xpl[0][1], self.xpl[1][0], self.xpl[1][1]]
        for s in self.sets:
            v += [s["n"], s["fa"]] + list(s["lo"]) + list(s["hi"]) + [s["va"], s["goff"]]
        v += [0] * (self.INTS_PER_SET * (self.MAX_SETS - len(self.sets)))
        return np.asarray(v, dtype=np.int32)


COMP_INDEX = {"Ex": 0, "Ey": 1, "Ez": 2, "Hx": 3, "Hy": 4, "Hz": 5}


def build_tfsf_sets(layout: YeeLayout, comps: Sequence[str], origin: Sequence[int], shape: Sequence[int],
                    boxes: Dict[str, Tuple], device, dtype, line_len: int) -> Optional[TfsfSets]:
    """:class:`TfsfSets` of the local array ``shape`` at ``origin`` (targets
    restricted to ``boxes``, as :func:`build_tfsf_tables`), or None when the
    incident direction is not along x or y (3D only)."""
    if layout.scheme != "3d":
        return None
    L, R = layout.tfsf_borders()
    zero = layout.zero_inc_coord_fp()
    dirv = layout.incident_direction()
    tol = 1e-9
    if abs(dirv[1]) < tol and abs(dirv[2]) < tol:
        va = 0
    elif abs(dirv[0]) < tol and abs(dirv[2]) < tol:
        va = 1
    else:
        return None
    out = TfsfSets()
    ent = {"E": [], "H": []}
    for kind in ("E", "H"):
        for comp in comps:
            if comp[0] != kind:
                continue
            box = boxes[comp]
            if any(box[1][d] <= box[0][d] for d in range(3)):
                continue
            m = MIN_COORD_FP[comp]
            for (s, axis, sign) in layout.curl_terms(comp):
                for dname in "LRDUBF":
                    if DIR_AXIS[dname] != axis or (comp, dname) not in TFSF_PREDICATES:
                        continue
                    if layout.incident_projection(s) == 0.0:
                        continue
                    pred = TFSF_PREDICATES[(comp, dname)]
                    lo, hi = [], []
                    for d in range(3):
                        idx = np.arange(box[0][d], box[1][d])
                        g = idx + origin[d] + m[d]
                        sel = _axis_mask(g, pred[d], L[d], R[d]) if layout.active(d) else np.ones_like(g, bool)
                        if not sel.any():
                            break
                        nzi = np.flatnonzero(sel)
                        if nzi[-1] - nzi[0] + 1 != nzi.size:
                            raise ValueError("TF/SF set is not a box")
                        lo.append(int(idx[nzi[0]]))
                        hi.append(int(idx[nzi[-1]]) + 1)
                    if len(lo) < 3:
                        continue
                    if len(out.sets) >= TfsfSets.MAX_SETS:
                        raise ValueError("too many TF/SF sets")
                    low = DIR_LOW[dname]
                    nb_off = (0 if low else -1) if kind == "E" else (0 if low else +1)
                    ms = MIN_COORD_FP[s]
                    a = np.arange(lo[va], hi[va])
                    pos = []
                    for d in range(3):
                        base = a if d == va else np.full(a.shape, lo[d])
                        pos.append(base + (nb_off if d == axis else 0) + origin[d] + ms[d])
                    dd = sum((pos[d] - zero[d]) * dirv[d] for d in range(3))
                    dd = dd - (0.5 if kind == "E" else 0.0)
                    i0 = np.floor(dd).astype(np.int64)
                    if (i0 < 0).any() or (i0 + 1 >= line_len).any():
                        raise ValueError("TF/SF box does not fit the incident line")
                    w1 = dd - i0
                    tsign = -sign if low else sign
                    cval = np.full(a.shape, tsign * layout.incident_projection(s))
                    out.sets.append({"n": COMP_INDEX[comp], "fa": axis, "lo": tuple(lo), "hi": tuple(hi), "va": va,
                                     "goff": 0, "kind": kind})
                    ent[kind].append((i0, 1.0 - w1, w1, cval))
    # E sets first: g index space [E entries | H entries]
    goff = 0
    parts = []
    for kind in ("E", "H"):
        k = 0 if kind == "E" else 1
        planes = set()
        for s_, e in zip([s for s in out.sets if s["kind"] == kind], ent[kind]):
            s_["goff"] = goff
            goff += e[0].size
            parts.append(e)
            if s_["fa"] == 0:
                planes.add(s_["lo"][0])
        planes = sorted(planes)
        if len(planes) > 2:
            raise ValueError("more than two TF/SF x-face planes per kind")
        for q, pl in enumerate(planes):
            out.xpl[k][q] = pl
        if kind == "E":
            out.n_e = goff
    out.n_h = goff - out.n_e
    out.sets.sort(key=lambda s_: 0 if s_["kind"] == "E" else 1)
    if not parts:
        return None
    cat = lambda i: np.concatenate([p[i] for p in parts])
    out.i0 = torch.as_tensor(cat(0).astype(np.int32), device=device)
    out.w0 = torch.as_tensor(cat(1), device=device, dtype=dtype)
    out.w1 = torch.as_tensor(cat(2), device=device, dtype=dtype)
    out.c = torch.as_tensor(cat(3), device=device, dtype=dtype)
    out.dev = torch.as_tensor(out.struct_ints(), device=device)
    return out
