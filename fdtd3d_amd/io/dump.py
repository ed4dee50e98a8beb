"""Field output used by the driver: final / intermediate / scattered-field dumps
and material dumps (reference ``Scheme3D.cpp:2314-2940`` and
``initGrids`` BMP dumps), in any of the DAT / BMP / TXT formats.

Decomposed runs either write per-rank files of the local grid (reference
behaviour, ``rank-<pid>`` in the name) or, with ``--gather-full-grid``, gather
the owned blocks on rank 0 and write one global file there.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import torch

from ..layout.yee import MIN_COORD_FP
from .bmp import BMPDumper
from .dat import DATDumper
from .naming import GridFileType
from .txt import TXTDumper


def selected_components(settings, comps: Sequence[str]) -> List[str]:
    only = [c for c in comps if getattr(settings, "save%sOnly" % c, False)]
    return only or list(comps)


def formats(settings) -> List[str]:
    f = []
    if settings.saveAsDAT:
        f.append("dat")
    if settings.saveAsTXT:
        f.append("txt")
    if settings.saveAsBMP or not f:
        f.append("bmp")
    return f


def incident_field(scheme, comp: str, plane: int = 0) -> Optional[torch.Tensor]:
    """Incident plane-wave value of ``comp`` at every local cell (TF/SF runs),
    interpolated from the 1D line exactly like the TF/SF corrections."""
    if not scheme.cfg.use_tfsf:
        return None
    lay = scheme.layout
    zero = lay.zero_inc_coord_fp()
    dirv = lay.incident_direction()
    m = MIN_COORD_FP[comp]
    o = scheme.domain.origin
    shp = scheme.domain.shape
    dev = scheme.device
    ax = [torch.arange(shp[a], device=dev, dtype=torch.float64) + o[a] + m[a] for a in range(3)]
    X, Y, Z = torch.meshgrid(ax[0], ax[1], ax[2], indexing="ij")
    d = (X - zero[0]) * dirv[0] + (Y - zero[1]) * dirv[1] + (Z - zero[2]) * dirv[2]
    line = scheme.einc[plane] if comp[0] == "E" else scheme.hinc[plane]
    if comp[0] == "H":
        d = d - 0.5
    i0 = torch.clamp(torch.floor(d).long(), 0, line.numel() - 2)
    w1 = d - i0
    lv = line.to(torch.float64)
    v = (1 - w1) * lv[i0] + w1 * lv[i0 + 1]
    return (v * lay.incident_projection(comp)).to(scheme.dtype)


def scattered_field(scheme, comp: str, plane: int = 0) -> torch.Tensor:
    """Total field minus the incident field inside the TF box (outside it the
    grid already holds the scattered field) -- ``Scheme3D.cpp:2593-2747``.
    HIP: one kernel pass (``ops.scattered``); torch: the expression below."""
    f = scheme.F[plane][comp]
    if not scheme.cfg.use_tfsf:
        return f
    if hasattr(scheme.ops, "scattered"):
        lay = scheme.layout
        L, R = lay.tfsf_borders()
        act = 0
        for a in lay.axes:
            act |= 1 << a
        geo = (list(MIN_COORD_FP[comp]) + list(lay.zero_inc_coord_fp()) + list(lay.incident_direction())
               + [float(v) for v in L] + [float(v) for v in R]
               + [float(lay.incident_projection(comp)), 0.5 if comp[0] == "H" else 0.0])
        line = scheme.einc[plane] if comp[0] == "E" else scheme.hinc[plane]
        return scheme.ops.scattered(f, line, geo, list(scheme.domain.origin) + [act])
    return scattered_field_torch(scheme, comp, plane)


def scattered_field_torch(scheme, comp: str, plane: int = 0) -> torch.Tensor:
    """Torch expression of :func:`scattered_field` (any backend / device)."""
    f = scheme.F[plane][comp]
    inc = incident_field(scheme, comp, plane)
    L, R = scheme.layout.tfsf_borders()
    m = MIN_COORD_FP[comp]
    o = scheme.domain.origin
    shp = scheme.domain.shape
    mask = torch.ones(shp, dtype=torch.bool, device=f.device)
    for a in scheme.layout.axes:
        idx = torch.arange(shp[a], device=f.device, dtype=torch.float64) + o[a] + m[a]
        inside = (idx > L[a]) & (idx < R[a])
        view = [1, 1, 1]
        view[a] = -1
        mask = mask & inside.view(view)
    return torch.where(mask, f - inc, f)


def dump_fields(scheme, settings, step: int, name_prefix: str = "", scattered: bool = False,
                directory: Optional[str] = None) -> List[str]:
    from ..parallel.halo import gather_field, gather_owned
    directory = directory or settings.outputDir
    rank = scheme.domain.rank
    gather = settings.doGatherFullGrid and scheme.halo is not None
    files: List[str] = []
    dim = {"3d": 3, "tmz": 2, "tez": 2, "1d": 1}[scheme.cfg.scheme]
    for c in selected_components(settings, scheme.comps):
        parts = []
        for p in range(scheme.planes):
            t = scattered_field(scheme, c, p) if scattered else scheme.F[p][c]
            if gather:
                # gather_field works on the scheme's fields; scattered output gathers the owned view
                if scattered:
                    gl = scheme.domain.ghost_lo
                    s = scheme.domain.owned_shape
                    own = t[gl[0]:gl[0] + s[0], gl[1]:gl[1] + s[1], gl[2]:gl[2] + s[2]]
                    full = gather_owned(scheme, own)
                else:
                    full = gather_field(scheme, c, p)
                parts.append(full)
            else:
                parts.append(t)
        if gather and rank != 0:
            continue
        re = parts[0]
        im = parts[1] if scheme.planes == 2 else None
        if re is None:
            continue
        name = "%s%s" % (name_prefix, c)
        for fmt in formats(settings):
            if fmt == "dat":
                files += DATDumper(step, GridFileType.CURRENT, rank, name, directory).dump_grid(re, im)
            elif fmt == "txt":
                files += TXTDumper(step, GridFileType.CURRENT, rank, name, directory).dump_grid(re, dim=dim)
            else:
                d = BMPDumper(step, GridFileType.CURRENT, rank, name, directory, settings.dumperPalette,
                              settings.dumperOrthAxis)
                if dim == 3:
                    # one slice through the middle of the grid along the orthogonal axis,
                    # as the reference's final dump (Scheme3D.cpp:1908-1960)
                    ax = settings.dumperOrthAxis
                    mid = re.shape[ax] // 2
                    start = [0, 0, 0]
                    end = list(re.shape)
                    start[ax], end[ax] = mid, mid + 1
                    files += d.dump_grid(re, im, start, end, dim=3)
                else:
                    files += d.dump_grid(re, im, dim=dim)
    return files


def dump_materials(scheme, settings, directory: Optional[str] = None) -> List[str]:
    """Eps / Mu (and Drude omega/gamma with metamaterials) on the eps layout of
    the local region (reference ``initGrids`` dumps)."""
    directory = directory or settings.outputDir
    rank = scheme.domain.rank
    names = ["eps", "mu"]
    if scheme.cfg.use_metamaterials:
        names += ["omega_pe", "gamma_e", "omega_pm", "gamma_m"]
    labels = {"eps": "Eps", "mu": "Mu", "omega_pe": "OmegaPE", "gamma_e": "GammaE", "omega_pm": "OmegaPM",
              "gamma_m": "GammaM"}
    files = []
    dim = {"3d": 3, "tmz": 2, "tez": 2, "1d": 1}[scheme.cfg.scheme]
    for n in names:
        g = scheme.sampler.grid(n)
        for fmt in formats(settings):
            if fmt == "dat":
                files += DATDumper(0, GridFileType.CURRENT, rank, labels[n], directory).dump_grid(g)
            elif fmt == "txt":
                files += TXTDumper(0, GridFileType.CURRENT, rank, labels[n], directory).dump_grid(g, dim=dim)
            else:
                d = BMPDumper(0, GridFileType.CURRENT, rank, labels[n], directory, settings.dumperPalette,
                              settings.dumperOrthAxis)
                if dim == 3:
                    ax = settings.dumperOrthAxis
                    mid = g.shape[ax] // 2
                    start, end = [0, 0, 0], list(g.shape)
                    start[ax], end[ax] = mid, mid + 1
                    files += d.dump_grid(g, None, start, end, dim=3)
                else:
                    files += d.dump_grid(g, None, dim=dim)
    return files
