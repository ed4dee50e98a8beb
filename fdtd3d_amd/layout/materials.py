"""Material scenes and per-component material averaging.

Materials live on the *eps layout* (cell centres, FP coordinate ``m + 0.5`` of
index ``m``; a grid twice as fine with ``--use-double-material-precision``),
exactly as the reference's ``Eps``/``Mu``/``Omega*``/``Gamma*`` grids
(``Scheme3D.cpp:3405-3660``).  Instead of storing those grids globally, each rank
evaluates the scene analytically on the part of the eps layout its allocated
region touches, then averages it onto every field component with the stencils
of :mod:`.yee` (``YeeGridLayout.h:1007-1263``).  The result feeds the update
coefficients; the hot loop never does layout math.

Scenes:

* ``reference`` -- the reference's hard-coded setups.  3D: eps=2 sphere at
  (40.5, 40.5, 40.5), r=20, with linear sub-cell smoothing; Drude electric
  sphere omega_p = sqrt(2)*2*pi*f at (57, 57, 23), r=8; magnetic Drude box
  [55,60)x[55,65)x[15,25) (``Scheme3D.cpp:3413-3532``).  TMz/TEz: vacuum
  with Drude boxes x in [437,487), y in [405,505) (``SchemeTMz.cpp:1966-2040``).
  The Drude parts are used only with ``--use-metamaterials``.
* ``vacuum`` -- eps = mu = 1 everywhere (headline benchmark).
* ``sphere`` -- one dielectric sphere from ``--sphere-*`` options.
* ``drude-sphere`` -- one electric Drude sphere (eps_inf = 1, omega_p =
  sqrt(2)*2*pi*f as in the reference scene, gamma = 0) at ``--sphere-center-*``
  with ``--sphere-radius``, in vacuum (BASELINE config 4).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch

from .approximation import approximate_drude, approximate_material, approximate_sphere
from .yee import MATERIAL_STENCIL, MATERIAL_STENCIL_DOUBLE, YeeLayout

SQRT2_F32 = float(np.float32(np.sqrt(np.float32(2.0))))  # reference uses sqrtf(2.0)


@dataclass
class Scene:
    kind: str = "reference"
    scheme: str = "3d"
    source_frequency: float = 1.0
    sphere_eps: float = 2.0
    sphere_radius: float = 20.0
    sphere_center: Tuple[float, float, float] = (40.5, 40.5, 40.5)

    # ------------------------------------------------------------------
    def _coords(self, lo: Sequence[int], shape: Sequence[int], mod: float, device, dtype):
        axes = []
        for d in range(3):
            axes.append(torch.arange(lo[d], lo[d] + shape[d], device=device, dtype=dtype) + 0.5)
        x, y, z = torch.meshgrid(axes[0], axes[1], axes[2], indexing="ij")
        return x, y, z

    def is_vacuum(self, metamaterials: bool) -> bool:
        if self.kind == "vacuum" or (self.kind == "drude-sphere" and not metamaterials):
            return True
        if self.kind == "reference" and self.scheme != "3d" and not metamaterials:
            return True
        return False

    def percell_kinds(self, metamaterials: bool) -> int:
        """Number of field kinds (E, H) whose plain update coefficient varies
        per cell -- the count ``models/blocking.py auto_time_block`` takes (the
        scheme derives the same count from its coefficients).  Every scene has
        mu = 1, so at most the E kind."""
        return 0 if self.is_vacuum(metamaterials) else 1

    def eps(self, x, y, z, mod: float) -> torch.Tensor:
        if self.kind in ("vacuum", "drude-sphere") or (self.kind == "reference" and self.scheme != "3d"):
            return torch.ones_like(x)
        if self.kind in ("reference", "sphere"):
            c = tuple(v * mod for v in self.sphere_center)
            if self.scheme == "3d":
                return approximate_sphere(x, y, z, c, self.sphere_radius * mod, self.sphere_eps)
            return approximate_sphere(x, y, torch.full_like(z, c[2]), c, self.sphere_radius * mod, self.sphere_eps)
        raise ValueError("unknown scene %r" % self.kind)

    def mu(self, x, y, z, mod: float) -> torch.Tensor:
        return torch.ones_like(x)

    def uniform(self, name: str) -> Optional[float]:
        """The value of material ``name`` when it is the same everywhere in
        this scene (None: it varies) -- lets the scheme keep a scalar instead
        of evaluating and averaging a full fp64 grid (8 GB per array at
        1024^3)."""
        two_d_ref = self.kind == "reference" and self.scheme != "3d"
        if name == "eps":
            return 1.0 if self.kind in ("vacuum", "drude-sphere") or two_d_ref else None
        if name == "mu":
            return 1.0
        if name in ("gamma_e", "gamma_m"):
            return 0.0
        if name == "omega_pe":
            return None if self.kind in ("drude-sphere", "reference") else 0.0
        if name == "omega_pm":
            return None if self.kind == "reference" else 0.0
        raise ValueError("unknown material %r" % name)

    def omega_pe(self, x, y, z, mod: float) -> torch.Tensor:
        w = SQRT2_F32 * 2 * math.pi * self.source_frequency
        if self.kind == "drude-sphere":
            c = tuple(v * mod for v in self.sphere_center)
            zz = z if self.scheme == "3d" else torch.full_like(z, c[2])
            inside = (x - c[0]) ** 2 + (y - c[1]) ** 2 + (zz - c[2]) ** 2 < (self.sphere_radius * mod) ** 2
            return torch.where(inside, torch.full_like(x, w), torch.zeros_like(x))
        if self.kind != "reference":
            return torch.zeros_like(x)
        if self.scheme == "3d":
            inside = (x - 57 * mod) ** 2 + (y - 57 * mod) ** 2 + (z - 23 * mod) ** 2 < (8 * mod) ** 2
        else:
            inside = (x >= 437 * mod) & (x < 487 * mod) & (y >= 405 * mod) & (y < 505 * mod)
        return torch.where(inside, torch.full_like(x, w), torch.zeros_like(x))

    def omega_pm(self, x, y, z, mod: float) -> torch.Tensor:
        w = SQRT2_F32 * 2 * math.pi * self.source_frequency
        if self.kind != "reference":
            return torch.zeros_like(x)
        if self.scheme == "3d":
            inside = ((x >= 55 * mod) & (x < 60 * mod) & (y >= 55 * mod) & (y < 65 * mod)
                      & (z >= 15 * mod) & (z < 25 * mod))
        else:
            inside = (x >= 437 * mod) & (x < 487 * mod) & (y >= 405 * mod) & (y < 505 * mod)
        return torch.where(inside, torch.full_like(x, w), torch.zeros_like(x))

    def gamma_e(self, x, y, z, mod: float) -> torch.Tensor:
        return torch.zeros_like(x)

    def gamma_m(self, x, y, z, mod: float) -> torch.Tensor:
        return torch.zeros_like(x)


class MaterialSampler:
    """Evaluates a :class:`Scene` on the eps layout covering a local region and
    averages it onto field components."""

    def __init__(self, layout: YeeLayout, scene: Scene, origin: Sequence[int], shape: Sequence[int],
                 device, dtype=torch.float64):
        self.layout = layout
        self.scene = scene
        self.origin = tuple(origin)
        self.shape = tuple(shape)
        self.device = device
        self.dtype = dtype
        self.double = layout.double_material_precision
        self.mod = 2.0 if self.double else 1.0
        self._cache: Dict[str, torch.Tensor] = {}

    def _eps_region(self):
        if self.double:
            lo = tuple(2 * o for o in self.origin)
            shp = tuple(2 * s + 2 for s in self.shape)
        else:
            lo = self.origin
            shp = tuple(s + 1 for s in self.shape)
        # inactive axes: single plane
        shp = tuple(shp[d] if self.layout.active(d) else 1 for d in range(3))
        lo = tuple(lo[d] if self.layout.active(d) else 0 for d in range(3))
        return lo, shp

    def grid(self, name: str) -> torch.Tensor:
        if name not in self._cache:
            lo, shp = self._eps_region()
            x, y, z = self.scene._coords(lo, shp, self.mod, self.device, self.dtype)
            fn = {"eps": self.scene.eps, "mu": self.scene.mu, "omega_pe": self.scene.omega_pe,
                  "omega_pm": self.scene.omega_pm, "gamma_e": self.scene.gamma_e,
                  "gamma_m": self.scene.gamma_m}[name]
            self._cache[name] = fn(x, y, z, self.mod)
        return self._cache[name]

    def _points(self, comp: str, g: torch.Tensor):
        s = self.shape
        act = [self.layout.active(d) for d in range(3)]
        pts = []
        if not self.double:
            for off in MATERIAL_STENCIL[comp]:
                o = [off[d] if act[d] else 0 for d in range(3)]
                pts.append(g[o[0]:o[0] + s[0], o[1]:o[1] + s[1], o[2]:o[2] + s[2]])
        else:
            for base, sub in MATERIAL_STENCIL_DOUBLE[comp]:
                o = [(2 * base[d] + sub[d]) if act[d] else 0 for d in range(3)]
                st = [2 if act[d] else 1 for d in range(3)]
                pts.append(g[o[0]:o[0] + st[0] * s[0]:st[0], o[1]:o[1] + st[1] * s[1]:st[1],
                             o[2]:o[2] + st[2] * s[2]:st[2]])
        # drop duplicate points created by inactive axes (keeps 2D/1D averages exact)
        return _dedupe_points(comp, pts, act, self.double)

    def averaged(self, comp: str, name: str) -> torch.Tensor:
        """Material ``name`` averaged at the positions of component ``comp``
        over the local allocated region (shape == local field shape)."""
        return approximate_material(self._points(comp, self.grid(name)))

    def averaged_drude(self, comp: str, electric: bool):
        w = self._points(comp, self.grid("omega_pe" if electric else "omega_pm"))
        g = self._points(comp, self.grid("gamma_e" if electric else "gamma_m"))
        return approximate_drude(w, g)

    def uniform(self, name: str) -> Optional[float]:
        return self.scene.uniform(name)

    def free(self) -> None:
        """Drop the cached eps-layout grids (recomputed on demand, e.g. by a
        material dump): they are only needed while the coefficients are
        built."""
        self._cache.clear()


def _dedupe_points(comp, pts, act, double):
    if all(act):
        return pts
    # With inactive axes several stencil points coincide; the reference's 2D
    # schemes average only over in-plane points, which equals averaging the
    # deduplicated list (pairs collapse to identical values, so the pairwise mean
    # is unchanged).  Keep the list as is -- identical pairs average exactly.
    return pts


def sigma_profile_1d(n_eps: int, pml: int, dx: float, double: bool, lo: int = 0) -> np.ndarray:
    """Polynomially graded UPML conductivity on the eps layout along one axis
    (grading order m=6, reflection 1e-16, integrated per cell;
    Scheme3D.cpp:3659-3818).  ``n_eps`` is the eps-layout size of the *global*
    axis, ``lo`` the first eps index wanted; returns ``n`` values."""
    from ..utils.constants import EPS0, MU0
    mod = 2 if double else 1
    P = pml * mod
    out = np.zeros(n_eps, dtype=np.float64)
    if P == 0:
        return out
    boundary = P * dx
    m = 6
    r_err = 1e-16
    sigma_max = -math.log(r_err) * (m + 1.0) / (2.0 * math.sqrt(MU0 / EPS0) * boundary)
    factor = sigma_max / (dx * (boundary ** m) * (m + 1))
    size_fp = n_eps + 0.5 - 0.5  # getEpsCoordFP(totalSize) = totalSize + 0.5; compare uses pos+0.5
    for idx in range(n_eps):
        pos = idx + 0.5
        if pos < P:
            dist = int(P - pos)  # grid_coord truncation of a .5 value
            x1 = (dist + 1) * dx
            x2 = dist * dx
            out[idx] = factor * (x1 ** (m + 1) - x2 ** (m + 1))
        elif pos >= (n_eps + 0.5) - P:
            dist = int(pos - ((n_eps + 0.5) - P))
            x1 = (dist + 1) * dx
            x2 = dist * dx
            out[idx] = factor * (x1 ** (m + 1) - x2 ** (m + 1))
    return out
