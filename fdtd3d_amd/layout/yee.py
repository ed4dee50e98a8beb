"""Yee staggered-grid layout.

Re-implements the behaviour of the reference ``YeeGridLayout``
(``Source/Layout/YeeGridLayout.h:23-511``, ``YeeGridLayout.cpp:3-845``) as data
rather than virtual methods, so that every consumer -- the torch reference ops,
the host-side table builders for the HIP kernels and the decomposition code --
reads the same tables:

* real (FP) position of index ``(i, j, k)`` of every component
  (``minExCoordFP = (1, .5, .5)`` ... ``YeeGridLayout.h:414-421``);
* computation start/end diffs (``YeeGridLayout.h:131-182``): a component is
  updated on ``[start, size - end)`` of the global grid;
* circuit neighbours, expressed as curl *terms* ``(source, axis, sign)``:
  an E component adds ``sign * (src[idx] - src[idx - e_axis])`` and an H
  component adds ``sign * (src[idx + e_axis] - src[idx])``
  (``YeeGridLayout.cpp:3-253`` + ``Kernels.h:13-29``);
* material-averaging stencils on the eps layout (2/4-point, or 8-point on the
  doubled grid with ``--use-double-material-precision``;
  ``YeeGridLayout.h:1007-1263``);
* PML and TF/SF region predicates (``YeeGridLayout.cpp:255-809``) and incident
  wave projections (``YeeGridLayout.cpp:811-845``).

1D and 2D schemes reuse the 3D tables with inactive axes dropped: TMz keeps
``Ez, Hx, Hy``, TEz keeps ``Ex, Ey, Hz`` (exactly the reference's 2D schemes)
and the 1D scheme keeps ``Ez, Hy`` along x (new; the reference has no 1D
scheme).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

from ..utils.coordinates import GridCoordinate, GridCoordinateFP3D

E_COMPONENTS = ("Ex", "Ey", "Ez")
H_COMPONENTS = ("Hx", "Hy", "Hz")
ALL_COMPONENTS = E_COMPONENTS + H_COMPONENTS

# real position of index 0 (YeeGridLayout.h:414-421)
MIN_COORD_FP: Dict[str, Tuple[float, float, float]] = {
    "Ex": (1.0, 0.5, 0.5),
    "Ey": (0.5, 1.0, 0.5),
    "Ez": (0.5, 0.5, 1.0),
    "Hx": (0.5, 1.0, 1.0),
    "Hy": (1.0, 0.5, 1.0),
    "Hz": (1.0, 1.0, 0.5),
    "Eps": (0.5, 0.5, 0.5),
}

# computation start / end diffs (YeeGridLayout.h:131-182)
START_DIFF: Dict[str, Tuple[int, int, int]] = {
    "Ex": (0, 1, 1), "Ey": (1, 0, 1), "Ez": (1, 1, 0),
    "Hx": (1, 0, 0), "Hy": (0, 1, 0), "Hz": (0, 0, 1),
}
END_DIFF: Dict[str, Tuple[int, int, int]] = {
    "Ex": (1, 0, 0), "Ey": (0, 1, 0), "Ez": (0, 0, 1),
    "Hx": (0, 1, 1), "Hy": (1, 0, 1), "Hz": (1, 1, 0),
}

# curl terms (source component, axis, sign)
CURL_TERMS: Dict[str, Tuple[Tuple[str, int, int], ...]] = {
    "Ex": (("Hz", 1, +1), ("Hy", 2, -1)),
    "Ey": (("Hx", 2, +1), ("Hz", 0, -1)),
    "Ez": (("Hy", 0, +1), ("Hx", 1, -1)),
    "Hx": (("Ey", 2, +1), ("Ez", 1, -1)),
    "Hy": (("Ez", 0, +1), ("Ex", 2, -1)),
    "Hz": (("Ex", 1, +1), ("Ey", 0, -1)),
}

# UPML axes per component (Scheme3D.cpp:266-416 and siblings): the D/B update
# uses sigma of AXIS_D, E-from-D uses Ca(sigma of AXIS_CA) and Cb/Cc(sigma of AXIS_CB).
UPML_AXES: Dict[str, Tuple[int, int, int]] = {
    "Ex": (1, 2, 0), "Ey": (2, 0, 1), "Ez": (0, 1, 2),
    "Hx": (1, 2, 0), "Hy": (2, 0, 1), "Hz": (0, 1, 2),
}

# Material averaging stencils: offsets (on the eps layout) of the points averaged
# for each component, in the reference's pairwise order.
MATERIAL_STENCIL: Dict[str, Tuple[Tuple[int, int, int], ...]] = {
    "Ex": ((0, 0, 0), (1, 0, 0)),
    "Ey": ((0, 0, 0), (0, 1, 0)),
    "Ez": ((0, 0, 0), (0, 0, 1)),
    "Hx": ((0, 0, 0), (0, 0, 1), (0, 1, 0), (0, 1, 1)),
    "Hy": ((0, 0, 0), (0, 0, 1), (1, 0, 0), (1, 0, 1)),
    "Hz": ((0, 0, 0), (0, 1, 0), (1, 0, 0), (1, 1, 0)),
}

# 8-point stencils on the doubled material grid: (base eps offset, sub offset),
# point = 2 * (idx + base) + sub  (YeeGridLayout.h:1030-1200).
MATERIAL_STENCIL_DOUBLE: Dict[str, Tuple[Tuple[Tuple[int, int, int], Tuple[int, int, int]], ...]] = {
    "Ex": (((0, 0, 0), (1, 0, 0)), ((0, 0, 0), (1, 1, 0)), ((1, 0, 0), (0, 0, 0)), ((1, 0, 0), (0, 1, 0)),
           ((0, 0, 0), (1, 0, 1)), ((0, 0, 0), (1, 1, 1)), ((1, 0, 0), (0, 0, 1)), ((1, 0, 0), (0, 1, 1))),
    "Ey": (((0, 0, 0), (0, 1, 0)), ((0, 0, 0), (1, 1, 0)), ((0, 1, 0), (0, 0, 0)), ((0, 1, 0), (1, 0, 0)),
           ((0, 0, 0), (0, 1, 1)), ((0, 0, 0), (1, 1, 1)), ((0, 1, 0), (0, 0, 1)), ((0, 1, 0), (1, 0, 1))),
    "Ez": (((0, 0, 0), (0, 0, 1)), ((0, 0, 0), (0, 1, 1)), ((0, 0, 0), (1, 0, 1)), ((0, 0, 0), (1, 1, 1)),
           ((0, 0, 1), (0, 0, 0)), ((0, 0, 1), (0, 1, 0)), ((0, 0, 1), (1, 0, 0)), ((0, 0, 1), (1, 1, 0))),
    "Hx": (((0, 0, 0), (0, 1, 1)), ((0, 0, 0), (1, 1, 1)), ((0, 0, 1), (0, 1, 0)), ((0, 0, 1), (1, 1, 0)),
           ((0, 1, 0), (0, 0, 1)), ((0, 1, 0), (1, 0, 1)), ((0, 1, 1), (0, 0, 0)), ((0, 1, 1), (1, 0, 0))),
    "Hy": (((0, 0, 0), (1, 0, 1)), ((0, 0, 0), (1, 1, 1)), ((0, 0, 1), (1, 0, 0)), ((0, 0, 1), (1, 1, 0)),
           ((1, 0, 0), (0, 0, 1)), ((1, 0, 0), (0, 1, 1)), ((1, 0, 1), (0, 0, 0)), ((1, 0, 1), (0, 1, 0))),
    "Hz": (((0, 0, 0), (1, 1, 0)), ((0, 0, 0), (1, 1, 1)), ((0, 1, 0), (1, 0, 0)), ((0, 1, 0), (1, 0, 1)),
           ((1, 0, 0), (0, 1, 0)), ((1, 0, 0), (0, 1, 1)), ((1, 1, 0), (0, 0, 0)), ((1, 1, 0), (0, 0, 1))),
}

SCHEME_COMPONENTS: Dict[str, Tuple[str, ...]] = {
    "3d": ALL_COMPONENTS,
    "tmz": ("Ez", "Hx", "Hy"),
    "tez": ("Ex", "Ey", "Hz"),
    "1d": ("Ez", "Hy"),
}

SCHEME_AXES: Dict[str, Tuple[int, ...]] = {
    "3d": (0, 1, 2),
    "tmz": (0, 1),
    "tez": (0, 1),
    "1d": (0,),
}


def is_e(comp: str) -> bool:
    return comp[0] in "ED"


@dataclass
class YeeLayout:
    """Layout of one scheme on a global grid of ``size`` cells (always 3 numbers;
    inactive axes have size 1)."""

    size: Tuple[int, int, int]
    scheme: str = "3d"
    pml_size: Tuple[int, int, int] = (0, 0, 0)
    tfsf_size: Tuple[int, int, int] = (0, 0, 0)
    theta: float = math.pi / 2
    phi: float = 0.0
    psi: float = math.pi / 2
    double_material_precision: bool = False

    def __post_init__(self):
        self.size = tuple(int(v) for v in self.size)
        self.components = SCHEME_COMPONENTS[self.scheme]
        self.axes = SCHEME_AXES[self.scheme]
        # reference YeeGridLayout.h:446-447
        if not (0 <= self.theta <= math.pi / 2 + 1e-12 and 0 <= self.phi <= math.pi / 2 + 1e-12):
            raise ValueError("incident angles theta/phi must lie in [0, pi/2]")

    # ---------------------------------------------------------------- geometry
    def active(self, axis: int) -> bool:
        return axis in self.axes

    def start_diff(self, comp: str) -> Tuple[int, int, int]:
        return tuple(START_DIFF[comp][a] if self.active(a) else 0 for a in range(3))

    def end_diff(self, comp: str) -> Tuple[int, int, int]:
        return tuple(END_DIFF[comp][a] if self.active(a) else 0 for a in range(3))

    def global_range(self, comp: str) -> Tuple[Tuple[int, int, int], Tuple[int, int, int]]:
        """``[lo, hi)`` in global indices on which ``comp`` is updated."""
        s = self.start_diff(comp)
        e = self.end_diff(comp)
        return s, tuple(self.size[a] - e[a] for a in range(3))

    def curl_terms(self, comp: str) -> Tuple[Tuple[str, int, int], ...]:
        return tuple(t for t in CURL_TERMS[comp] if t[0] in self.components and self.active(t[1]))

    def min_coord_fp(self, comp: str) -> Tuple[float, float, float]:
        return MIN_COORD_FP[comp]

    def coord_fp(self, comp: str, idx: Sequence[int]) -> GridCoordinate:
        """Real (staggered) coordinate of cell ``idx`` of ``comp``: the
        reference's ``getTotalPosition`` + ``getMinCoordFP``
        (``YeeGridLayout.h:407-424``) as a 3D FP coordinate."""
        return GridCoordinateFP3D(*idx) + GridCoordinateFP3D(*MIN_COORD_FP[comp])

    # ---------------------------------------------------------------- PML
    def pml_borders(self):
        left = self.pml_size
        right = tuple(self.size[a] - self.pml_size[a] for a in range(3))
        return left, right

    def is_in_pml(self, real) -> bool:
        """``YeeGridLayout::isInPML`` (YeeGridLayout.cpp:255-279); ``real`` is
        a :class:`GridCoordinate` or a sequence of 3 reals."""
        if isinstance(real, GridCoordinate):
            real = real.as_tuple()
        left, right = self.pml_borders()
        for a in self.axes:
            if left[a] != right[a] and (real[a] < left[a] or real[a] >= right[a]):
                return True
        return False

    # ---------------------------------------------------------------- TF/SF
    def tfsf_borders(self):
        left = self.tfsf_size
        right = tuple(self.size[a] - self.tfsf_size[a] for a in range(3))
        return left, right

    def zero_inc_coord_fp(self) -> Tuple[float, float, float]:
        """Origin of the incident 1D line (YeeGridLayout.h:436-440)."""
        left, _ = self.tfsf_borders()
        st, ct = math.sin(self.theta), math.cos(self.theta)
        sp, cp = math.sin(self.phi), math.cos(self.phi)
        if self.scheme == "3d":
            return (left[0] - 2.5 * st * cp, left[1] - 2.5 * st * sp, left[2] - 2.5 * ct)
        # 2D schemes: propagation in the xy plane (theta = pi/2)
        return (left[0] - 2.5 * cp, left[1] - 2.5 * sp, 0.0)

    def incident_direction(self) -> Tuple[float, float, float]:
        if self.scheme == "3d":
            return (math.sin(self.theta) * math.cos(self.phi),
                    math.sin(self.theta) * math.sin(self.phi),
                    math.cos(self.theta))
        return (math.cos(self.phi), math.sin(self.phi), 0.0)

    def incident_projection(self, comp: str) -> float:
        """Multiplier turning the scalar incident E (H) into ``comp``
        (YeeGridLayout.cpp:811-845)."""
        t, p, s = self.theta, self.phi, self.psi
        if self.scheme in ("tmz", "tez", "1d"):
            t = math.pi / 2
        v = {
            "Ex": math.cos(s) * math.sin(p) - math.sin(s) * math.cos(t) * math.cos(p),
            "Ey": -math.cos(s) * math.cos(p) - math.sin(s) * math.cos(t) * math.sin(p),
            "Ez": math.sin(s) * math.sin(t),
            "Hx": math.sin(s) * math.sin(p) + math.cos(s) * math.cos(t) * math.cos(p),
            "Hy": -math.sin(s) * math.cos(p) + math.cos(s) * math.cos(t) * math.sin(p),
            "Hz": -(math.cos(s) * math.sin(t)),
        }[comp]
        # cos(pi/2) = 6e-17 in floating point: a projection that is zero in
        # exact arithmetic (the reference default theta = 90, phi = 0, psi =
        # 90 excites only Ez / Hy) is zero here too, so its corrections --
        # 1e-17 of the incident wave, below fp64 round-off -- are not applied
        return 0.0 if abs(v) < 1e-12 else v


def component_shape(size: Sequence[int]) -> Tuple[int, int, int]:
    return tuple(int(v) for v in size)
