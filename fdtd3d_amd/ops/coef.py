"""Factorised update coefficients.

Every coefficient in the Yee/UPML/Drude updates is a product of

    scalar * px[i] * py[j] * pz[k] * cell[i, j, k]

with each factor optional: vacuum runs need only the scalar, UPML conductivity
profiles are 1D along one axis (the reference's sigma grids vary along a single
axis, ``Scheme3D.cpp:3659-3818``), and only inhomogeneous media need a per-cell
array.  The same object drives the torch reference ops (broadcast multiply) and
the HIP kernels (pointer arguments, ``nullptr`` = factor absent), so both
backends evaluate identical coefficient values.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Tuple

import torch


@dataclass
class Coef:
    scalar: float = 1.0
    px: Optional[torch.Tensor] = None
    py: Optional[torch.Tensor] = None
    pz: Optional[torch.Tensor] = None
    cell: Optional[torch.Tensor] = None

    @property
    def is_scalar(self) -> bool:
        return self.px is None and self.py is None and self.pz is None and self.cell is None

    def to(self, device=None, dtype=None) -> "Coef":
        f = lambda t: None if t is None else t.to(device=device, dtype=dtype).contiguous()
        return Coef(self.scalar, f(self.px), f(self.py), f(self.pz), f(self.cell))

    def materialize(self, sl: Tuple[slice, slice, slice]):
        """Value over a local box given as slices (torch broadcastable)."""
        v = self.scalar
        if self.px is not None:
            v = v * self.px[sl[0]].view(-1, 1, 1)
        if self.py is not None:
            v = v * self.py[sl[1]].view(1, -1, 1)
        if self.pz is not None:
            v = v * self.pz[sl[2]].view(1, 1, -1)
        if self.cell is not None:
            v = v * self.cell[sl]
        return v

    def at(self, i: int, j: int, k: int) -> float:
        v = float(self.scalar)
        if self.px is not None:
            v *= float(self.px[i])
        if self.py is not None:
            v *= float(self.py[j])
        if self.pz is not None:
            v *= float(self.pz[k])
        if self.cell is not None:
            v *= float(self.cell[i, j, k])
        return v

    def at_many(self, idx: torch.Tensor) -> torch.Tensor:
        """Values at an (n, 3) tensor of local indices (float64)."""
        v = torch.full((idx.shape[0],), float(self.scalar), dtype=torch.float64, device=idx.device)
        if self.px is not None:
            v = v * self.px.to(torch.float64)[idx[:, 0]]
        if self.py is not None:
            v = v * self.py.to(torch.float64)[idx[:, 1]]
        if self.pz is not None:
            v = v * self.pz.to(torch.float64)[idx[:, 2]]
        if self.cell is not None:
            v = v * self.cell.to(torch.float64)[idx[:, 0], idx[:, 1], idx[:, 2]]
        return v
