"""Region-local storage of the UPML / Drude auxiliary fields.

The reference allocates every auxiliary grid (D, B, D1, B1 at three time
levels) over the whole domain (``Scheme3D.cpp:3413-4032``), although D / B
carry information only inside the absorbing slabs and D1 / B1 only inside the
dispersive material: elsewhere the UPML / Drude chain collapses to the plain
Yee update (sigma = 0, omega = 0) and the scheme runs the plain kernels there
(models/scheme.py ``_init_chain_regions``).  A :class:`RegionLevel` holds one
time level of one component's auxiliary field over exactly the static chain
boxes of that component -- the six PML slabs and the dispersive box -- so a
1024^3 Drude + UPML run keeps ~6% (slabs) and ~1/8 (sphere box) of the
full-grid arrays.

Kernels address a part through its storage box (``csrc/chain_kernels.hip``
``ChainComp::dbox``); the torch oracle slices it the same way.
"""

from __future__ import annotations

from typing import List, Tuple

import torch

from ..parallel.domain import box_empty, box_volume

Box = Tuple[Tuple[int, int, int], Tuple[int, int, int]]


class RegionLevel:
    """One auxiliary time level stored over a few disjoint local boxes."""

    def __init__(self, boxes: List[Box], dtype, device):
        self.boxes = [b for b in boxes if not box_empty(b)]
        self.data = [torch.zeros(tuple(b[1][d] - b[0][d] for d in range(3)), dtype=dtype, device=device)
                     for b in self.boxes]

    def part(self, box: Box):
        """(tensor, storage box) of the part holding the local ``box``
        (an empty box: (None, empty box))."""
        if box_empty(box):
            return None, ((0, 0, 0), (0, 0, 0))
        for t, b in zip(self.data, self.boxes):
            if all(b[0][d] <= box[0][d] and box[1][d] <= b[1][d] for d in range(3)):
                return t, b
        raise ValueError("box %s is not inside one storage region of %s" % (box, self.boxes))

    def view(self, box: Box) -> torch.Tensor:
        """The values of the local ``box`` (a view into its part)."""
        t, b = self.part(box)
        return t[tuple(slice(box[0][d] - b[0][d], box[1][d] - b[0][d]) for d in range(3))]

    def cells(self) -> int:
        return sum(box_volume(b) for b in self.boxes)
