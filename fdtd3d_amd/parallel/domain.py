"""Local sub-domain bookkeeping: owned box, ghost layers, local<->global maps
and per-step computation windows.

The reference stores each rank's chunk plus ghost layers of width
``bufferSize`` on the sides that have neighbours (``Source/Grid/ParallelGrid.h:26-206``)
and shrinks the computation window by ``shareStep + 1`` on those sides
(``ParallelGrid.cpp:2365-2489``).  Here a :class:`Domain` owns global cells
``[lo, hi)`` and allocates ``ghost_lo``/``ghost_hi`` extra layers.  Windows:

* ``buffer_size == 1`` (default): E and H are updated on the owned cells only;
  H low faces and E high faces are exchanged every half step (face-only,
  because the Yee curl is axis aligned).
* ``buffer_size == B > 1`` (deep halo, communication avoiding): after a full
  exchange of every state array (edges and corners included), step ``s`` of the
  ``B``-step window updates E on ``[lo-B+1+s, hi+B-s)`` and H on
  ``[lo-B+1+s, hi+B-1-s)`` along split axes (redundant ghost compute), so the
  next exchange is due after ``B`` steps -- the reference's scheme, with the
  windows derived for a staggered E/H pair.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

Box = Tuple[Tuple[int, int, int], Tuple[int, int, int]]


def box_intersect(a: Box, b: Box) -> Box:
    lo = tuple(max(a[0][d], b[0][d]) for d in range(3))
    hi = tuple(min(a[1][d], b[1][d]) for d in range(3))
    return lo, hi


def box_empty(b: Box) -> bool:
    return any(b[1][d] <= b[0][d] for d in range(3))


def box_volume(b: Box) -> int:
    if box_empty(b):
        return 0
    v = 1
    for d in range(3):
        v *= b[1][d] - b[0][d]
    return v


def box_subtract(a: Box, b: Box) -> List[Box]:
    """``a`` minus ``b`` as exactly 6 disjoint boxes (x-low, x-high, y-low,
    y-high, z-low, z-high slabs; some may be empty).  The fixed order lets
    callers launch the same slab of several staggered components together."""
    out: List[Box] = []
    lo, hi = list(a[0]), list(a[1])
    inter = box_intersect(a, b)
    if box_empty(inter):
        out.append((tuple(lo), tuple(hi)))
        empty = (tuple(lo), tuple(lo))
        return out + [empty] * 5
    for d in range(3):
        slo, shi = list(lo), list(hi)
        shi[d] = inter[0][d]
        out.append((tuple(slo), tuple(shi)))
        slo, shi = list(lo), list(hi)
        slo[d] = inter[1][d]
        out.append((tuple(slo), tuple(shi)))
        lo[d], hi[d] = inter[0][d], inter[1][d]
    return out


def box_shift(b: Box, off: Sequence[int]) -> Box:
    return (tuple(b[0][d] + off[d] for d in range(3)), tuple(b[1][d] + off[d] for d in range(3)))


@dataclass
class Domain:
    """One rank's piece of a global grid of ``global_size`` cells."""

    global_size: Tuple[int, int, int]
    lo: Tuple[int, int, int]
    hi: Tuple[int, int, int]
    ghost_lo: Tuple[int, int, int] = (0, 0, 0)
    ghost_hi: Tuple[int, int, int] = (0, 0, 0)
    # neighbour ranks (-1 if none) per axis: (low, high)
    neighbors: Tuple[Tuple[int, int], ...] = ((-1, -1), (-1, -1), (-1, -1))
    buffer_size: int = 1
    rank: int = 0
    coords: Tuple[int, int, int] = (0, 0, 0)
    topology: Tuple[int, int, int] = (1, 1, 1)
    # extra allocated cells past the high ghosts (alignment padding, never owned)
    pad_hi: Tuple[int, int, int] = (0, 0, 0)

    @classmethod
    def serial(cls, size: Sequence[int]) -> "Domain":
        size = tuple(int(v) for v in size)
        return cls(size, (0, 0, 0), size)

    # ------------------------------------------------------------------ shape
    @property
    def origin(self) -> Tuple[int, int, int]:
        """Global index of local index 0."""
        return tuple(self.lo[d] - self.ghost_lo[d] for d in range(3))

    @property
    def shape(self) -> Tuple[int, int, int]:
        return tuple(self.hi[d] - self.lo[d] + self.ghost_lo[d] + self.ghost_hi[d] + self.pad_hi[d]
                     for d in range(3))

    @property
    def owned_shape(self) -> Tuple[int, int, int]:
        return tuple(self.hi[d] - self.lo[d] for d in range(3))

    @property
    def is_serial(self) -> bool:
        return all(n == (-1, -1) for n in self.neighbors)

    def has_low(self, axis: int) -> bool:
        return self.neighbors[axis][0] >= 0

    def has_high(self, axis: int) -> bool:
        return self.neighbors[axis][1] >= 0

    def allocated_global(self) -> Box:
        o = self.origin
        return o, tuple(o[d] + self.shape[d] for d in range(3))

    def owned_global(self) -> Box:
        return self.lo, self.hi

    # ------------------------------------------------------------- mappings
    def to_local(self, b: Box) -> Box:
        o = self.origin
        return box_shift(b, tuple(-v for v in o))

    def to_global(self, b: Box) -> Box:
        return box_shift(b, self.origin)

    def local_index(self, gidx: Sequence[int]) -> Optional[Tuple[int, int, int]]:
        """Local index of a global cell, or None when not allocated here."""
        o = self.origin
        s = self.shape
        li = tuple(int(gidx[d]) - o[d] for d in range(3))
        if all(0 <= li[d] < s[d] for d in range(3)):
            return li
        return None

    def owns(self, gidx: Sequence[int]) -> bool:
        return all(self.lo[d] <= gidx[d] < self.hi[d] for d in range(3))

    # -------------------------------------------------------------- windows
    def window(self, kind: str, sub_step: int) -> Box:
        """Global box on which E (``kind='E'``) or H is computed at sub-step
        ``sub_step`` (0 .. buffer_size-1) of the current halo window."""
        B = self.buffer_size
        lo, hi = list(self.lo), list(self.hi)
        if B > 1:
            for d in range(3):
                if self.has_low(d):
                    lo[d] = self.lo[d] - B + 1 + sub_step
                if self.has_high(d):
                    hi[d] = self.hi[d] + B - sub_step - (1 if kind == "H" else 0)
        return tuple(lo), tuple(hi)

    def window_fused(self, kind: str, sub_step: int) -> Box:
        """Windows of the fused E+H kernel: the deep-halo windows for any
        ``buffer_size >= 1`` (E extends one layer further than H on the high
        side; ``B = 1`` needs a 1-deep full exchange every step)."""
        B = self.buffer_size
        lo, hi = list(self.lo), list(self.hi)
        for d in range(3):
            if self.has_low(d):
                lo[d] = self.lo[d] - B + 1 + sub_step
            if self.has_high(d):
                hi[d] = self.hi[d] + B - sub_step - (1 if kind == "H" else 0)
        return tuple(lo), tuple(hi)
