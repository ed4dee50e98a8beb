"""Virtual process topology: rank grid, neighbours, chunk sizes, halo
directions and the topology optimiser.

Equivalent of the reference's ``ParallelGridCore`` + ``ParallelBuffer{2D,3D}`` +
``ParallelYeeGridLayout`` (``Source/Grid/ParallelGridCore.cpp``,
``ParallelBuffer3D.cpp:272-395``, ``Source/Layout/ParallelYeeGridLayout.cpp:9-68``):

* rank ``r`` sits at ``(px, py, pz)`` with ``r = px + py*Nx + pz*Nx*Ny``
  (``ParallelGridCore.cpp:707-797``);
* every axis is block-distributed: ``core = N / P`` cells per rank and the last
  rank on the axis takes the remainder (``ParallelYeeGridLayout.cpp:9-68``);
* the split shape is chosen at run time (``--topology x|y|z|xy|yz|xz|xyz``)
  instead of at build time (``CMakeLists.txt:114-191``);
* the optimiser enumerates *all* factorisations ``Nx*Ny*Nz = P`` over the allowed
  axes and minimises the per-rank halo surface (the reference's cost idea,
  ``ParallelBuffer3D.cpp:365-369``, without its divisibility restrictions);
  ``--topology-size{x,y,z}`` (parsed but ignored by the reference) are honoured,
  as is ``--available-topologies FILE``.
* the 26 halo directions of the reference (``BufferPosition.inc.h:8-61``) are
  enumerated by :func:`buffer_directions` for deep-halo bookkeeping and tests.
"""

from __future__ import annotations

import itertools
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from .domain import Domain

AXIS_NAMES = "xyz"


def parse_topology_axes(spec: str) -> Tuple[int, ...]:
    spec = spec.lower()
    out = tuple(sorted({AXIS_NAMES.index(c) for c in spec}))
    if not out or any(c not in AXIS_NAMES for c in spec):
        raise ValueError("bad --topology %r" % spec)
    return out


def chunk_bounds(n: int, p: int, coord: int) -> Tuple[int, int]:
    """Owned ``[lo, hi)`` of rank ``coord`` among ``p`` along an axis of ``n``
    cells: ``n // p`` each, remainder to the last rank."""
    core = n // p
    lo = coord * core
    hi = n if coord == p - 1 else lo + core
    return lo, hi


def halo_cost(size: Sequence[int], topo: Sequence[int]) -> float:
    """Halo cells of the busiest rank: along a split axis an interior rank has
    two face neighbours (one when the axis has just 2 ranks)."""
    chunk = [size[a] / topo[a] for a in range(3)]
    cost = 0.0
    for a in range(3):
        if topo[a] > 1:
            other = 1.0
            for b in range(3):
                if b != a:
                    other *= chunk[b]
            cost += (2 if topo[a] > 2 else 1) * other
    return cost


def _factorizations(p: int, axes: Sequence[int]) -> List[Tuple[int, int, int]]:
    out = []
    for px in range(1, p + 1):
        if p % px:
            continue
        for py in range(1, p // px + 1):
            if (p // px) % py:
                continue
            pz = p // (px * py)
            t = (px, py, pz)
            if all(t[a] == 1 for a in range(3) if a not in axes):
                out.append(t)
    return out


def optimal_topology(size: Sequence[int], nprocs: int, axes: Sequence[int] = (0, 1, 2),
                     available: Optional[Sequence[Tuple[int, int, int]]] = None) -> Tuple[int, int, int]:
    """Rank grid minimising halo traffic; ties prefer even division, then
    fewer split axes, then splitting the slowest-varying (x) axis."""
    cands = _factorizations(nprocs, axes)
    if available:
        avail = {tuple(a) for a in available}
        cands = [c for c in cands if c in avail] or cands
    cands = [c for c in cands if all(size[a] >= c[a] for a in range(3))] or cands

    def key(t):
        uneven = sum(size[a] % t[a] for a in range(3))
        nsplit = sum(1 for a in range(3) if t[a] > 1)
        return (halo_cost(size, t), uneven, nsplit, -t[0], -t[1])

    return min(cands, key=key)


def read_available_topologies(path: str) -> List[Tuple[int, int, int]]:
    out = []
    with open(path) as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 3:
                out.append((int(parts[0]), int(parts[1]), int(parts[2])))
    return out


def rank_coords(rank: int, topo: Sequence[int]) -> Tuple[int, int, int]:
    nx, ny, _ = topo
    return rank % nx, (rank // nx) % ny, rank // (nx * ny)


def coords_rank(c: Sequence[int], topo: Sequence[int]) -> int:
    return c[0] + c[1] * topo[0] + c[2] * topo[0] * topo[1]


@dataclass
class ParallelGridCore:
    """Rank grid of one job."""

    size: Tuple[int, int, int]
    nprocs: int
    topology: Tuple[int, int, int]

    @classmethod
    def create(cls, size: Sequence[int], nprocs: int, axes_spec: str = "xyz",
               requested: Optional[Sequence[int]] = None, optimal: bool = True,
               available: Optional[Sequence[Tuple[int, int, int]]] = None,
               active_axes: Sequence[int] = (0, 1, 2)) -> "ParallelGridCore":
        size = tuple(int(v) for v in size)
        axes = tuple(a for a in parse_topology_axes(axes_spec) if a in active_axes) or (active_axes[0],)
        topo = None
        if requested is not None and not optimal:
            r = tuple(int(v) for v in requested)
            if r[0] * r[1] * r[2] == nprocs:
                topo = r
        if topo is None:
            topo = optimal_topology(size, nprocs, axes, available)
        for a in range(3):
            if topo[a] > size[a]:
                raise ValueError("topology %s does not fit grid %s" % (topo, size))
        return cls(size, nprocs, topo)

    @property
    def used_procs(self) -> int:
        return self.topology[0] * self.topology[1] * self.topology[2]

    def domain(self, rank: int, buffer_size: int = 1, align_z: int = 1, align_axis: int = 2) -> Domain:
        """Sub-domain of ``rank``.  ``align_z`` > 1 pads the local allocation at
        the high end of ``align_axis`` (z; y for the 2D schemes, whose rows run
        along y) so that its extent is a multiple of ``align_z`` (the float4
        kernels need it % 4 == 0); padding cells are never owned, exchanged or
        stored."""
        topo = self.topology
        c = rank_coords(rank, topo)
        lo, hi, nbr = [], [], []
        for a in range(3):
            l, h = chunk_bounds(self.size[a], topo[a], c[a])
            lo.append(l)
            hi.append(h)
            lo_n = coords_rank(tuple(c[b] - (1 if b == a else 0) for b in range(3)), topo) if c[a] > 0 else -1
            hi_n = coords_rank(tuple(c[b] + (1 if b == a else 0) for b in range(3)), topo) if c[a] < topo[a] - 1 else -1
            nbr.append((lo_n, hi_n))
        B = int(buffer_size)
        for a in range(3):
            if topo[a] > 1:
                core = self.size[a] // topo[a]
                if B > core:
                    raise ValueError("--buffer-size %d exceeds the chunk size %d along %s" % (B, core, AXIS_NAMES[a]))
        gl = tuple(B if nbr[a][0] >= 0 else 0 for a in range(3))
        gh = tuple(B if nbr[a][1] >= 0 else 0 for a in range(3))
        d = Domain(self.size, tuple(lo), tuple(hi), gl, gh, tuple(nbr), B, rank, c, topo)
        if align_z > 1:
            n = d.shape[align_axis]
            d.pad_hi = tuple((-n) % align_z if a == align_axis else 0 for a in range(3))
        return d


# 26 halo directions (faces, edges, corners) in the reference's naming
_DIR_LETTERS = {(-1, 0): "L", (1, 0): "R", (-1, 1): "D", (1, 1): "U", (-1, 2): "B", (1, 2): "F"}


def buffer_directions(axes: Sequence[int] = (0, 1, 2)) -> Dict[str, Tuple[int, int, int]]:
    """Name -> offset for every non-zero neighbour offset over ``axes``
    (e.g. ``'L'``, ``'LD'``, ``'LDB'``)."""
    out = {}
    rng = [(-1, 0, 1) if a in axes else (0,) for a in range(3)]
    for off in itertools.product(*rng):
        if off == (0, 0, 0):
            continue
        name = "".join(_DIR_LETTERS[(off[a], a)] for a in range(3) if off[a] != 0)
        out[name] = off
    return out


def opposite(direction: str) -> str:
    swap = {"L": "R", "R": "L", "D": "U", "U": "D", "B": "F", "F": "B"}
    return "".join(swap[c] for c in direction)
