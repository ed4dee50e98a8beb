"""Time-levelled grids: the reference's ``Grid<TCoord>`` / ``FieldPointValue``
and ``ParallelGrid`` API on flat device tensors.

The reference keeps every grid point as a heap object with up to three time
levels and rotates them point by point in ``nextTimeStep``
(``Source/Kernels/FieldPoint.h:9-72``, ``Source/Grid/Grid.h:219-234``); the
distributed grid adds ghost layers, ``share()`` and ``gatherFullGrid()``
(``Source/Grid/ParallelGrid.h:207-423``).  Here a :class:`Grid` is a list of
contiguous tensors (one per level) over a :class:`~fdtd3d_amd.parallel.domain.Domain`
and a time step rotates tensor references (no copy).  The solver's hot path
uses bare tensors; these classes are the user-facing API for grids with
history (DAT dumps of ``current`` / ``previous`` / ``previous2`` levels,
custom schemes) and the subject of the reference's parallel-grid unit test
(``Tests/unit-test-parallel-grid.cpp``, mirrored by
``tests/test_grid_parallel_cpu.py``).
"""

from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..io.dat import write_dat
from ..io.naming import GridFileType, grid_file_name, levels as file_levels
from ..parallel.domain import Box, Domain

LEVEL_NAMES = (GridFileType.CURRENT, GridFileType.PREVIOUS, GridFileType.PREVIOUS2)


class Grid:
    """A field with ``time_levels`` (1..3) levels on one domain.

    Level 0 is the current value, 1 the previous, 2 the one before
    (reference ``ONE_TIME_STEP`` / ``TWO_TIME_STEPS`` builds keep 2 / 3)."""

    def __init__(self, domain: Domain, name: str = "grid", time_levels: int = 3, dtype=torch.float64,
                 device="cpu"):
        if not 1 <= time_levels <= 3:
            raise ValueError("time_levels must be 1, 2 or 3")
        self.domain = domain
        self.name = name
        self.levels: List[torch.Tensor] = [torch.zeros(domain.shape, dtype=dtype, device=device)
                                           for _ in range(time_levels)]
        self.time_step = 0

    # ---- reference accessors
    @property
    def size(self) -> Tuple[int, int, int]:
        """Local allocated size, ghosts included (``Grid::getSize``)."""
        return tuple(self.domain.shape)

    @property
    def current(self) -> torch.Tensor:
        return self.levels[0]

    @property
    def previous(self) -> torch.Tensor:
        return self.levels[1]

    @property
    def previous2(self) -> torch.Tensor:
        return self.levels[2]

    def next_time_step(self) -> None:
        """``Grid::nextTimeStep`` / ``FieldPointValue::shiftInTime``: the
        current values become the previous ones; the new current level starts
        as a copy of them (the reference copies value -> previous and keeps
        the value)."""
        if len(self.levels) > 1:
            oldest = self.levels.pop()
            oldest.copy_(self.levels[0])
            self.levels.insert(0, oldest)
        self.time_step += 1

    def computation_start(self, diff: Sequence[int] = (0, 0, 0)) -> Tuple[int, int, int]:
        """First local index of the computation range (``Grid::getComputationStart``)."""
        return tuple(self.domain.ghost_lo[d] + int(diff[d]) for d in range(3))

    def computation_end(self, diff: Sequence[int] = (0, 0, 0)) -> Tuple[int, int, int]:
        """One past the last local index (``Grid::getComputationEnd``)."""
        return tuple(self.domain.ghost_lo[d] + self.domain.owned_shape[d] - int(diff[d]) for d in range(3))

    def total_position(self, local: Sequence[int]) -> Tuple[int, int, int]:
        """Global index of a local index (``getTotalPosition``)."""
        o = self.domain.origin
        return tuple(int(local[d]) + o[d] for d in range(3))

    def relative_position(self, glob: Sequence[int]) -> Tuple[int, int, int]:
        """Local index of a global index (``getRelativePosition``)."""
        o = self.domain.origin
        return tuple(int(glob[d]) - o[d] for d in range(3))

    def has_value_for(self, glob: Sequence[int]) -> bool:
        return self.domain.local_index(glob) is not None

    def get(self, glob: Sequence[int], level: int = 0):
        li = self.domain.local_index(glob)
        if li is None:
            raise IndexError("global cell %s is not allocated on this rank" % (tuple(glob),))
        return self.levels[level][li]

    def set(self, glob: Sequence[int], value, level: int = 0) -> None:
        li = self.domain.local_index(glob)
        if li is None:
            raise IndexError("global cell %s is not allocated on this rank" % (tuple(glob),))
        self.levels[level][li] = value

    def owned(self, level: int = 0) -> torch.Tensor:
        gl, s = self.domain.ghost_lo, self.domain.owned_shape
        return self.levels[level][gl[0]:gl[0] + s[0], gl[1]:gl[1] + s[1], gl[2]:gl[2] + s[2]]

    # ---- output
    def save(self, directory: str, kind: GridFileType = GridFileType.ALL, rank: int = 0) -> List[str]:
        """DAT files of the requested levels, reference naming
        (``Commons.h:56-68``): ``current[<step>]_rank-<r>_<name>.dat`` ..."""
        os.makedirs(directory, exist_ok=True)
        out = []
        for lv in file_levels(kind):
            n = LEVEL_NAMES.index(lv)
            if n >= len(self.levels):
                continue
            path = grid_file_name(self.time_step, lv, rank, self.name, directory) + ".dat"
            write_dat(path, self.levels[n])
            out.append(path)
        return out


class ParallelGrid(Grid):
    """A :class:`Grid` on one rank's sub-domain with ghost exchange and
    full-grid gather (reference ``ParallelGrid``)."""

    def __init__(self, domain: Domain, halo, ops, name: str = "grid", time_levels: int = 3,
                 dtype=torch.float64, device="cpu"):
        super().__init__(domain, name, time_levels, dtype, device)
        self.halo = halo
        self.ops = ops
        self.share_step = 0

    # the exchanger's protocol: every state tensor of the "scheme"
    def state_tensors(self) -> List[torch.Tensor]:
        return list(self.levels)

    def share(self) -> None:
        """Exchange the ``buffer_size``-deep ghosts of every level with all
        neighbours, edges and corners included (``ParallelGrid::share``)."""
        self.halo.exchange_all(self)

    def next_time_step(self) -> None:
        """Rotate levels; share every ``buffer_size`` steps (the reference's
        deep-halo trigger, ``ParallelGrid.cpp:2161-2194``)."""
        super().next_time_step()
        self.share_step += 1
        if self.share_step >= self.domain.buffer_size:
            self.share()
            self.share_step = 0

    def gather_full_grid(self, level: int = 0, group=None) -> torch.Tensor:
        """The global array of one level on EVERY rank
        (``ParallelGrid::gatherFullGrid``): owned blocks are all-gathered
        once (padded to the largest block) instead of the reference's
        per-rank broadcast loop."""
        own = self.owned(level).contiguous()
        d = self.domain
        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return own.clone()
        from ..parallel.topology import ParallelGridCore
        world = dist.get_world_size(group)
        core = ParallelGridCore(tuple(d.global_size), world, tuple(d.topology))
        doms = [core.domain(r, d.buffer_size) for r in range(world)]
        n_max = max(int(torch.tensor(x.owned_shape).prod()) for x in doms)
        buf = torch.zeros(n_max, dtype=own.dtype, device=own.device)
        buf[:own.numel()] = own.flatten()
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
        full = torch.zeros(tuple(d.global_size), dtype=own.dtype, device=own.device)
        for r, x in enumerate(doms):
            if r >= core.used_procs:
                continue
            n = int(torch.tensor(x.owned_shape).prod())
            full[x.lo[0]:x.hi[0], x.lo[1]:x.hi[1], x.lo[2]:x.hi[2]] = parts[r][:n].view(x.owned_shape)
        return full
