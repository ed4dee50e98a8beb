"""TXT format: one ``i [j [k]] value`` line per point (real part), a blank line
after every x plane (reference ``TXTDumper.cpp:8-337``), and a loader for it.
"""

from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch

from .naming import GridFileType, grid_file_name, levels


def write_txt(path: str, t: torch.Tensor, dim: int = 3) -> str:
    if not path.endswith(".txt"):
        path = path + ".txt"
    a = t.detach().cpu().double().numpy()
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        if dim == 1:
            a1 = a.reshape(-1)
            for i in range(a1.shape[0]):
                f.write("%d %.17g\n" % (i, a1[i]))
            return path
        a3 = a.reshape(a.shape[0], a.shape[1], -1)
        nz = a3.shape[2] if dim == 3 else 1
        for i in range(a3.shape[0]):
            jj, kk = np.meshgrid(np.arange(a3.shape[1]), np.arange(nz), indexing="ij")
            vals = a3[i, :, :nz]
            if dim == 3:
                rows = np.stack([np.full(jj.size, i), jj.ravel(), kk.ravel()], axis=1)
                lines = ["%d %d %d %.17g" % (r[0], r[1], r[2], v) for r, v in zip(rows, vals.ravel())]
            else:
                lines = ["%d %d %.17g" % (i, j, v) for j, v in zip(range(a3.shape[1]), vals[:, 0])]
            f.write("\n".join(lines))
            f.write("\n\n")
    return path


def read_txt(path: str, shape: Sequence[int]) -> torch.Tensor:
    if not path.endswith(".txt"):
        path = path + ".txt"
    out = np.zeros(tuple(shape))
    flat = out.reshape(shape[0], -1) if len(shape) > 1 else out.reshape(-1, 1)
    with open(path) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            idx = tuple(int(v) for v in p[:-1])
            full = idx + (0,) * (len(shape) - len(idx))
            out[full] = float(p[-1])
    return torch.from_numpy(out)


class TXTDumper:
    def __init__(self, step=0, kind=GridFileType.CURRENT, rank=0, name="", directory="."):
        self.step, self.kind, self.rank, self.name, self.directory = step, kind, rank, name, directory

    def init(self, step, kind, rank, name):
        self.step, self.kind, self.rank, self.name = step, kind, rank, name

    def dump_grid(self, t: torch.Tensor, dim: Optional[int] = None):
        dim = dim if dim is not None else (sum(1 for s in t.shape if s > 1) or 1)
        return [write_txt(grid_file_name(self.step, lv, self.rank, self.name, self.directory), t, dim)
                for lv in levels(self.kind)]
