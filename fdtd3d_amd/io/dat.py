"""DAT format: headerless raw binary of every value of a (local) grid in
linear index order, z fastest (reference ``DATDumper.h:32-159``,
``DATLoader.h:193-321``).

The element type is the field type: ``float``/``double`` (4/8 bytes), or the
reference's ``std::complex<T>`` layout (real, imag interleaved) for complex
runs.  A file therefore holds exactly ``prod(shape) * sizeof(T)`` bytes and is
byte-compatible with the reference for the same grid shape and value type.

Time levels: the solver keeps one level for E/H (leapfrog in place), so
``PREVIOUS`` files hold the same values as ``CURRENT`` at a step boundary --
what the reference's ``nextTimeStep`` copy leaves behind -- and
``PREVIOUS2`` is written from an explicitly supplied older level when one is
given (UPML/Drude auxiliaries).
"""

from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch

from .naming import GridFileType, grid_file_name, levels


def _to_numpy(t: torch.Tensor, imag: Optional[torch.Tensor] = None) -> np.ndarray:
    a = t.detach().cpu().contiguous().numpy()
    if imag is None:
        return a
    b = imag.detach().cpu().contiguous().numpy()
    out = np.empty(a.shape, dtype=np.complex64 if a.dtype == np.float32 else np.complex128)
    out.real = a
    out.imag = b
    return out


def write_dat(path: str, t: torch.Tensor, imag: Optional[torch.Tensor] = None) -> str:
    if not path.endswith(".dat"):
        path = path + ".dat"
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    _to_numpy(t, imag).tofile(path)
    return path


def read_dat(path: str, shape: Sequence[int], dtype: torch.dtype, complex_values: bool = False):
    """Returns a tensor (real) or a pair (real, imag)."""
    if not path.endswith(".dat"):
        path = path + ".dat"
    npd = {torch.float32: np.float32, torch.float64: np.float64}[dtype]
    if complex_values:
        npd = np.complex64 if npd == np.float32 else np.complex128
    n = int(np.prod(shape))
    a = np.fromfile(path, dtype=npd)
    if a.size != n:
        raise ValueError("%s holds %d values, expected %d for shape %s" % (path, a.size, n, tuple(shape)))
    a = a.reshape(tuple(shape))
    if complex_values:
        return torch.from_numpy(np.ascontiguousarray(a.real)), torch.from_numpy(np.ascontiguousarray(a.imag))
    return torch.from_numpy(a)


class DATDumper:
    """``DATDumper::init(step, type, rank, name)`` + ``dumpGrid``."""

    def __init__(self, step: int = 0, kind: GridFileType = GridFileType.CURRENT, rank: int = 0, name: str = "",
                 directory: str = "."):
        self.init(step, kind, rank, name, directory)

    def init(self, step, kind, rank, name, directory="."):
        self.step, self.kind, self.rank, self.name, self.directory = step, kind, rank, name, directory

    def dump_grid(self, t: torch.Tensor, imag: Optional[torch.Tensor] = None,
                  older: Optional[torch.Tensor] = None):
        out = []
        for lv in levels(self.kind):
            src = t
            if lv == GridFileType.PREVIOUS2 and older is not None:
                src = older
            out.append(write_dat(grid_file_name(self.step, lv, self.rank, self.name, self.directory), src, imag))
        return out


class DATLoader:
    def __init__(self, step: int = 0, kind: GridFileType = GridFileType.CURRENT, rank: int = 0, name: str = "",
                 directory: str = "."):
        self.step, self.kind, self.rank, self.name, self.directory = step, kind, rank, name, directory

    def load_grid(self, shape, dtype, complex_values=False, level: GridFileType = GridFileType.CURRENT):
        return read_dat(grid_file_name(self.step, level, self.rank, self.name, self.directory), shape, dtype,
                        complex_values)
