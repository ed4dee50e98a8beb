"""Synthetic field data and field checksums for benchmarks and self-checks.

``hash_fill`` gives every *global* cell of a component a pseudo-random value
in [-1, 1) from an integer hash of its global linear index, so a decomposed
run starts from exactly the same fields as a serial one whatever the
topology (each rank fills its own allocation, ghosts included).  ``energy``
is the fp64 sum of squares of a box, reduced plane-chunk by plane-chunk so a
1024^3 fp32 field never needs a full fp64 copy.

The reference starts every run from zero fields (``Scheme3D.cpp:3830-4032``);
random initial fields are the benchmark convention of BASELINE.json
("synthetic vacuum/dielectric grids with random-init fields").
"""

from __future__ import annotations

from typing import Sequence, Tuple

import torch

_M1 = -7046029254386353131   # 0x9E3779B97F4A7C15 as a signed int64
_M2 = -4658895280553007687   # 0xBF58476D1CE4E5B9
_M3 = -7723592293110705685   # 0x94D049BB133111EB
_MASK24 = (1 << 24) - 1

# x planes per chunk of the fill / reduction (bounds the int64 / fp64 temporaries)
_CHUNK_CELLS = 1 << 24


def _mix(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 finaliser on int64 (wrapping multiply; arithmetic shifts are
    masked to logical ones)."""
    x = x * _M1
    x = x ^ ((x >> 30) & ((1 << 34) - 1))
    x = x * _M2
    x = x ^ ((x >> 27) & ((1 << 37) - 1))
    x = x * _M3
    x = x ^ ((x >> 31) & ((1 << 33) - 1))
    return x


def hash_fill(t: torch.Tensor, origin: Sequence[int], global_size: Sequence[int], seed: int) -> None:
    """Fill local array ``t`` (local index 0 = global cell ``origin``) with
    the hash values of the global cells; cells outside the global grid
    (alignment padding) get 0."""
    nx, ny, nz = t.shape
    G = tuple(int(v) for v in global_size)
    dev = t.device
    jj = torch.arange(ny, device=dev, dtype=torch.int64) + int(origin[1])
    kk = torch.arange(nz, device=dev, dtype=torch.int64) + int(origin[2])
    okj = (jj >= 0) & (jj < G[1])
    okk = (kk >= 0) & (kk < G[2])
    step = max(1, _CHUNK_CELLS // max(1, ny * nz))
    salt = int(seed) * 0x632BE5AB + 0x1234567
    for i0 in range(0, nx, step):
        i1 = min(nx, i0 + step)
        ii = torch.arange(i0, i1, device=dev, dtype=torch.int64) + int(origin[0])
        lin = (ii.view(-1, 1, 1) * G[1] + jj.view(1, -1, 1)) * G[2] + kk.view(1, 1, -1)
        h = _mix(lin + salt)
        u = ((h >> 20) & _MASK24).to(torch.float64) * (2.0 / (1 << 24)) - 1.0
        ok = ((ii >= 0) & (ii < G[0])).view(-1, 1, 1) & okj.view(1, -1, 1) & okk.view(1, 1, -1)
        t[i0:i1] = torch.where(ok, u, torch.zeros_like(u)).to(t.dtype)


def energy(t: torch.Tensor, box: Tuple[Tuple[int, int, int], Tuple[int, int, int]]) -> float:
    """Sum of squares of ``t`` over a local box, accumulated in fp64."""
    lo, hi = box
    v = t[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]]
    if v.numel() == 0:
        return 0.0
    plane = max(1, v.shape[1] * v.shape[2])
    step = max(1, _CHUNK_CELLS // plane)
    acc = torch.zeros((), dtype=torch.float64, device=t.device)
    for i0 in range(0, v.shape[0], step):
        c = v[i0:i0 + step].to(torch.float64)
        acc += (c * c).sum()
    return float(acc)
