"""Checkpoint / resume.

The reference has a per-rank raw DAT format but never wires it into the
solver (``--load-from-file`` is on its TODO list, ``Settings.inc:128``).
Here a checkpoint is, per rank:

* one DAT file per state array in the reference's naming and byte layout --
  ``current[<step>]_rank-<r>_<name>.dat``, local grid incl. ghost layers, z
  fastest (``DATDumper.h:85-118``) -- so field files stay readable by
  reference tooling;
* a JSON sidecar ``checkpoint[<step>]_rank-<r>.json`` with the step, global
  size, local box, dtype, topology and the list of arrays.

``load_checkpoint`` validates the sidecar against the running scheme (same
global grid, decomposition and dtype) and restores every array in place, so a
resumed run continues bit-identically.
"""

from __future__ import annotations

import json
import os
from typing import Optional

import torch

from ..version import __version__
from .dat import read_dat, write_dat
from .naming import GridFileType, grid_file_name


def _sidecar(directory: str, step: int, rank: int) -> str:
    return os.path.join(directory, "checkpoint[%d]_rank-%d.json" % (step, rank))


def save_checkpoint(scheme, directory: str) -> str:
    os.makedirs(directory, exist_ok=True)
    d = scheme.domain
    rank = d.rank
    step = scheme.t
    names = []
    for name, t in scheme.named_state().items():
        write_dat(grid_file_name(step, GridFileType.CURRENT, rank, name, directory), t)
        names.append({"name": name, "shape": list(t.shape)})
    meta = {
        "format": "fdtd3d-amd-checkpoint-1",
        "version": __version__,
        "step": step,
        "sub_step": scheme.sub_step,
        "scheme": scheme.cfg.scheme,
        "size": list(scheme.cfg.size),
        "dtype": scheme.cfg.dtype,
        "complex": scheme.planes == 2,
        "rank": rank,
        "topology": list(d.topology),
        "buffer_size": d.buffer_size,
        "lo": list(d.lo),
        "hi": list(d.hi),
        "origin": list(d.origin),
        "local_shape": list(d.shape),
        "dx": scheme.dx,
        "dt": scheme.dt,
        "arrays": names,
    }
    path = _sidecar(directory, step, rank)
    with open(path, "w") as f:
        json.dump(meta, f, indent=1)
    return path


def latest_step(directory: str, rank: int = 0) -> Optional[int]:
    best = None
    if not os.path.isdir(directory):
        return None
    suffix = "]_rank-%d.json" % rank
    for fn in os.listdir(directory):
        if fn.startswith("checkpoint[") and fn.endswith(suffix):
            s = int(fn[len("checkpoint["):-len(suffix)])
            best = s if best is None or s > best else best
    return best


def load_checkpoint(scheme, directory: str, step: Optional[int] = None) -> int:
    d = scheme.domain
    rank = d.rank
    if step is None:
        step = latest_step(directory, rank)
        if step is None:
            raise FileNotFoundError("no checkpoint for rank %d in %s" % (rank, directory))
    with open(_sidecar(directory, step, rank)) as f:
        meta = json.load(f)
    checks = [("size", list(scheme.cfg.size)), ("dtype", scheme.cfg.dtype), ("complex", scheme.planes == 2),
              ("local_shape", list(d.shape)), ("origin", list(d.origin)), ("scheme", scheme.cfg.scheme)]
    for key, want in checks:
        if meta[key] != want:
            raise ValueError("checkpoint %s mismatch: file %r, run %r" % (key, meta[key], want))
    state = scheme.named_state()
    listed = {a["name"] for a in meta["arrays"]}
    missing = set(state) - listed
    if missing:
        raise ValueError("checkpoint lacks arrays %s" % sorted(missing))
    for name, t in state.items():
        v = read_dat(grid_file_name(step, GridFileType.CURRENT, rank, name, directory), tuple(t.shape), t.dtype)
        t.copy_(v.to(t.device))
    scheme.t = int(meta["step"])
    scheme.sub_step = int(meta.get("sub_step", 0))
    return scheme.t
