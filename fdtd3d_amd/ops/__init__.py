"""Compute backends.

``hip``   -- hand-written gfx950 kernels (:mod:`.hip_ops`), the production path.
``torch`` -- vectorised torch reference ops (:mod:`.torch_ops`), the CPU oracle.
"""

import torch

from .coef import Coef
from .torch_ops import TorchOps


def resolve_backend(backend: str = "auto", device: str = "auto"):
    """Pick (backend, device).  ``auto`` means HIP on a GPU when one is
    visible, torch on CPU otherwise."""
    has_gpu = torch.cuda.is_available()
    if device == "auto":
        device = "cuda" if has_gpu else "cpu"
    if backend == "auto":
        backend = "hip" if (has_gpu and str(device).startswith("cuda")) else "torch"
    return backend, device


def make_ops(backend: str, layout, device, dtype, **kw):
    if backend == "hip":
        from .hip_ops import HipOps
        return HipOps(layout, device, dtype, **kw)
    if backend == "torch":
        return TorchOps(layout, device, dtype)
    raise ValueError("unknown backend %r" % backend)
