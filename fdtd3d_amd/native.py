"""ctypes bindings of the native host runtime (``libfdtd3d_host.so``).

The standalone ``fdtd3d`` executable (csrc/main.cpp) is built from the same
objects; these bindings exist so the Python tests can pin the native settings
parser and topology optimiser to their Python counterparts
(utils/settings.py, parallel/topology.py).
"""
from __future__ import annotations

import ctypes
import json
import os
import threading
from typing import Dict, Sequence, Tuple

from .ops.build import EXE, LIB_HOST

_lib = None
_lock = threading.Lock()


def _host_stale() -> bool:
    """The host library is missing or older than a host source (the object
    files do not travel to the GPU boxes, so their timestamps say nothing)."""
    if not os.path.exists(LIB_HOST):
        return True
    from .ops import build as _b
    t = os.path.getmtime(LIB_HOST)
    return any(os.path.getmtime(d) > t for src in _b.host_sources() for d in _b._deps(src))


def load_host_library(build_if_missing: bool = True) -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:  # decomposed thread ranks reach here together on their first hybrid plan
        if _lib is not None:
            return _lib
        return _load_host_library(build_if_missing)


def _load_host_library(build_if_missing: bool) -> ctypes.CDLL:
    global _lib
    if build_if_missing and _host_stale():
        from .ops import build as _b
        _b.build(exe=False, hip=False)  # incremental: rebuilds only when csrc changed
    lib = ctypes.CDLL(LIB_HOST)
    lib.fdtd_settings_parse_json.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                             ctypes.c_char_p, ctypes.c_int]
    lib.fdtd_settings_parse_json.restype = ctypes.c_int
    lib.fdtd_optimal_topology.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_int)]
    lib.fdtd_optimal_topology.restype = None
    ip = ctypes.POINTER(ctypes.c_int)
    lib.fdtd_hybrid_windows.argtypes = [ip, ip, ip, ip, ip, ctypes.c_int, ip, ctypes.c_int]
    lib.fdtd_hybrid_windows.restype = ctypes.c_int
    _lib = lib
    return lib


def parse_settings(argv: Sequence[str]) -> Tuple[int, object]:
    """Parse ``argv`` with the native parser: (status, dict-or-message)."""
    lib = load_host_library()
    arr = (ctypes.c_char_p * len(argv))(*[a.encode() for a in argv])
    buf = ctypes.create_string_buffer(1 << 16)
    st = lib.fdtd_settings_parse_json(len(argv), arr, buf, len(buf))
    text = buf.value.decode()
    if st == 0:
        return st, json.loads(text)
    return st, text


def optimal_topology(size: Sequence[int], nprocs: int, axes: Sequence[int] = (0, 1, 2)) -> Tuple[int, int, int]:
    lib = load_host_library()
    s = (ctypes.c_int * 3)(*size)
    ax = (ctypes.c_int * len(axes))(*axes)
    out = (ctypes.c_int * 3)()
    lib.fdtd_optimal_topology(s, nprocs, ax, len(axes), out)
    return tuple(out)


def hybrid_windows(alloc, core, cut, size: Sequence[int], active: Sequence[bool], T: int):
    """Geometry of a hybrid pass (``csrc/host_native.cpp`` ``fdtd::hybrid_windows``,
    the plan the native driver uses too): per step s of the pass the stepped
    shell's windows, and the boxes copied into the core pass's output
    afterwards.  Boxes are ((lo), (hi)); ``cut`` is a box cut out of the core
    and stepped with the shell (None: none).  None when a step's core
    vanishes."""
    lib = load_host_library()

    def flat(b):
        return (ctypes.c_int * 6)(*(list(b[0]) + list(b[1])))

    none = ((0, 0, 0), (0, 0, 0))
    cap = 6 * 16 * (T + 1) + T + 1
    out = (ctypes.c_int * cap)()
    n = lib.fdtd_hybrid_windows(flat(alloc), flat(core), flat(cut if cut is not None else none),
                                (ctypes.c_int * 3)(*size), (ctypes.c_int * 3)(*[1 if a else 0 for a in active]),
                                int(T), out, cap)
    if n == -1:
        return None
    if n < 0:
        raise RuntimeError("fdtd_hybrid_windows: output table too small")
    vals, q, lists = list(out[:n]), 0, []
    for _ in range(T + 1):
        cnt = vals[q]
        q += 1
        boxes = []
        for _ in range(cnt):
            b = vals[q:q + 6]
            q += 6
            boxes.append((tuple(b[:3]), tuple(b[3:])))
        lists.append(boxes)
    return lists[:T], lists[T]


def executable() -> str:
    return EXE


def settings_dict_equal(native: Dict[str, object], py: Dict[str, object]) -> bool:
    for k, v in py.items():
        n = native.get(k)
        if isinstance(v, float):
            if n is None or abs(float(n) - v) > 1e-12 * max(1.0, abs(v)):
                return False
        elif n != v:
            return False
    return True
