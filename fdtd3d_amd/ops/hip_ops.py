"""HIP backend: the solver operations as launches of the hand-written gfx950
kernels in ``libfdtd3d_hip.so`` (``fdtd3d_amd/csrc/*.hip``).

The library is a plain C ABI loaded with ctypes *after* ``import torch``, so
it binds to the HIP runtime PyTorch already loaded; every launch goes to
``torch.cuda.current_stream()``, which makes the whole time step capturable
in a HIP graph (``torch.cuda.CUDAGraph``) and orders it with RCCL work issued
by ``torch.distributed``.

Every entry point validates on the host that the boxes it passes keep all
stencil reads inside the arrays (the kernels do no bounds checks beyond their
boxes), and raises if the library is missing -- a GPU run never silently falls
back to the torch reference ops.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..layout.yee import YeeLayout
from ..models.regions import RegionLevel
from .coef import Coef

Box = Tuple[Tuple[int, int, int], Tuple[int, int, int]]

_LIB = None
TB_MAX_STEPS = 6  # steps per pass of the blocked kernels (fdtd_tb_max_steps)
TB_MAX_STEPS_F64 = 5  # fp64 blocked kernel (fdtd_tb64_max_steps)
TB2D_MAX_STEPS = 8  # 2D TMz / TEz blocked kernel, fp32 (fdtd_tb2d_max_steps)
TB2D_MAX_STEPS_F64 = 8  # fp64 (fdtd_tb2d64_max_steps)
TB2D_MODES = {("Ez",): (0, ("Ez",), ("Hx", "Hy")), ("Ex", "Ey"): (1, ("Ex", "Ey"), ("Hz",))}
# FDTD3D_HIP_LIB: another build of the library (A/B kernel measurements)
_LIB_PATH = os.environ.get("FDTD3D_HIP_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                            "libfdtd3d_hip.so")

c_int = ctypes.c_int
c_ll = ctypes.c_longlong
c_double = ctypes.c_double
c_vp = ctypes.c_void_p


class HipError(RuntimeError):
    pass


def lib_path() -> str:
    return _LIB_PATH


_LIB_LOCK = threading.Lock()


def load_library(build_if_missing: bool = True):
    if _LIB is not None:
        return _LIB
    with _LIB_LOCK:  # thread ranks construct their ops together
        return _load_library(build_if_missing)


def _load_library(build_if_missing: bool):
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(_LIB_PATH) and build_if_missing:
        from .build import build
        build(exe=False)
    if not os.path.exists(_LIB_PATH):
        raise HipError("libfdtd3d_hip.so not found at %s: run `python -m fdtd3d_amd.ops.build`" % _LIB_PATH)
    _LIB = ctypes.CDLL(_LIB_PATH)
    _LIB.fdtd_abi_version.restype = c_int
    return _LIB


def available() -> bool:
    try:
        load_library(build_if_missing=False)
    except (HipError, OSError):
        return False
    return torch.cuda.is_available()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise HipError("%s failed: hipError %d" % (what, rc))


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _box_arr(boxes: Sequence[Box]):
    vals = []
    for b in boxes:
        vals += list(b[0]) + list(b[1])
    return (c_int * len(vals))(*vals)


def _empty(b: Box) -> bool:
    return any(b[1][d] <= b[0][d] for d in range(3))


class _RecFn:
    """A ``libfdtd3d_hip`` entry point that, while its ops object records
    (:meth:`HipOps.record`), also appends (function, arguments, returns a
    status) to the record: every argument is already a ctypes value, so the
    call replays as is."""
    __slots__ = ("f", "ops", "status")

    def __init__(self, f, ops, status):
        self.f, self.ops, self.status = f, ops, status

    def __call__(self, *args):
        rec = self.ops._rec
        if rec is not None:
            rec.append((self.f, args, self.status))
        return self.f(*args)


class _LibProxy:
    """``libfdtd3d_hip`` seen through :class:`_RecFn` wrappers."""

    def __init__(self, lib, ops):
        self._lib, self._ops, self._w = lib, ops, {}

    def __getattr__(self, name):
        w = self._w.get(name)
        if w is None:
            f = getattr(self._lib, name)
            # the knob setters (fdtd_set_tb_*, ...) return void; everything else an hipError status
            status = not (name.startswith("fdtd_set_") and not name.startswith("fdtd_set_value"))
            w = self._w[name] = _RecFn(f, self._ops, status) if name.startswith("fdtd_") else f
        return w


# a CPML term table with no slab (9 terms x 5 null pointers, 9 x 4 zero ranges): the
# folded-CPML kernels then run the plain update
_EMPTY_CPML = ((c_vp * 45)(), (c_int * 36)())


class HipOps:
    name = "hip"
    # fp64 3D split updates on the double4 lanes of yee3d_cpml.hip (FDTD3D_F64_V4=1): 512^3 stepped vacuum
    # +6%, but the UPML shell windows -3% (profiles/physics_r6.md): off by default
    f64_v4 = os.environ.get("FDTD3D_F64_V4", "0") == "1"

    def __init__(self, layout: Optional[YeeLayout], device, dtype, xchunk: int = 0, vec4: bool = True):
        self.vec4 = vec4
        self.layout = layout
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise HipError("the HIP backend needs a GPU device, got %s" % self.device)
        self.dtype = dtype
        self.suf = {torch.float32: "f32", torch.float64: "f64"}[dtype]
        self._rec = None
        self.lib = _LibProxy(load_library(), self)
        self.xchunk = xchunk
        self._fn: Dict[str, object] = {}
        self.launches = 0

    def fn(self, name: str):
        f = self._fn.get(name)
        if f is None:
            f = getattr(self.lib, "fdtd_%s_%s" % (name, self.suf))
            f.f.restype = c_int
            self._fn[name] = f
        return f

    # ------------------------------------------------------------ launch records
    def record(self, rec: Optional[list]) -> None:
        """Start (a list) / stop (None) recording every library call: the
        calls still run; :meth:`replay` re-issues the recorded ones.  Only
        kernel launches through this object are recorded -- the recorded
        section must not depend on torch operations."""
        self._rec = rec

    @staticmethod
    def replay(rec: list) -> None:
        """Re-issue recorded library calls in order, as recorded (pointers,
        boxes and the stream are baked into the arguments): a pass's launches
        straight from a list, without the Python planning around them."""
        for f, args, status in rec:
            rc = f(*args)
            if status and rc:
                raise HipError("replayed launch failed: hipError %d" % rc)

    # ------------------------------------------------------------ validation
    def _check_tensor(self, t: torch.Tensor, shape=None) -> None:
        if t.device.type != "cuda" or t.dtype != self.dtype or not t.is_contiguous():
            raise HipError("HIP op got a tensor on %s/%s (contiguous=%s)" % (t.device, t.dtype, t.is_contiguous()))
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise HipError("HIP op shape mismatch %s vs %s" % (tuple(t.shape), tuple(shape)))

    def _check_stencil_box(self, kind: str, comp: str, box: Box, shape) -> None:
        for d in range(3):
            if box[0][d] < 0 or box[1][d] > shape[d]:
                raise HipError("box %s of %s outside array %s" % (box, comp, shape))
        for (s, axis, _) in self.layout.curl_terms(comp):
            if kind == "E" and box[0][axis] < 1:
                raise HipError("E box %s of %s would read index -1 along axis %d" % (box, comp, axis))
            if kind == "H" and box[1][axis] > shape[axis] - 1:
                raise HipError("H box %s of %s would read past the array along axis %d" % (box, comp, axis))

    def _coef_args(self, c: Coef):
        ps = (c_vp * 4)(*[None if t is None else t.data_ptr() for t in (c.px, c.py, c.pz, c.cell)])
        for t in (c.px, c.py, c.pz, c.cell):
            if t is not None:
                self._check_tensor(t)
        return c_double(c.scalar), ps

    @staticmethod
    def _cell_or_none(c: Coef):
        if c.px is not None or c.py is not None or c.pz is not None:
            raise HipError("fast-path coefficient must be scalar or per-cell")
        return c.cell

    # ------------------------------------------------------------------ curl
    multi2d = True  # 2D windows of a half step in one launch (curl_update_multi)

    def curl_update_multi(self, kind: str, windows: Sequence[Dict[str, Box]], dst: Dict[str, torch.Tensor],
                          src: Dict[str, torch.Tensor], cb: Dict[str, Coef]) -> None:
        """2D (TMz / TEz): :meth:`curl_update` of several disjoint windows
        (per window the component boxes) in one launch per 8 windows
        (yee_lowdim.hip ``Win2``: the hybrid shell's strips replay from a HIP
        graph, where a step costs its launch count)."""
        scheme = self.layout.scheme
        if scheme not in ("tmz", "tez"):
            for w in windows:
                self.curl_update(kind, w, dst, src, cb)
            return
        names = {("tmz", "E"): ("Ez",), ("tmz", "H"): ("Hx", "Hy"), ("tez", "E"): ("Ex", "Ey"),
                 ("tez", "H"): ("Hz",)}[(scheme, kind)]
        shape = tuple(dst[names[0]].shape)
        for c in names:
            self._check_tensor(dst[c], shape)
        wins = [w for w in windows if not all(_empty(w[c]) for c in names)]
        for w in wins:
            for c in names:
                if not _empty(w[c]):
                    self._check_stencil_box(kind, c, w[c], shape)
        st = _stream()
        for q in range(0, len(wins), 8):
            part = wins[q:q + 8]
            bx = _box_arr([w[c] for w in part for c in names])
            n = c_int(len(part))
            if scheme == "tmz" and kind == "E":
                rc = self.fn("tmz_e_multi")(_ptr(dst["Ez"]), _ptr(src["Hx"]), _ptr(src["Hy"]), self._cellp(cb["Ez"]),
                                            c_double(self._scal(cb["Ez"])), c_int(shape[0]), c_int(shape[1]), bx, n,
                                            st)
            elif scheme == "tmz":
                rc = self.fn("tmz_h_multi")(_ptr(dst["Hx"]), _ptr(dst["Hy"]), _ptr(src["Ez"]), self._cellp(cb["Hx"]),
                                            self._cellp(cb["Hy"]), c_double(self._scal(cb["Hx"])), c_int(shape[0]),
                                            c_int(shape[1]), bx, n, st)
            elif kind == "E":
                rc = self.fn("tez_e_multi")(_ptr(dst["Ex"]), _ptr(dst["Ey"]), _ptr(src["Hz"]), self._cellp(cb["Ex"]),
                                            self._cellp(cb["Ey"]), c_double(self._scal(cb["Ex"])), c_int(shape[0]),
                                            c_int(shape[1]), bx, n, st)
            else:
                rc = self.fn("tez_h_multi")(_ptr(dst["Hz"]), _ptr(src["Ex"]), _ptr(src["Ey"]), self._cellp(cb["Hz"]),
                                            c_double(self._scal(cb["Hz"])), c_int(shape[0]), c_int(shape[1]), bx, n,
                                            st)
            _check(rc, "%s_%s_multi" % (scheme, kind.lower()))
            self.launches += 1

    def curl_update(self, kind: str, boxes: Dict[str, Box], dst: Dict[str, torch.Tensor],
                    src: Dict[str, torch.Tensor], cb: Dict[str, Coef]) -> None:
        lay = self.layout
        comps = list(boxes.keys())
        any_t = dst[comps[0]]
        shape = tuple(any_t.shape)
        for c in comps:
            self._check_tensor(dst[c], shape)
            if not _empty(boxes[c]):
                self._check_stencil_box(kind, c, boxes[c], shape)
        scheme = lay.scheme
        st = _stream()
        if scheme == "3d":
            names = ("Ex", "Ey", "Ez") if kind == "E" else ("Hx", "Hy", "Hz")
            other = ("Hx", "Hy", "Hz") if kind == "E" else ("Ex", "Ey", "Ez")
            for c in other:
                self._check_tensor(src[c], shape)
            per = [self._cell_or_none(cb[c]) for c in names]
            if any(p is None for p in per) and not all(p is None for p in per):
                raise HipError("mixed scalar/per-cell coefficients")
            scal = cb[names[0]].scalar
            if per[0] is None and any(cb[c].scalar != scal for c in names):
                raise HipError("scalar coefficients must agree across components")
            bx = _box_arr([boxes[c] for c in names])
            base = "update_e3d" if kind == "E" else "update_h3d"
            per_p = [_ptr(p) if p is not None else None for p in per]
            if per[0] is not None:
                scal_use = 1.0
                # per-cell arrays already include the scalar? No: multiply on the host once
                per_p = [_ptr(self._scaled_cell(cb[c])) for c in names]
            else:
                scal_use = scal
            args = [*[_ptr(dst[c]) for c in names], *[_ptr(src[c]) for c in other], *per_p, c_double(scal_use),
                    c_int(shape[0]), c_int(shape[1]), c_int(shape[2]), bx, c_int(self.xchunk)]
            if self.vec4 and self.dtype == torch.float64 and shape[2] % 4 == 0 and self.f64_v4:
                # fp64: the 4-cell double4 lanes of yee3d_cpml.hip with an empty CPML
                # table -- the plain update, with the thin-box lane layouts (a z-thin
                # shell window runs 8- or 16-lane rows instead of idle 64-lane ones)
                rc = self.fn(base + "_cpml_v4")(*args, _EMPTY_CPML[0], _EMPTY_CPML[1], st)
                _check(rc, "update_%s3d" % kind.lower())
                self.launches += 1
                return
            if self.vec4 and self.dtype == torch.float32 and shape[2] % 4 == 0:
                base += "_v4"
            rc = self.fn(base)(*args, st)
            _check(rc, "update_%s3d" % kind.lower())
            self.launches += 1
            return
        if scheme == "tmz":
            if kind == "E":
                b = boxes["Ez"]
                rc = self.fn("tmz_e")(_ptr(dst["Ez"]), _ptr(src["Hx"]), _ptr(src["Hy"]),
                                      self._cellp(cb["Ez"]), c_double(self._scal(cb["Ez"])),
                                      c_int(shape[0]), c_int(shape[1]), _box_arr([b]), c_int(0), st)
            else:
                rc = self.fn("tmz_h")(_ptr(dst["Hx"]), _ptr(dst["Hy"]), _ptr(src["Ez"]),
                                      self._cellp(cb["Hx"]), self._cellp(cb["Hy"]), c_double(self._scal(cb["Hx"])),
                                      c_int(shape[0]), c_int(shape[1]), _box_arr([boxes["Hx"], boxes["Hy"]]),
                                      c_int(0), st)
        elif scheme == "tez":
            if kind == "E":
                rc = self.fn("tez_e")(_ptr(dst["Ex"]), _ptr(dst["Ey"]), _ptr(src["Hz"]),
                                      self._cellp(cb["Ex"]), self._cellp(cb["Ey"]), c_double(self._scal(cb["Ex"])),
                                      c_int(shape[0]), c_int(shape[1]), _box_arr([boxes["Ex"], boxes["Ey"]]),
                                      c_int(0), st)
            else:
                rc = self.fn("tez_h")(_ptr(dst["Hz"]), _ptr(src["Ex"]), _ptr(src["Ey"]),
                                      self._cellp(cb["Hz"]), c_double(self._scal(cb["Hz"])),
                                      c_int(shape[0]), c_int(shape[1]), _box_arr([boxes["Hz"]]), c_int(0), st)
        else:  # 1d
            if kind == "E":
                b = boxes["Ez"]
                rc = self.fn("1d_e")(_ptr(dst["Ez"]), _ptr(src["Hy"]), self._cellp(cb["Ez"]),
                                     c_double(self._scal(cb["Ez"])), c_int(b[0][0]), c_int(b[1][0] if not _empty(b) else b[0][0]), st)
            else:
                b = boxes["Hy"]
                rc = self.fn("1d_h")(_ptr(dst["Hy"]), _ptr(src["Ez"]), self._cellp(cb["Hy"]),
                                     c_double(self._scal(cb["Hy"])), c_int(b[0][0]), c_int(b[1][0] if not _empty(b) else b[0][0]), st)
        _check(rc, "%s %s update" % (scheme, kind))
        self.launches += 1

    def resident_1d_max_cells(self) -> int:
        return int(self.lib.fdtd_res1d_max_cells(c_int(self.dtype.itemsize)))

    def resident_1d(self, F: Dict[str, torch.Tensor], boxes: Dict[str, Box], cb: Dict[str, Coef], nsteps: int,
                    src_i: Optional[int] = None, vals: Optional[torch.Tensor] = None) -> None:
        """``nsteps`` 1D leapfrog steps of (Ez, Hy) in place in ONE launch of
        one register-resident workgroup (yee1d_res.hip); ``vals`` = device
        tensor of the hard Ez source value at cell ``src_i`` for each step."""
        ez, hy = F["Ez"], F["Hy"]
        n = ez.numel()
        self._check_tensor(ez, tuple(ez.shape))
        self._check_tensor(hy, tuple(ez.shape))
        if n > self.resident_1d_max_cells():
            raise HipError("resident 1D kernel holds at most %d cells, got %d" % (self.resident_1d_max_cells(), n))
        be, bh = boxes["Ez"], boxes["Hy"]
        lim = lambda b: (b[0][0], b[1][0]) if not _empty(b) else (0, 0)
        (elo, ehi), (hlo, hhi) = lim(be), lim(bh)
        if (ehi > elo and (elo < 1 or ehi > n)) or (hhi > hlo and (hlo < 0 or hhi > n - 1)):
            raise HipError("1D boxes %s / %s read outside %d cells" % (be, bh, n))
        if self._cell_or_none(cb["Ez"]) is not None or self._cell_or_none(cb["Hy"]) is not None:
            pe, ph = self._cell_array(cb["Ez"], tuple(ez.shape)), self._cell_array(cb["Hy"], tuple(ez.shape))
            pe_p, ph_p, cbv, dbv = pe.data_ptr(), ph.data_ptr(), 1.0, 1.0
        else:
            pe_p, ph_p, cbv, dbv = None, None, cb["Ez"].scalar, cb["Hy"].scalar
        vp = None
        si = -1
        if vals is not None:
            if src_i is None or not (0 <= src_i < n) or vals.numel() < nsteps:
                raise HipError("resident_1d: bad source (%s, %d values for %d steps)" % (src_i, vals.numel(), nsteps))
            self._check_tensor(vals, tuple(vals.shape))
            vp, si = vals.data_ptr(), int(src_i)
        rc = self.fn("res1d")(c_vp(ez.data_ptr()), c_vp(hy.data_ptr()), c_vp(pe_p), c_vp(ph_p), c_double(cbv),
                              c_double(dbv), c_int(n), (c_int * 4)(elo, ehi, hlo, hhi), c_int(nsteps), c_int(si),
                              c_vp(vp), _stream())
        _check(rc, "res1d")
        self.launches += 1

    def fused_step(self, fin: Dict[str, torch.Tensor], fout: Dict[str, torch.Tensor], boxes: Dict[str, Box],
                   cb: Dict[str, Coef], source=None) -> None:
        """One fused E+H leapfrog step (yee3d.hip ``k_fused3d``): reads
        ``fin``, writes ``fout`` on the union of the six boxes.  ``source`` =
        (component, local index, value) of a hard point source or None."""
        E, H = ("Ex", "Ey", "Ez"), ("Hx", "Hy", "Hz")
        shape = tuple(fin["Ex"].shape)
        for c in E + H:
            self._check_tensor(fin[c], shape)
            self._check_tensor(fout[c], shape)
            if fin[c].data_ptr() == fout[c].data_ptr():
                raise HipError("fused step needs distinct in/out buffers")
            b = boxes[c]
            if not _empty(b):
                self._check_stencil_box("E" if c[0] == "E" else "H", c, b, shape)
        pe = [self._cell_or_none(cb[c]) for c in E]
        ph = [self._cell_or_none(cb[c]) for c in H]
        percell = any(p is not None for p in pe + ph)
        if percell:
            cbs, cbv = self._kind_coef_args(cb, E, pe, shape)
            dbs, dbv = self._kind_coef_args(cb, H, ph, shape)
        else:
            cbs = (c_vp * 3)(None, None, None)
            dbs = (c_vp * 3)(None, None, None)
            cbv, dbv = cb["Ex"].scalar, cb["Hx"].scalar
            if any(cb[c].scalar != cbv for c in E) or any(cb[c].scalar != dbv for c in H):
                raise HipError("fused step: scalar coefficients must agree per kind")
        src_off, src_comp, src_val = -1, -1, 0.0
        if source is not None:
            comp, idx, val = source
            if comp not in E:
                raise HipError("fused step supports E point sources only")
            for d in range(3):
                if not (0 <= idx[d] < shape[d]):
                    raise HipError("source index outside array")
            src_off = (idx[0] * shape[1] + idx[1]) * shape[2] + idx[2]
            src_comp = E.index(comp)
            src_val = val
        arr = lambda names, f: (c_vp * 3)(*[f[c].data_ptr() for c in names])
        name = "fused3d"
        if self.vec4 and self.dtype == torch.float32 and shape[2] % 4 == 0:
            name = "fused3d_v4"
        rc = self.fn(name)(arr(E, fin), arr(H, fin), arr(E, fout), arr(H, fout), cbs, dbs, c_double(cbv),
                                c_double(dbv), c_int(shape[0]), c_int(shape[1]), c_int(shape[2]),
                                _box_arr([boxes[c] for c in E + H]), c_int(self.xchunk), c_ll(src_off),
                                c_int(src_comp), c_double(src_val), _stream())
        _check(rc, "fused3d")
        self.launches += 1

    # per-cell coefficient arrays for the fast kernels are scalar*cell, cached
    def _scaled_cell(self, c: Coef) -> torch.Tensor:
        key = "_scaled"
        cached = getattr(c, key, None)
        if cached is None:
            cached = (c.cell * c.scalar).to(self.dtype).contiguous()
            setattr(c, key, cached)
        return cached

    def _cell_array(self, c: Coef, shape) -> torch.Tensor:
        """scalar*cell as a full array; a scalar coefficient becomes a
        cached constant array (kernels with one per-cell form for E and H)."""
        if c.cell is not None:
            return self._scaled_cell(c)
        cached = getattr(c, "_const_arr", None)
        if cached is None or tuple(cached.shape) != tuple(shape):
            cached = torch.full(tuple(shape), float(c.scalar), dtype=self.dtype, device=self.device)
            c._const_arr = cached
        return cached

    def _kind_coef_args(self, cb: Dict[str, Coef], names, cells, shape):
        """(3 array pointers, scalar) of one kind (E or H) for the per-cell
        forms of the fused / blocked kernels.  A kind whose three
        coefficients are one scalar passes null arrays and that scalar, so a
        dielectric scene's H update reads no constant coefficient planes."""
        sc = cb[names[0]].scalar
        if all(p is None for p in cells) and all(cb[c].scalar == sc for c in names):
            return (c_vp * 3)(None, None, None), sc
        return (c_vp * 3)(*[self._cell_array(cb[c], shape).data_ptr() for c in names]), 1.0

    def _sparse_kind(self, cb: Dict[str, Coef], names, shape):
        """Sparse per-cell form of one kind's coefficients for the multi-row
        blocked kernel: (float4 array over the box of cells whose value
        differs from the kind's dominant value -- one (x, y, z, 0) vector per
        cell --, that box, the dominant value).  A kind of one scalar gives
        (None, empty box, scalar).  Cached on the kind's first Coef."""
        sc = cb[names[0]].scalar
        if all(cb[c].cell is None for c in names) and all(cb[c].scalar == sc for c in names):
            return None, ((0, 0, 0), (0, 0, 0)), sc
        cached = getattr(cb[names[0]], "_sparse4", None)
        if cached is not None and cached[3] == tuple(shape):
            return cached[:3]
        arrs = [self._cell_array(cb[c], shape) for c in names]
        flat = arrs[0].reshape(-1)
        sample = flat[:: max(1, flat.numel() // (1 << 20))]
        dom = float(torch.mode(sample).values)  # fp32 value, exact in a double
        diff = (arrs[0] != dom) | (arrs[1] != dom) | (arrs[2] != dom)
        lo, hi = [], []
        for d in range(3):
            other = tuple(a for a in range(3) if a != d)
            nz = torch.nonzero(diff.any(dim=other)).view(-1)
            if nz.numel() == 0:
                lo, hi = [0, 0, 0], [0, 0, 0]
                break
            lo.append(int(nz[0]))
            hi.append(int(nz[-1]) + 1)
        box = (tuple(lo), tuple(hi))
        if _empty(box):
            out = (None, box, dom)
        else:
            sl = tuple(slice(lo[d], hi[d]) for d in range(3))
            v = torch.zeros(tuple(hi[d] - lo[d] for d in range(3)) + (4,), dtype=self.dtype, device=self.device)
            for n in range(3):
                v[..., n] = arrs[n][sl]
            out = (v.contiguous(), box, dom)
        cb[names[0]]._sparse4 = out + (tuple(shape),)
        return out

    def _cellp(self, c: Coef):
        self._cell_or_none(c)
        return None if c.cell is None else _ptr(self._scaled_cell(c))

    @staticmethod
    def _scal(c: Coef) -> float:
        return 1.0 if c.cell is not None else c.scalar

    def curl_general(self, kind: str, comp: str, box: Box, out: torch.Tensor, inp: torch.Tensor,
                     src: Dict[str, torch.Tensor], ca: Coef, cb: Coef) -> None:
        if _empty(box):
            return
        shape = tuple(out.shape)
        self._check_tensor(out, shape)
        self._check_tensor(inp, shape)
        self._check_stencil_box(kind, comp, box, shape)
        terms = self.layout.curl_terms(comp)
        srcs = (c_vp * 2)(*[src[s].data_ptr() for (s, _, _) in terms] + [0] * (2 - len(terms)))
        axes = (c_int * 2)(*[a for (_, a, _) in terms] + [0] * (2 - len(terms)))
        signs = (c_int * 2)(*[g for (_, _, g) in terms] + [1] * (2 - len(terms)))
        for (s, _, _) in terms:
            self._check_tensor(src[s], shape)
        cas, cap = self._coef_args(ca)
        cbs, cbp = self._coef_args(cb)
        rc = self.fn("curl_general")(_ptr(out), _ptr(inp), srcs, axes, signs, c_int(len(terms)),
                                     c_int(1 if kind == "E" else 0), cas, cap, cbs, cbp, c_int(shape[1]),
                                     c_int(shape[2]), _box_arr([box]), _stream())
        _check(rc, "curl_general")
        self.launches += 1

    def lincomb(self, out: torch.Tensor, box: Box, terms: Sequence[Tuple[Coef, torch.Tensor]]) -> None:
        if _empty(box):
            return
        shape = tuple(out.shape)
        self._check_tensor(out, shape)
        n = len(terms)
        scal = (c_double * n)(*[c.scalar for c, _ in terms])
        ptrs = []
        for c, x in terms:
            self._check_tensor(x, shape)
            for t in (c.px, c.py, c.pz, c.cell):
                if t is not None:
                    self._check_tensor(t)
                ptrs.append(None if t is None else t.data_ptr())
        pa = (c_vp * len(ptrs))(*ptrs)
        xs = (c_vp * n)(*[x.data_ptr() for _, x in terms])
        rc = self.fn("lincomb")(_ptr(out), c_int(n), scal, pa, xs, c_int(shape[1]), c_int(shape[2]),
                                _box_arr([box]), _stream())
        _check(rc, "lincomb")
        self.launches += 1

    def cpml_apply(self, kind: str, target: torch.Tensor, src: torch.Tensor, axis: int, sign: int,
                   psi: torch.Tensor, psi_box: Box, box: Box, b: torch.Tensor, c: torch.Tensor,
                   kinv_m1: torch.Tensor, cb: Coef) -> None:
        if _empty(box):
            return
        shape = tuple(target.shape)
        self._check_tensor(target, shape)
        self._check_tensor(src, shape)
        for d in range(3):
            if not (psi_box[0][d] <= box[0][d] and box[1][d] <= psi_box[1][d]):
                raise HipError("CPML box %s outside psi box %s" % (box, psi_box))
            if box[0][d] < 0 or box[1][d] > shape[d]:
                raise HipError("CPML box %s outside array %s" % (box, shape))
        if kind == "E" and box[0][axis] < 1 or kind == "H" and box[1][axis] > shape[axis] - 1:
            raise HipError("CPML box %s would read outside the array" % (box,))
        if tuple(psi.shape) != tuple(psi_box[1][d] - psi_box[0][d] for d in range(3)):
            raise HipError("psi shape mismatch")
        cbs, cbp = self._coef_args(cb)
        rc = self.fn("cpml_apply")(_ptr(target), _ptr(src), _ptr(psi), c_int(axis), c_int(sign),
                                   c_int(1 if kind == "E" else 0), _ptr(b), _ptr(c), _ptr(kinv_m1), cbs, cbp,
                                   c_int(shape[1]), c_int(shape[2]), _box_arr([box]), _box_arr([psi_box]), _stream())
        _check(rc, "cpml_apply")
        self.launches += 1

    def cpml_apply_many(self, kind: str, items) -> None:
        """Several :meth:`cpml_apply` corrections of one kind in one launch
        per 8 (generic_kernels.hip ``k_cpml_many``); ``items`` are the
        argument tuples of :meth:`cpml_apply` without ``kind`` (their boxes
        must be disjoint in the targets they update)."""
        items = [it for it in items if not _empty(it[6])]
        for q in range(0, len(items), 8):
            part = items[q:q + 8]
            P, CP, S, I = [], [], [], []
            ny = nz = None
            for target, src, axis, sign, psi, psi_box, box, b, c, kinv_m1, cb in part:
                shape = tuple(target.shape)
                self._check_tensor(target, shape)
                self._check_tensor(src, shape)
                for d in range(3):
                    if not (psi_box[0][d] <= box[0][d] and box[1][d] <= psi_box[1][d]):
                        raise HipError("CPML box %s outside psi box %s" % (box, psi_box))
                    if box[0][d] < 0 or box[1][d] > shape[d]:
                        raise HipError("CPML box %s outside array %s" % (box, shape))
                if kind == "E" and box[0][axis] < 1 or kind == "H" and box[1][axis] > shape[axis] - 1:
                    raise HipError("CPML box %s would read outside the array" % (box,))
                if tuple(psi.shape) != tuple(psi_box[1][d] - psi_box[0][d] for d in range(3)):
                    raise HipError("psi shape mismatch")
                if ny is None:
                    ny, nz = shape[1], shape[2]
                elif (ny, nz) != (shape[1], shape[2]):
                    raise HipError("cpml_apply_many: one array shape per launch")
                cbs, cbp = self._coef_args(cb)
                P += [target.data_ptr(), src.data_ptr(), psi.data_ptr(), b.data_ptr(), c.data_ptr(),
                      kinv_m1.data_ptr()]
                CP += list(cbp)
                S.append(float(cbs.value))
                I += [axis, sign] + list(box[0]) + list(box[1]) + list(psi_box[0]) + list(psi_box[1])
            rc = self.fn("cpml_apply_many")((c_vp * len(P))(*P), (c_vp * len(CP))(*CP), (c_double * len(S))(*S),
                                            (c_int * len(I))(*I), c_int(len(part)), c_int(1 if kind == "E" else 0),
                                            c_int(ny), c_int(nz), _stream())
            _check(rc, "cpml_apply_many")
            self.launches += 1

    # --------------------------------------------------------------- sources
    def set_value(self, t: torch.Tensor, idx: Sequence[int], value: float) -> None:
        s = t.shape
        for d in range(3):
            if not (0 <= idx[d] < s[d]):
                raise HipError("source index %s outside %s" % (idx, tuple(s)))
        off = (idx[0] * s[1] + idx[1]) * s[2] + idx[2]
        _check(self.fn("set_value")(_ptr(t), c_ll(off), c_double(value), _stream()), "set_value")
        self.launches += 1

    def set_values(self, t: torch.Tensor, flat_idx: torch.Tensor, value: float) -> None:
        if flat_idx.numel() == 0:
            return
        if flat_idx.device != t.device or flat_idx.dtype != torch.int64:
            raise HipError("set_values needs int64 indices on the field device")
        _check(self.fn("set_values")(_ptr(t), _ptr(flat_idx), c_int(flat_idx.numel()), c_double(value), _stream()),
               "set_values")
        self.launches += 1

    # ------------------------------------------------------------------ halo
    def pack(self, tensors: Sequence[torch.Tensor], box: Box, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        shape = tuple(tensors[0].shape)
        n = 1
        for d in range(3):
            n *= max(0, box[1][d] - box[0][d])
            if box[0][d] < 0 or box[1][d] > shape[d]:
                raise HipError("pack box %s outside %s" % (box, shape))
        if out is None:
            out = torch.empty(n * len(tensors), dtype=self.dtype, device=self.device)
        if out.numel() < n * len(tensors):
            raise HipError("pack buffer too small")
        for t in tensors:
            self._check_tensor(t, shape)
        ptrs = (c_vp * len(tensors))(*[t.data_ptr() for t in tensors])
        rc = self.fn("box_pack")(ptrs, _ptr(out), c_int(len(tensors)), c_int(shape[1]), c_int(shape[2]),
                                 _box_arr([box]), _stream())
        _check(rc, "box_pack")
        self.launches += 1
        return out

    def box_list(self, table: torch.Tensor, n: int, nblocks: int, pack: bool) -> None:
        """Many (array, box) <-> contiguous buffer copies in one launch
        (aux_kernels.hip k_box_list); ``table`` = n device entries of
        ``box_ent_size()`` bytes (parallel/halo.py ``_BoxList`` builds them and
        checked every box against its array)."""
        if table.device.type != "cuda" or not table.is_contiguous():
            raise HipError("box_list: a contiguous device table")
        rc = self.fn("box_list")(_ptr(table), c_int(n), c_int(nblocks), c_int(1 if pack else 0), _stream())
        _check(rc, "box_list")
        self.launches += 1

    def box_ent_size(self) -> int:
        return int(self.lib.fdtd_box_ent_size())

    def unpack(self, tensors: Sequence[torch.Tensor], box: Box, buf: torch.Tensor) -> None:
        shape = tuple(tensors[0].shape)
        n = 1
        for d in range(3):
            n *= max(0, box[1][d] - box[0][d])
            if box[0][d] < 0 or box[1][d] > shape[d]:
                raise HipError("unpack box %s outside %s" % (box, shape))
        if buf.numel() < n * len(tensors):
            raise HipError("unpack buffer too small")
        for t in tensors:
            self._check_tensor(t, shape)
        ptrs = (c_vp * len(tensors))(*[t.data_ptr() for t in tensors])
        rc = self.fn("box_unpack")(ptrs, _ptr(buf), c_int(len(tensors)), c_int(shape[1]), c_int(shape[2]),
                                   _box_arr([box]), _stream())
        _check(rc, "box_unpack")
        self.launches += 1

    def copy_box(self, src: Sequence[torch.Tensor], dst: Sequence[torch.Tensor], box: Box) -> None:
        """dst[c][box] = src[c][box] for up to 8 component pairs, one launch
        (aux_kernels.hip k_box_xfer)."""
        if _empty(box) or not src:
            return
        if len(src) != len(dst) or len(src) > 8:
            raise HipError("copy_box: 1..8 matching component pairs")
        shape = tuple(src[0].shape)
        for d in range(3):
            if box[0][d] < 0 or box[1][d] > shape[d]:
                raise HipError("copy box %s outside %s" % (box, shape))
        for t in list(src) + list(dst):
            self._check_tensor(t, shape)
        rc = self.fn("box_xfer")((c_vp * len(src))(*[t.data_ptr() for t in src]),
                                 (c_vp * len(dst))(*[t.data_ptr() for t in dst]), c_int(len(src)),
                                 c_int(shape[1]), c_int(shape[2]), _box_arr([box]), _stream())
        _check(rc, "box_xfer")
        self.launches += 1

    # ------------------------------------------------------------ reductions
    def _scratch_u32(self):
        s = getattr(self, "_u32", None)
        if s is None:
            s = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._u32 = s
        return s

    def maxabs(self, t: torch.Tensor, box: Box) -> float:
        if _empty(box):
            return 0.0
        self._check_tensor(t)
        s = self._scratch_u32()
        s.zero_()
        rc = self.fn("box_maxabs")(_ptr(t), c_int(t.shape[1]), c_int(t.shape[2]), _box_arr([box]), _ptr(s), _stream())
        _check(rc, "box_maxabs")
        return float(s.view(torch.float32).item())

    def amplitude_update(self, f: torch.Tensor, amp: torch.Tensor, box: Box, accuracy: float) -> int:
        if _empty(box):
            return 0
        self._check_tensor(f)
        self._check_tensor(amp, tuple(f.shape))
        s = self._scratch_u32()
        s.zero_()
        rc = self.fn("amplitude_update")(_ptr(f), _ptr(amp), c_int(f.shape[1]), c_int(f.shape[2]), _box_arr([box]),
                                         c_double(accuracy), _ptr(s), _stream())
        _check(rc, "amplitude_update")
        return int(s.item())

    def _check_amp(self, amps: Sequence[torch.Tensor], shape) -> int:
        """Running-maximum arrays: the field shape, rows contiguous, one x
        stride for all (models/scheme.py keeps the six components of an x plane
        together); returns that stride."""
        xs = amps[0].stride(0)
        for a in amps:
            if a.device.type != "cuda" or a.dtype != self.dtype or tuple(a.shape) != tuple(shape):
                raise HipError("amplitude array %s/%s %s vs field shape %s" % (a.device, a.dtype, tuple(a.shape),
                                                                              tuple(shape)))
            if a.stride() != (xs, shape[2], 1) or xs < shape[1] * shape[2]:
                raise HipError("amplitude arrays need strides (xs, nz, 1), got %s" % (a.stride(),))
        return xs

    def amplitude_update_many(self, fields: Sequence[torch.Tensor], amps: Sequence[torch.Tensor],
                              boxes: Sequence[Box], accuracy: float, counter: torch.Tensor) -> None:
        """Amplitude update of several components in one launch; the number
        of changed cells is ADDED to the device int32 ``counter`` (one
        element) -- no host synchronisation."""
        shape = tuple(fields[0].shape)
        xs = self._check_amp(amps, shape)
        for f in fields:
            self._check_tensor(f, shape)
        for b in boxes:
            for d in range(3):
                if not _empty(b) and (b[0][d] < 0 or b[1][d] > shape[d]):
                    raise HipError("amplitude box %s outside array %s" % (b, shape))
        if counter.device.type != "cuda" or counter.dtype != torch.int32 or counter.numel() < 1:
            raise HipError("amplitude counter: one int32 on the device")
        n = len(fields)
        rc = self.fn("amplitude_many")((c_vp * n)(*[f.data_ptr() for f in fields]),
                                       (c_vp * n)(*[a.data_ptr() for a in amps]), c_int(n), c_int(shape[1]),
                                       c_int(shape[2]), _box_arr(boxes), ctypes.c_longlong(xs), c_double(accuracy),
                                       c_vp(counter.data_ptr()), _stream())
        _check(rc, "amplitude_many")
        self.launches += 1

    # ----------------------------------------------------------------- TF/SF
    def inc_step_e(self, einc: torch.Tensor, hinc: torch.Tensor, coef: float, source: float) -> None:
        _check(self.fn("inc_e")(_ptr(einc), _ptr(hinc), c_int(einc.numel()), c_double(coef), c_double(source),
                                _stream()), "inc_e")

    def inc_step_h(self, einc: torch.Tensor, hinc: torch.Tensor, coef: float) -> None:
        _check(self.fn("inc_h")(_ptr(einc), _ptr(hinc), c_int(einc.numel()), c_double(coef), _stream()), "inc_h")

    def tfsf_apply(self, target: torch.Tensor, table, inc: torch.Tensor, box: Box) -> None:
        if table.n == 0 or _empty(box):
            return
        max_off = getattr(table, "max_off", None)
        if max_off is None:  # tables built elsewhere: one (syncing) check, then cached
            table.max_off = max_off = int(table.off.max())
            table.max_inc = int(table.i0.max()) + 1
        if max_off >= target.numel() or table.max_inc >= inc.numel():
            raise HipError("TF/SF table reads or writes outside its arrays")
        bb = getattr(table, "bbox", None)  # host-side, set where the table is built (no sync under capture)
        whole = bb is not None and all(box[0][d] <= bb[0][d] and bb[1][d] <= box[1][d] for d in range(3))
        rc = self.fn("tfsf_apply")(_ptr(target), _ptr(table.off), _ptr(table.i0), _ptr(table.w0), _ptr(table.w1),
                                   _ptr(table.coef), None if whole else _ptr(table.ijk), c_int(table.n), _ptr(inc),
                                   _box_arr([box]), _stream())
        _check(rc, "tfsf_apply")
        self.launches += 1

    def _tfsf_compact(self, table):
        """int32 offsets / line indices and folded weights (coef w0, coef w1)
        of a correction table, built once (None past 2^31 elements)."""
        cmp = getattr(table, "_compact", None)
        if cmp is None:
            if table.max_off >= 2 ** 31 - 1 or table.max_inc >= 2 ** 31 - 1:
                table._compact = False
                return None
            c = table.coef.double()
            cmp = (table.off.to(torch.int32).contiguous(), table.i0.to(torch.int32).contiguous(),
                   (c * table.w0.double()).to(self.dtype).contiguous(), (c * table.w1.double()).to(self.dtype).contiguous())
            table._compact = cmp
        return cmp or None

    def tfsf_apply_many(self, items, inc: torch.Tensor) -> None:
        """Whole-grid TF/SF corrections of several (target, table) pairs in as
        few launches as possible (generic_kernels.hip k_tfsf_apply_many, at most
        8 tables a launch, the layers of one target in successive launches, in
        order)."""
        launches = []
        for target, tab in items:
            if tab.n == 0:
                continue
            if getattr(tab, "max_off", None) is None:
                tab.max_off = int(tab.off.max())
                tab.max_inc = int(tab.i0.max()) + 1
            if tab.max_off >= target.numel() or tab.max_inc >= inc.numel():
                raise HipError("TF/SF table reads or writes outside its arrays")
            self._check_tensor(target)
            cmp = self._tfsf_compact(tab)
            if cmp is None:
                self.tfsf_apply(target, tab, inc, ((0, 0, 0), tuple(target.shape)))
                continue
            ptr = target.data_ptr()
            for L in launches:  # first fit: a launch never holds one target twice
                if len(L) < 8 and all(t.data_ptr() != ptr for t, _, _ in L):
                    L.append((target, tab, cmp))
                    break
            else:
                launches.append([(target, tab, cmp)])
        self._check_tensor(inc)
        for L in launches:
            P, N = [], []
            for target, tab, cmp in L:
                P += [target.data_ptr()] + [t.data_ptr() for t in cmp]
                N.append(int(tab.n))
            rc = self.fn("tfsf_apply_many")((c_vp * len(P))(*P), (c_int * len(N))(*N), c_int(len(L)), _ptr(inc),
                                            _stream())
            _check(rc, "tfsf_apply_many")
            self.launches += 1

    def scattered(self, f: torch.Tensor, line: torch.Tensor, geo: Sequence[float], igeo: Sequence[int]) -> torch.Tensor:
        """Scattered field of a TF/SF run in one pass (generic_kernels.hip
        k_scattered): ``geo`` = m[3] zero[3] dir[3] L[3] R[3] proj shift,
        ``igeo`` = origin[3] active-axis bits."""
        self._check_tensor(f)
        self._check_tensor(line)
        out = torch.empty_like(f)
        s = f.shape
        rc = self.fn("scattered")(_ptr(f), _ptr(out), _ptr(line), c_int(line.numel()), c_int(s[0]), c_int(s[1]),
                                  c_int(s[2]), (c_double * 17)(*geo), (c_int * 4)(*igeo), _stream())
        _check(rc, "scattered")
        self.launches += 1
        return out

    # ------------------------------------------------------ temporal blocking
    tfsf_sets_ok = True  # the blocked kernels (fp32 and fp64) apply TfsfSets corrections

    def tfsf_pass(self, einc: torch.Tensor, hinc: torch.Tensor, ce: float, ch: float, src_vals, reach: int,
                  sets, slot: int = 0, dry: bool = False) -> torch.Tensor:
        """Advance the incident line ``len(src_vals)`` steps and return the
        g table of the pass (levels x sets.ld, yee3d_tb.hip k_tfsf_pass);
        ``slot`` selects the table buffer (one per field plane).  ``dry``:
        the line stays as it is -- the pass runs on scratch copies
        (fdtd_tfsf_table_f32; hybrid passes, whose shell steps the line)."""
        T = len(src_vals)
        if not (1 <= T <= 8):
            raise HipError("tfsf_pass: 1..8 steps")
        sfx = "f32" if self.dtype == torch.float32 else "f64"
        if int(self.lib.fdtd_tfdev_size()) != 4 * sets.dev.numel():
            raise HipError("TfDev layout mismatch (%d vs %d bytes)" % (self.lib.fdtd_tfdev_size(),
                                                                       4 * sets.dev.numel()))
        need = T * max(1, sets.ld)
        tabs = sets.__dict__.setdefault("gtab", {})
        g = tabs.get(slot)
        if g is None or g.numel() < need:
            g = tabs[slot] = torch.zeros(8 * max(1, sets.ld), dtype=self.dtype, device=self.device)
        for t_ in (einc, hinc):
            self._check_tensor(t_)
        if einc.numel() != hinc.numel():
            raise HipError("tfsf_pass: E / H lines of different length")
        vals8 = (c_double * 8)(*(list(src_vals) + [0.0] * (8 - T)))
        tail = (c_int(T), c_int(min(einc.numel(), reach)), c_int(sets.n_e), c_int(sets.n_h), _ptr(sets.i0),
                _ptr(sets.w0), _ptr(sets.w1), _ptr(sets.c), _ptr(g), _stream())
        if dry:
            scr = sets.__dict__.setdefault("scratch_lines", {})
            sl = scr.get(slot)
            if sl is None or sl[0].numel() != einc.numel():
                # zero beyond every reach a pass copies: cells past the wave front read 0
                sl = scr[slot] = (torch.zeros_like(einc), torch.zeros_like(hinc))
            rc = getattr(self.lib, "fdtd_tfsf_table_" + sfx)(_ptr(einc), _ptr(hinc), _ptr(sl[0]), _ptr(sl[1]),
                                                             c_int(einc.numel()), c_double(ce), c_double(ch), vals8,
                                                             *tail)
        else:
            rc = getattr(self.lib, "fdtd_tfsf_pass_" + sfx)(_ptr(einc), _ptr(hinc), c_int(einc.numel()), c_double(ce),
                                                            c_double(ch), vals8, *tail)
        _check(rc, "tfsf_pass")
        self.launches += 1
        return g

    tb_amp_max_steps = 3  # amplitude passes: the kernel's LDS hand-off holds T - 1 levels

    def tb_amp_step(self, fin: Dict[str, torch.Tensor], fout: Dict[str, torch.Tensor], boxes: Dict[str, Box],
                    obox: Box, cb: Dict[str, Coef], steps: int, line, vals, amps: Sequence[torch.Tensor],
                    aboxes: Sequence[Box], accuracy: float, counts: torch.Tensor) -> None:
        """``steps`` (<= 3) fused leapfrog steps with the amplitude update of
        every step folded in (tb3d_mr.h AmpDev, fdtd_tb3d_amp_f32): the
        running maxima ``amps`` (Ex .. Hz, one allocation, equally spaced) of
        the cells of ``obox`` inside ``aboxes`` advance level by level, and
        ``counts[l]`` (int32, device) gets the changed cells of step l added.
        ``line`` = (E component, i, j, k0, k1) of the hard z-line source, or
        None; ``vals`` its value per step.  Uniform media only."""
        E, H = ("Ex", "Ey", "Ez"), ("Hx", "Hy", "Hz")
        if self.dtype != torch.float32 or not (1 <= steps <= self.tb_amp_max_steps):
            raise HipError("amplitude passes: fp32, 1..%d steps" % self.tb_amp_max_steps)
        shape = tuple(fin["Ex"].shape)
        if shape[2] % 4 != 0:
            raise HipError("fp32 tb_amp_step needs nz %% 4 == 0, got %s" % (shape,))
        for c in E + H:
            self._check_tensor(fin[c], shape)
            self._check_tensor(fout[c], shape)
            if fin[c].data_ptr() == fout[c].data_ptr():
                raise HipError("tb_amp_step needs distinct in/out buffers")
            if self._cell_or_none(cb[c]) is not None:
                raise HipError("tb_amp_step: uniform media only")
        for bx in list(boxes.values()) + [obox] + list(aboxes):
            for d in range(3):
                if not _empty(bx) and (bx[0][d] < 0 or bx[1][d] > shape[d]):
                    raise HipError("box %s outside array %s" % (bx, shape))
        cbv, dbv = cb["Ex"].scalar, cb["Hx"].scalar
        if any(cb[c].scalar != cbv for c in E) or any(cb[c].scalar != dbv for c in H):
            raise HipError("tb_amp_step: scalar coefficients must agree per kind")
        xs = self._check_amp(amps, shape)
        plane = shape[1] * shape[2]
        es = amps[0].element_size()
        if xs != 6 * plane or 6 * plane * es >= 2 ** 28:
            raise HipError("amplitude passes need the six arrays interleaved per x plane (x stride 6 ny nz)")
        for n, a in enumerate(amps):
            if a.data_ptr() != amps[0].data_ptr() + n * plane * es:
                raise HipError("amplitude arrays must be the planes of one [x][6][y][z] allocation")
        if counts.device.type != "cuda" or counts.dtype != torch.int32 or counts.numel() < steps:
            raise HipError("amplitude counts: %d int32 on the device" % steps)
        src = [-1, -1, -1, -1, -1]
        v8 = [0.0] * 8
        if line is not None:
            comp, i, j, k0, k1 = line
            if comp not in E or not (0 <= i < shape[0] and 0 <= j < shape[1] and 0 <= k0 <= k1 <= shape[2]):
                raise HipError("tb_amp_step: bad line source %s" % (line,))
            src = [i, j, k0, E.index(comp), k1]
            v8[:steps] = [float(v) for v in vals[:steps]]
        arr = lambda names, f: (c_vp * 3)(*[f[c].data_ptr() for c in names])
        rc = self.lib.fdtd_tb3d_amp_f32(
            arr(E, fin), arr(H, fin), arr(E, fout), arr(H, fout), c_double(cbv), c_double(dbv), c_int(shape[0]),
            c_int(shape[1]), c_int(shape[2]), _box_arr([boxes[c] for c in E + H]), _box_arr([obox]),
            c_int(self.tb_xchunk), c_int(steps), (c_int * 5)(*src), (c_double * 8)(*v8),
            (c_vp * 6)(*[a.data_ptr() for a in amps]), _box_arr(list(aboxes)), c_double(accuracy),
            c_vp(counts.data_ptr()), _stream())
        _check(rc, "tb3d_amp")
        self.launches += 1

    tb_drude_max_steps = 5  # Drude passes: the dispersive state of T - 1 levels rides in registers
    # Drude variant tiles: 0 = 8 waves x 2 rows, 1 = 16 waves x 1 row (both 16 rows)
    tb_dr_shape = int(os.environ.get("FDTD3D_TB_DR_SHAPE", "0"))

    def tb_drude_step(self, fin: Dict[str, torch.Tensor], fout: Dict[str, torch.Tensor], boxes: Dict[str, Box],
                      obox: Box, cb: Dict[str, Coef], steps: int, sources, drude: dict) -> None:
        """``steps`` (<= 5) fused leapfrog steps over ``obox`` with the Drude
        box folded in (tb3d_mr.h DrDev, fdtd_tb3d_drude_f32): inside
        ``drude["box"]`` (local) the E components take the dispersive update
        from the state ``drude["sin"]`` (two float4 arrays over the box:
        delta + material ids, E of the previous step), written advanced to
        ``drude["sout"]``; ``drude["lut"]`` = (3, nid, 4) float32 tuples
        (b0 cbd, b2, m1, m2), ``drude["cbd"]`` the D coefficient.  Uniform
        media elsewhere; ``sources`` as :meth:`tb_step`."""
        E, H = ("Ex", "Ey", "Ez"), ("Hx", "Hy", "Hz")
        if not (1 <= steps <= self.tb_drude_max_steps):
            raise HipError("Drude passes: 1..%d steps" % self.tb_drude_max_steps)
        shape = tuple(fin["Ex"].shape)
        f32 = self.dtype == torch.float32
        if f32 and shape[2] % 4 != 0:
            raise HipError("fp32 tb_drude_step needs nz %% 4 == 0, got %s" % (shape,))
        for c in E + H:
            self._check_tensor(fin[c], shape)
            self._check_tensor(fout[c], shape)
            if fin[c].data_ptr() == fout[c].data_ptr():
                raise HipError("tb_drude_step needs distinct in/out buffers")
            if self._cell_or_none(cb[c]) is not None:
                raise HipError("tb_drude_step: uniform media outside the Drude box only")
        B = drude["box"]
        for bx in list(boxes.values()) + [obox, B]:
            for d in range(3):
                if not _empty(bx) and (bx[0][d] < 0 or bx[1][d] > shape[d]):
                    raise HipError("box %s outside array %s" % (bx, shape))
        for c in E:
            b = boxes[c]
            if any(B[0][d] < b[0][d] or B[1][d] > b[1][d] for d in range(3)):
                raise HipError("Drude box %s not inside the update box %s of %s" % (B, b, c))
        bshape = tuple(B[1][d] - B[0][d] for d in range(3)) + (4,)
        for t in list(drude["sin"]) + list(drude["sout"]):
            self._check_tensor(t, bshape)
        if any(a.data_ptr() == b.data_ptr() for a in drude["sin"] for b in drude["sout"]):
            raise HipError("tb_drude_step needs distinct state in / out buffers")
        lut = drude["lut"]
        nid = int(lut.shape[1])
        self._check_tensor(lut, (3, nid, 4))
        cbv, dbv = cb["Ex"].scalar, cb["Hx"].scalar
        if any(cb[c].scalar != cbv for c in E) or any(cb[c].scalar != dbv for c in H):
            raise HipError("tb_drude_step: scalar coefficients must agree per kind")
        src = [-1, -1, -1, -1]
        vals = [0.0] * 8
        if sources is not None and any(s is not None for s in sources):
            first = next(s for s in sources if s is not None)
            comp, idx = first[0], tuple(first[1])
            if comp not in E or not all(0 <= idx[d] < shape[d] for d in range(3)):
                raise HipError("tb_drude_step: E point source inside the array only")
            for l, s in enumerate(sources):
                if s is None or s[0] != comp or tuple(s[1]) != idx:
                    raise HipError("tb_drude_step: the source must be the same point at every step")
                vals[l] = float(s[2])
            src = [idx[0], idx[1], idx[2], E.index(comp)]
        arr = lambda names, f: (c_vp * 3)(*[f[c].data_ptr() for c in names])
        two = lambda ts: (c_vp * 2)(*[t.data_ptr() for t in ts])
        if f32:
            self.lib.fdtd_set_tb_dr_shape(c_int(self.tb_dr_shape))
        rc = (self.lib.fdtd_tb3d_drude_f32 if f32 else self.lib.fdtd_tb3d_drude_f64)(
            arr(E, fin), arr(H, fin), arr(E, fout), arr(H, fout), c_double(cbv), c_double(dbv), c_int(shape[0]),
            c_int(shape[1]), c_int(shape[2]), _box_arr([boxes[c] for c in E + H]), _box_arr([obox]),
            c_int(self.tb_xchunk), c_int(steps), (c_int * 4)(*src), (c_double * 8)(*vals), _box_arr([B]),
            two(drude["sin"]), two(drude["sout"]), c_vp(lut.data_ptr()), c_int(nid), c_double(drude["cbd"]),
            _stream())
        _check(rc, "tb3d_drude")
        self.launches += 1

    def tb_step(self, fin: Dict[str, torch.Tensor], fout: Dict[str, torch.Tensor], boxes: Dict[str, Box],
                obox: Box, cb: Dict[str, Coef], steps: int, sources=None, tfsf=None) -> None:
        """``steps`` fused leapfrog steps in one HBM pass (yee3d_tb.hip).

        ``boxes`` are the update boxes (each component changes only there, at
        every inner step), ``obox`` the cells stored to ``fout``.  The kernel
        never reads outside the arrays whatever the boxes, but the caller must
        give every stored cell ``steps`` valid layers of input around it.
        ``sources`` = per-step list of (E component, local index, value) or
        None.  ``tfsf`` = (TfsfSets, g table, first level) from
        ``tfsf_pass``."""
        if len(fin) == 3:
            self._tb2d_step(fin, fout, boxes, obox, cb, steps, sources)
            return
        E, H = ("Ex", "Ey", "Ez"), ("Hx", "Hy", "Hz")
        if not (1 <= steps <= self.tb_max_steps):
            raise HipError("tb_step supports 1..%d steps per pass" % self.tb_max_steps)
        shape = tuple(fin["Ex"].shape)
        if self.dtype == torch.float32 and shape[2] % 4 != 0:
            raise HipError("fp32 tb_step needs nz %% 4 == 0, got %s" % (shape,))
        for c in E + H:
            self._check_tensor(fin[c], shape)
            self._check_tensor(fout[c], shape)
            if fin[c].data_ptr() == fout[c].data_ptr():
                raise HipError("tb_step needs distinct in/out buffers")
            b = boxes[c]
            for d in range(3):
                if not _empty(b) and (b[0][d] < 0 or b[1][d] > shape[d]):
                    raise HipError("update box %s of %s outside array %s" % (b, c, shape))
        for d in range(3):
            if obox[0][d] < 0 or obox[1][d] > shape[d]:
                raise HipError("output box %s outside array %s" % (obox, shape))
        pe = [self._cell_or_none(cb[c]) for c in E]
        ph = [self._cell_or_none(cb[c]) for c in H]
        percell = any(p is not None for p in pe + ph)
        if percell:
            cbs, cbv = self._kind_coef_args(cb, E, pe, shape)
            dbs, dbv = self._kind_coef_args(cb, H, ph, shape)
        else:
            cbs = (c_vp * 3)(None, None, None)
            dbs = (c_vp * 3)(None, None, None)
            cbv, dbv = cb["Ex"].scalar, cb["Hx"].scalar
            if any(cb[c].scalar != cbv for c in E) or any(cb[c].scalar != dbv for c in H):
                raise HipError("tb_step: scalar coefficients must agree per kind")
        src = [-1, -1, -1, -1]
        vals = [0.0] * 8
        if sources is not None and any(s is not None for s in sources):
            first = next(s for s in sources if s is not None)
            comp, idx = first[0], tuple(first[1])
            if comp not in E:
                raise HipError("tb_step supports E point sources only")
            for d in range(3):
                if not (0 <= idx[d] < shape[d]):
                    raise HipError("source index outside array")
            for l, s in enumerate(sources):
                if s is None or s[0] != comp or tuple(s[1]) != idx:
                    raise HipError("tb_step: the source must be the same point at every step")
                vals[l] = float(s[2])
            src = [idx[0], idx[1], idx[2], E.index(comp)]
        arr = lambda names, f: (c_vp * 3)(*[f[c].data_ptr() for c in names])
        if tfsf is not None and self.dtype != torch.float32:
            # fp64 kernel with the TF/SF corrections (yee3d_tb64.hip TFS)
            sets, gtab, level0 = tfsf
            if int(self.lib.fdtd_tfdev_size()) != 4 * sets.dev.numel():
                raise HipError("TfDev layout mismatch")
            self.lib.fdtd_set_tb64_shape(c_int(self.tb64_half))
            rc = self.lib.fdtd_tb3d_tf_f64(
                arr(E, fin), arr(H, fin), arr(E, fout), arr(H, fout), cbs, dbs, c_double(cbv), c_double(dbv),
                c_int(shape[0]), c_int(shape[1]), c_int(shape[2]), _box_arr([boxes[c] for c in E + H]), _box_arr([obox]),
                c_int(self.tb_xchunk), c_int(steps), (c_int * 4)(*src), (c_double * 8)(*vals), _ptr(sets.dev),
                c_vp(gtab.data_ptr() + gtab.element_size() * level0 * sets.ld), _stream())
            _check(rc, "tb3d_tf_f64")
            self.launches += 1
            return
        if (percell and self.dtype == torch.float32 and self.tb_sparse) or tfsf is not None:
            # multi-row kernel with sparse per-cell coefficients / TF/SF sets
            if percell and steps > 5:
                raise HipError("per-cell coefficients: at most 5 steps per pass")
            if percell:
                ce, ebox, cbv = self._sparse_kind(cb, E, shape)
                ch, hbox, dbv = self._sparse_kind(cb, H, shape)
            else:
                ce = ch = None
                ebox = hbox = ((0, 0, 0), (0, 0, 0))
            tfp = gp = None
            if tfsf is not None:
                sets, gtab, level0 = tfsf
                tfp = _ptr(sets.dev)
                gp = c_vp(gtab.data_ptr() + 4 * level0 * sets.ld)
            rc = self.lib.fdtd_tb3d_ext_f32(
                arr(E, fin), arr(H, fin), arr(E, fout), arr(H, fout), _ptr(ce), _box_arr([ebox]), _ptr(ch),
                _box_arr([hbox]), c_double(cbv), c_double(dbv), c_int(shape[0]), c_int(shape[1]), c_int(shape[2]),
                _box_arr([boxes[c] for c in E + H]), _box_arr([obox]), c_int(self.tb_xchunk), c_int(steps),
                (c_int * 4)(*src), (c_double * 8)(*vals), tfp, gp, _stream())
            _check(rc, "tb3d_ext")
            self.launches += 1
            return
        if self.dtype == torch.float32:
            self.lib.fdtd_set_tb_vec(c_int(self.tb_vec))
            self.lib.fdtd_set_tb_rows(c_int(self.tb_rows))
            self.lib.fdtd_set_tb_xcd(c_int(self.tb_xcd))
            mr = self.tb_mrows
            mr_shape = self.tb_mr_shape
            if mr == 0 and self.tb_thin_single_row and steps <= 4 and obox[1][1] - obox[0][1] <= 8:
                # thin y shells of a decomposed pass: 16-row tiles waste half
                # as many rows as the 32-row multi-row tiles -- the single-row
                # kernel's, or the multi-row kernel's 8-wave form (tb_thin_mr16)
                if self.tb_thin_mr16:
                    mr_shape = 2
                else:
                    mr = 1
            self.lib.fdtd_set_tb_mrows(c_int(mr))
            self.lib.fdtd_set_tb_variant(c_int(self.tb_variant))
            self.lib.fdtd_set_tb_mr_shape(c_int(mr_shape))
        else:
            self.lib.fdtd_set_tb64_shape(c_int(self.tb64_half))
        # fp32: yee3d_tb.hip (multi-row / single-row tiles); fp64: yee3d_tb64.hip
        rc = self.fn("tb3d_v4" if self.dtype == torch.float32 else "tb3d")(arr(E, fin), arr(H, fin), arr(E, fout), arr(H, fout), cbs, dbs, c_double(cbv),
                                c_double(dbv), c_int(shape[0]), c_int(shape[1]), c_int(shape[2]),
                                _box_arr([boxes[c] for c in E + H]), _box_arr([obox]), c_int(self.tb_xchunk),
                                c_int(steps), (c_int * 4)(*src), (c_double * 8)(*vals), _stream())
        _check(rc, "tb3d")
        self.launches += 1

    def _tb2d_step(self, fin, fout, boxes, obox, cb, steps, sources) -> None:
        """2D (TMz / TEz) blocked pass (yee2d_tb.hip): (nx, ny, 1) arrays
        whose rows are whole 16-byte lanes (ny % 4 == 0 fp32, % 2 fp64); the
        point source may sit on any of the three components (TEz's reference
        source is on Hz)."""
        ecomps = tuple(c for c in ("Ex", "Ey", "Ez") if c in fin)
        if ecomps not in TB2D_MODES:
            raise HipError("2D tb_step: TMz (Ez, Hx, Hy) or TEz (Ex, Ey, Hz) only")
        mode, E, H = TB2D_MODES[ecomps]
        comps = E + H
        if not (1 <= steps <= self.tb2d_max_steps):
            raise HipError("2D tb_step supports 1..%d steps per pass" % self.tb2d_max_steps)
        shape = tuple(fin[comps[0]].shape)
        vec = 16 // self.dtype.itemsize
        if len(shape) != 3 or shape[2] != 1 or shape[1] % vec != 0:
            raise HipError("2D tb_step needs (nx, ny, 1) arrays with ny %% %d == 0, got %s" % (vec, shape))
        for c in comps:
            self._check_tensor(fin[c], shape)
            self._check_tensor(fout[c], shape)
            if fin[c].data_ptr() == fout[c].data_ptr():
                raise HipError("tb_step needs distinct in/out buffers")
            b = boxes[c]
            for d in range(2):
                if not _empty(b) and (b[0][d] < 0 or b[1][d] > shape[d]):
                    raise HipError("update box %s of %s outside array %s" % (b, c, shape))
        for d in range(2):
            if obox[0][d] < 0 or obox[1][d] > shape[d]:
                raise HipError("output box %s outside array %s" % (obox, shape))
        # per kind: per-cell arrays when any component of the kind has them,
        # else null pointers and the kind's scalar (no constant planes streamed)
        ptrs, sv = [], {}
        for kind, names in (("E", E), ("H", H)):
            if any(self._cell_or_none(cb[c]) is not None for c in names):
                ptrs += [self._cell_array(cb[c], shape).data_ptr() for c in names]
                sv[kind] = 1.0
            else:
                ptrs += [None] * len(names)
                sv[kind] = cb[names[0]].scalar
                if any(cb[c].scalar != sv[kind] for c in names):
                    raise HipError("tb_step: scalar coefficients must agree per kind")
        cs = (c_vp * 3)(*ptrs)
        cbv, dbv = sv["E"], sv["H"]
        src = [-1, -1, -1]
        vals = [0.0] * 8
        if sources is not None and any(s is not None for s in sources):
            first = next(s for s in sources if s is not None)
            comp, idx = first[0], tuple(first[1])
            if comp not in comps:
                raise HipError("2D tb_step: source component %s not in %s" % (comp, comps))
            if not (0 <= idx[0] < shape[0] and 0 <= idx[1] < shape[1]):
                raise HipError("source index outside array")
            for l, s in enumerate(sources):
                if s is None or s[0] != comp or tuple(s[1]) != idx:
                    raise HipError("tb_step: the source must be the same point at every step")
                vals[l] = float(s[2])
            src = [idx[0], idx[1], comps.index(comp)]
        two = lambda names, f: (c_vp * 2)(*([f[c].data_ptr() for c in names] + [None] * (2 - len(names))))
        rc = self.fn("tb2d")(c_int(mode), two(E, fin), two(H, fin), two(E, fout), two(H, fout), cs,
                                    c_double(cbv), c_double(dbv), c_int(shape[0]), c_int(shape[1]),
                                    _box_arr([boxes[c] for c in comps]), _box_arr([obox]), c_int(self.tb_xchunk),
                                    c_int(steps), (c_int * 3)(*src), (c_double * 8)(*vals), _stream())
        _check(rc, "tb2d")
        self.launches += 1

    @property
    def tb2d_max_steps(self) -> int:
        return TB2D_MAX_STEPS if self.dtype == torch.float32 else TB2D_MAX_STEPS_F64

    @property
    def tb_max_steps(self) -> int:
        return TB_MAX_STEPS if self.dtype == torch.float32 else TB_MAX_STEPS_F64

    tb_xchunk = int(os.environ.get("FDTD3D_TB_XCHUNK", "0"))  # x planes per blocked workgroup: 0 automatic
    tb_vec = 0  # lane width of the blocked kernel: 0 auto (4 for T <= 2, 2 above), 2 or 4
    tb_rows = 0  # grid rows per wave: 0 auto (1), 1 or 2
    tb_xcd = 0  # XCD-aware tile order (off: measured no gain)
    tb_variant = 4  # multi-row kernel: bit 0 deferred stores, bit 1 two planes prefetched, bit 2 XCD tile order
    tb_mrows = 0  # adjacent y rows per wave (multi-row kernel): 0 auto, 1 single-row kernel, 2
    tb_thin_single_row = True  # auto mode: output boxes <= 8 rows in y use 16-row tiles
    tb_thin_mr16 = os.environ.get("FDTD3D_TB_THIN_MR16", "0") == "1"  # ... of the multi-row kernel (else single-row)
    tb_sparse = True  # per-cell fp32 coefficients: sparse float4 boxes on the multi-row kernel
    # plain multi-row tile shape: 0 = 16 waves x 2 rows, 1 = 8 waves x 4 rows (two workgroups per CU)
    tb_mr_shape = int(os.environ.get("FDTD3D_TB_MR_SHAPE", "0"))
    # fp64 tiles: 1 = two rows of 32 z lanes per wave (32 x 32), 0 = one row of 64 (16 x 64)
    tb64_half = int(os.environ.get("FDTD3D_TB64_HALF", "1"))

    # ------------------------------------------------------------ UPML chain
    def chain_update(self, kind: str, boxes: Dict[str, Box], F: Dict[str, torch.Tensor], upml: Dict[str, dict],
                     p: int, drude: bool, plain_form: bool = False, plain: Optional[Dict[str, Box]] = None,
                     cb: Optional[Dict[str, Coef]] = None, rows=None) -> None:
        """Fused UPML/Drude chain (chain_kernels.hip) of the three components
        of a kind (one launch).  ``upml[c]`` holds the factored coefficient
        profiles (``prof``), the Drude cell coefficients and the D / D1 level
        lists of scheme._init_upml; new levels go to the last list entry.
        ``rows`` (dispersive launches on sigma = 0 boxes): ``(table, lo0, lo1)``
        with ``table`` int32 ``(nx, ny, 2)`` = per local row (x, y) the z range
        of the dispersive cells; the rest of the box takes the plain update
        with ``cb`` (the plain scheme's coefficients)."""
        if rows is not None and (not drude or cb is None):
            raise HipError("chain_update rows: dispersive launches with the plain coefficients only")
        comps = list(boxes.keys())
        if len(comps) != 3:
            raise HipError("chain_update launches the three components of a kind together")
        shape = tuple(F[comps[0]].shape)
        P, S, I = [], [], []
        any_box = False
        for c in comps:
            st = upml[c]
            pr = st["plain"]["prof"] if plain_form else st["prof"]
            b = boxes[c]
            terms = self.layout.curl_terms(c)
            if len(terms) != 2:
                raise HipError("chain_update is the 3D chain (2 curl terms per component)")
            if not _empty(b):
                any_box = True
                self._check_stencil_box(kind, c, b, shape)
            D = st["D"][p]
            aux = [D[-1], D[0], D[1] if drude else None]
            if drude:
                D1 = st["D1"][p]
                aux += [D1[2], D1[0], D1[1]]
            else:
                aux += [None, None, None]
            dbox = ((0, 0, 0), (0, 0, 0))
            if isinstance(D[0], RegionLevel):
                # region-local levels (models/regions.py): the parts holding this launch's box
                parts = [None if t is None else t.part(b) for t in aux]
                boxes_ = {pt[1] for pt in parts if pt is not None and pt[0] is not None}
                if len(boxes_) > 1:
                    raise HipError("chain_update: D / D1 parts of %s in different storage boxes" % c)
                dbox = boxes_.pop() if boxes_ else dbox
                aux = [None if pt is None else pt[0] for pt in parts]
                dshape = tuple(dbox[1][d] - dbox[0][d] for d in range(3))
                for t in aux:
                    if t is not None:
                        self._check_tensor(t, dshape)
            else:
                for t in aux:
                    if t is not None:
                        self._check_tensor(t, shape)
            fields = [F[c]] + aux + [F[terms[0][0]], F[terms[1][0]]]
            for t in (F[c], F[terms[0][0]], F[terms[1][0]]):
                self._check_tensor(t, shape)
            aD, aA, aB = pr["axes"]
            profs = [pr["caD"], pr["cbD"], pr["caE"], pr["ica"], pr["cbEa"], pr["ccEa"]]
            for t, a in zip(profs, (aD, aD, aA, aA, aB, aB)):
                self._check_tensor(t, (shape[a],))
            cell = pr["cell"]
            if cell is not None:
                self._check_tensor(cell, shape)
            dr = [None] * 5
            lut = (None, None)
            if drude:
                pre = st.get("_drude_lut")
                if self.drude_lut and pre is not None and pre[0] is not None:
                    # built at initialisation (scheme._init_upml): index + table only
                    lut = pre
                    ids, tab = lut
                    if (ids.device.type != "cuda" or ids.dtype != torch.uint8 or tuple(ids.shape) != shape
                            or not ids.is_contiguous() or tab.dtype != self.dtype or tab.dim() != 2
                            or tab.shape[1] != 5 or tab.device.type != "cuda"):
                        raise HipError("Drude index / table of %s malformed" % c)
                else:
                    dr = [st[n].cell for n in ("b0", "b1", "b2", "ma1", "ma2")]
                    for n, t in zip(("b0", "b1", "b2", "ma1", "ma2"), dr):
                        if st[n].scalar != 1.0 or t is None:
                            raise HipError("Drude coefficient %s must be a plain per-cell array" % n)
                        self._check_tensor(t, shape)
                    if self.drude_lut:
                        lut = self._drude_lut(st, dr, shape)
            # plain Yee cells folded into the launch (F += c curl; c scalar or scaled per cell)
            pb = plain.get(c, ((0, 0, 0), (0, 0, 0))) if plain else ((0, 0, 0), (0, 0, 0))
            pcell, pcb = None, 1.0
            if not _empty(pb) or rows is not None:
                if not _empty(pb):
                    any_box = True
                    self._check_stencil_box(kind, c, pb, shape)
                if self._cell_or_none(cb[c]) is not None:
                    pcell = self._scaled_cell(cb[c])
                else:
                    pcb = float(cb[c].scalar)
            P += [None if t is None else t.data_ptr() for t in fields + profs + [cell] + dr + list(lut) + [pcell]]
            S += [float(pr["s"]), pcb]
            I += ([terms[0][1], terms[1][1], terms[0][2], terms[1][2], aD, aA, aB] + list(b[0]) + list(b[1])
                  + list(pb[0]) + list(pb[1]) + list(dbox[0]) + list(dbox[1]))
        if not any_box:
            return
        if rows is not None:
            tab, lo0, lo1 = rows
            if (tab.device.type != "cuda" or tab.dtype != torch.int32 or not tab.is_contiguous() or tab.dim() != 3
                    or tab.shape[2] != 2):
                raise HipError("chain_update rows: contiguous int32 (nx, ny, 2) device table expected")
            R = (c_int * 4)(int(lo0), int(lo1), int(tab.shape[0]), int(tab.shape[1]))
            rc = self.fn("chain3d_rows")((c_vp * len(P))(*P), (c_double * len(S))(*S), (c_int * len(I))(*I),
                                         c_int(1 if kind == "E" else 0), c_int(shape[1]), c_int(shape[2]),
                                         c_vp(tab.data_ptr()), R, _stream())
            _check(rc, "chain3d_rows")
            self.launches += 1
            return
        rc = self.fn("chain3d")((c_vp * len(P))(*P), (c_double * len(S))(*S), (c_int * len(I))(*I),
                                c_int(1 if drude else 0), c_int(1 if kind == "E" else 0), c_int(shape[1]),
                                c_int(shape[2]), _stream())
        _check(rc, "chain3d")
        self.launches += 1

    chain_rows = True  # dispersive chain launches on sigma = 0 boxes: chain inside the per-row material range only
    drude_lut = True  # Drude chain: uint8 material index + coefficient table (falls back past 256 tuples)
    chain_fold = True  # thin plain boxes next to a z PML slab ride in the slab's chain launch
    region_aux = True  # chain launches address region-local D / D1 levels (models/regions.py)

    def _drude_lut(self, st: dict, dr, shape):
        """(uint8 id array, (n, 5) table) of a component's five Drude
        coefficient arrays, built once per component (None, None when the
        arrays hold more than 256 distinct tuples)."""
        got = st.get("_drude_lut")
        if got is None:
            M = torch.stack([t.reshape(-1) for t in dr], 1)
            tab, inv = torch.unique(M, dim=0, return_inverse=True)
            if tab.shape[0] <= 256:
                got = (inv.to(torch.uint8).reshape(shape).contiguous(), tab.contiguous())
            else:
                got = (None, None)
            del M, inv
            st["_drude_lut"] = got
        return got

    # ------------------------------------------------------------ fused CPML
    def fused_cpml_ok(self, scheme) -> bool:
        # fp32 float4 / fp64 double4 lanes of 4 z cells (yee3d_cpml.hip)
        return (self.vec4 and self.dtype in (torch.float32, torch.float64) and scheme.cfg.scheme == "3d"
                and scheme.domain.shape[2] % 4 == 0)

    def curl_update_cpml(self, kind: str, boxes: Dict[str, Box], dst: Dict[str, torch.Tensor],
                         src: Dict[str, torch.Tensor], cb: Dict[str, Coef], table) -> None:
        """Plain 3D half step with the CPML convolution terms folded in
        (yee3d_cpml.hip).  ``table`` = CPML.kernel_table(kind, plane)."""
        names = ("Ex", "Ey", "Ez") if kind == "E" else ("Hx", "Hy", "Hz")
        other = ("Hx", "Hy", "Hz") if kind == "E" else ("Ex", "Ey", "Ez")
        shape = tuple(dst[names[0]].shape)
        for c in names:
            self._check_tensor(dst[c], shape)
            if not _empty(boxes[c]):
                self._check_stencil_box(kind, c, boxes[c], shape)
        for c in other:
            self._check_tensor(src[c], shape)
        if shape[2] % 4 != 0 or self.dtype not in (torch.float32, torch.float64):
            raise HipError("fused CPML kernel needs fp32 / fp64 and nz % 4 == 0")
        per = [self._cell_or_none(cb[c]) for c in names]
        if per[0] is not None:
            per_p = [_ptr(self._scaled_cell(cb[c])) for c in names]
            scal = 1.0
        else:
            per_p = [None, None, None]
            scal = cb[names[0]].scalar
            if any(cb[c].scalar != scal for c in names):
                raise HipError("scalar coefficients must agree across components")
        ptrs, ints, _keep = table
        fn = self.fn("update_e3d_cpml_v4" if kind == "E" else "update_h3d_cpml_v4")
        rc = fn(*[_ptr(dst[c]) for c in names], *[_ptr(src[c]) for c in other], *per_p, c_double(scal),
                c_int(shape[0]), c_int(shape[1]), c_int(shape[2]), _box_arr([boxes[c] for c in names]),
                c_int(self.xchunk), (c_vp * len(ptrs))(*ptrs), (c_int * len(ints))(*ints), _stream())
        _check(rc, "update_%s3d_cpml" % kind.lower())
        self.launches += 1

    def curl_update_cpml_multi(self, kind: str, windows: Sequence[Dict[str, Box]], dst: Dict[str, torch.Tensor],
                               src: Dict[str, torch.Tensor], cb: Dict[str, Coef], table) -> None:
        """:meth:`curl_update_cpml` of several disjoint windows (per window the
        component boxes) in one launch per row layout (yee3d_cpml.hip
        ``Win3``, <= 8 windows a launch): the hybrid shell's windows of a half
        step."""
        names = ("Ex", "Ey", "Ez") if kind == "E" else ("Hx", "Hy", "Hz")
        other = ("Hx", "Hy", "Hz") if kind == "E" else ("Ex", "Ey", "Ez")
        shape = tuple(dst[names[0]].shape)
        for c in names:
            self._check_tensor(dst[c], shape)
        for c in other:
            self._check_tensor(src[c], shape)
        if shape[2] % 4 != 0 or self.dtype not in (torch.float32, torch.float64):
            raise HipError("fused CPML kernel needs fp32 / fp64 and nz % 4 == 0")
        wins = [w for w in windows if not all(_empty(w[c]) for c in names)]
        for w in wins:
            for c in names:
                if not _empty(w[c]):
                    self._check_stencil_box(kind, c, w[c], shape)
        if not wins:
            return
        per = [self._cell_or_none(cb[c]) for c in names]
        if per[0] is not None:
            per_p = [_ptr(self._scaled_cell(cb[c])) for c in names]
            scal = 1.0
        else:
            per_p = [None, None, None]
            scal = cb[names[0]].scalar
            if any(cb[c].scalar != scal for c in names):
                raise HipError("scalar coefficients must agree across components")
        ptrs, ints, _keep = table
        fn = self.fn("update_e3d_cpml_multi" if kind == "E" else "update_h3d_cpml_multi")
        rc = fn(*[_ptr(dst[c]) for c in names], *[_ptr(src[c]) for c in other], *per_p, c_double(scal),
                c_int(shape[0]), c_int(shape[1]), c_int(shape[2]), _box_arr([w[c] for w in wins for c in names]),
                c_int(len(wins)), (c_vp * len(ptrs))(*ptrs), (c_int * len(ints))(*ints), _stream())
        _check(rc, "update_%s3d_cpml_multi" % kind.lower())
        self.launches += 1

    # ------------------------------------------------------------ HIP graphs
    def set_value_tab(self, t: torch.Tensor, idx: Sequence[int], tab: torch.Tensor, counter: torch.Tensor,
                      lag: int) -> None:
        """Hard source whose value is ``tab[counter + lag]`` (device table and
        step counter): replayable inside a captured HIP graph."""
        s = t.shape
        for d in range(3):
            if not (0 <= idx[d] < s[d]):
                raise HipError("source index %s outside %s" % (idx, tuple(s)))
        if tab.dtype != torch.float64 or counter.dtype != torch.int32:
            raise HipError("source table must be float64 and the counter int32")
        off = (idx[0] * s[1] + idx[1]) * s[2] + idx[2]
        _check(self.fn("set_value_tab")(_ptr(t), c_ll(off), _ptr(tab), _ptr(counter), c_int(lag), _stream()),
               "set_value_tab")
        self.launches += 1

    def inc_step_e_tab(self, einc: torch.Tensor, hinc: torch.Tensor, coef: float, tab: torch.Tensor,
                       counter: torch.Tensor, lag: int) -> None:
        _check(self.fn("inc_e_tab")(_ptr(einc), _ptr(hinc), c_int(einc.numel()), c_double(coef), _ptr(tab),
                                    _ptr(counter), c_int(lag), _stream()), "inc_e_tab")

    def counter_add(self, counter: torch.Tensor, n: int) -> None:
        _check(self.lib.fdtd_counter_add(_ptr(counter), c_int(n), _stream()), "counter_add")
