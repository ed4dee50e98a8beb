"""Region-local UPML state for the single-pass hybrid shell.

The reference stores the UPML auxiliary D (B) field of every component on
every cell of the grid (``Scheme3D.cpp:3413-4032`` allocates all 27 grids)
and runs the three-sweep D/B update everywhere (``Scheme3D.cpp:266-416``).
The auxiliary only carries information where some sigma is non-zero: here it
lives in the six disjoint boxes of ``alloc - I``, ``I`` = the cells where
every component's sigma vanishes (x slabs over the whole y / z extent, y slabs
over I's x range, z slabs over I's x / y ranges -- ``box_subtract`` order),
two copies per component (the shell kernel reads D^n from one and writes
D^{n+1} to the other, because tiles recompute their neighbours' halo cells).
At 1024^3 with 10-cell layers that is 61 M cells per copy instead of 1.07 G.

Each component's six UPML profiles are passed as (a, b) pairs per axis --
(caD, cbD) along aD, (caE, ica) along aCa, (cbEa, ccEa) along aCb -- the
factored form ``models/scheme.py _init_upml`` builds for the chain kernels.
"""

from __future__ import annotations

import struct
from typing import Dict, List, Tuple

import torch

from ..layout.yee import UPML_AXES
from ..parallel.domain import box_empty, box_intersect, box_subtract

Box = Tuple[Tuple[int, int, int], Tuple[int, int, int]]


class UPMLRegions:
    def __init__(self, scheme):
        self.s = scheme
        dom = scheme.domain
        I = None
        for c in scheme.comps:
            z = dom.to_local(scheme._chain_sigma0[c])
            I = z if I is None else box_intersect(I, z)
        alloc = ((0, 0, 0), tuple(dom.shape))
        if I is None or box_empty(I):
            raise ValueError("UPML regions: no cell where every sigma vanishes")
        self.core: Box = I
        self.boxes: List[Box] = box_subtract(alloc, I)
        dev, dt = scheme.device, scheme.dtype
        shp = lambda b: tuple(max(0, b[1][d] - b[0][d]) for d in range(3))
        # D[p][c] = [copy 0 boxes, copy 1 boxes]; copy `cur[p]` holds D^n
        self.D: List[Dict[str, List[List[torch.Tensor]]]] = [
            {c: [[torch.zeros(shp(b), dtype=dt, device=dev) for b in self.boxes] for _ in range(2)]
             for c in scheme.comps} for _ in range(scheme.planes)]
        self.cur = [0] * scheme.planes
        self.pairs: Dict[str, List[torch.Tensor]] = {}
        self.scal: Dict[str, float] = {}
        for c in scheme.comps:
            st = scheme.upml[c]
            # with dispersion the slabs run the non-dispersive chain form
            pr = st["plain"]["prof"] if "plain" in st else st["prof"]
            if pr["cell"] is not None:
                raise ValueError("UPML regions: per-cell material coefficients are not supported")
            aD, aA, aB = pr["axes"]
            assert (aD, aA, aB) == UPML_AXES[c]
            by_axis = {aD: (pr["caD"], pr["cbD"]), aA: (pr["caE"], pr["ica"]), aB: (pr["cbEa"], pr["ccEa"])}
            self.pairs[c] = [torch.stack([by_axis[a][0], by_axis[a][1]], 1).to(dt).contiguous() for a in range(3)]
            self.scal[c] = float(pr["s"])

    def cells(self) -> int:
        n = 0
        for b in self.boxes:
            if not box_empty(b):
                n += (b[1][0] - b[0][0]) * (b[1][1] - b[0][1]) * (b[1][2] - b[0][2])
        return n

    # ------------------------------------------------------------- kernel
    def host_table(self, p: int) -> torch.Tensor:
        """ShUpml block (csrc/yee3d_shell.hip) of plane ``p`` as host bytes
        (the kernel takes it by value): boxes, D^n / D^{n+1} pointers per
        (component, box), profile pairs, scalars."""
        s = self.s
        rd, wr = self.cur[p], 1 - self.cur[p]
        key = (p, rd)
        cache = self.__dict__.setdefault("_dev", {})
        if key in cache:
            return cache[key]
        ints = []
        for b in self.boxes:
            ints += list(b[0])
        for b in self.boxes:
            ints += list(b[1])
        comps = list(s.comps)
        ptr = lambda t: t.data_ptr() if t.numel() else 0
        d = [ptr(self.D[p][c][rd][q]) for c in comps for q in range(6)]
        dn = [ptr(self.D[p][c][wr][q]) for c in comps for q in range(6)]
        pr = [self.pairs[c][a].data_ptr() for c in comps for a in range(3)]
        raw = struct.pack("<36i", *ints) + struct.pack("<%dQ" % (36 + 36 + 18), *(d + dn + pr))
        raw += struct.pack("<6fi", *[self.scal[c] for c in comps], 0)
        raw += b"\0" * ((-len(raw)) % 8)
        host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
        cache[key] = host
        return host

    def shell_arg(self, p: int, ops):
        return self.host_table(p) if ops.name == "hip" else (self, p)

    def flip(self, p: int) -> None:
        self.cur[p] = 1 - self.cur[p]

    # ---------------------------------------------------------- state
    def named(self, p: int, sfx: str) -> Dict[str, torch.Tensor]:
        out = {}
        for c in self.s.comps:
            for q, t in enumerate(self.D[p][c][self.cur[p]]):
                if t.numel():
                    out["%s%s-upml-box%d%s" % ("D" if c[0] == "E" else "B", c[1], q, sfx)] = t
        return out


class DrudeBox:
    """Region-local dispersive (Drude / Lorentz) state of the single-pass
    shell (csrc/yee3d_shell.hip, the dispersive-box class): the bounding box
    ``box`` (local) of every component's dispersive cells -- inside the
    all-sigma-zero core, so the chain's profiles are scalars there -- and per
    component with dispersion three D and three D1 levels over the box (cur,
    prev, next; the reference keeps both on every cell of the grid,
    ``Scheme3D.cpp:3830-4032``), a uint8 material index + 1 (0 = the cell
    lies outside its kind's per-row material range or outside the
    component's own dispersive box and takes the plain update, exactly the
    stepped chain's split, ``models/scheme.py _drude_rows``) and the
    (b0, b1, b2, ma1, ma2) table of the distinct coefficient tuples."""

    MAX_LUT = 16

    def __init__(self, scheme):
        self.s = scheme
        dom = scheme.domain
        boxes = {}
        for c in scheme.comps:
            a = scheme.upml[c].get("drude_active")
            b = dom.to_local(scheme._bbox_global(a)) if a is not None else None
            if b is not None and not box_empty(b):
                boxes[c] = b
        if not boxes:
            raise ValueError("dispersive box: no dispersive cell")
        B = None
        for b in boxes.values():
            B = b if B is None else (tuple(min(B[0][d], b[0][d]) for d in range(3)),
                                     tuple(max(B[1][d], b[1][d]) for d in range(3)))
        self.box: Box = B
        shp = tuple(B[1][d] - B[0][d] for d in range(3))
        sl = tuple(slice(B[0][d], B[1][d]) for d in range(3))
        dev, dt = scheme.device, scheme.dtype
        self.ids: Dict[str, torch.Tensor] = {}
        self.lut: Dict[str, torch.Tensor] = {}
        self.scal: Dict[str, Tuple[float, ...]] = {}
        self.D: List[Dict[str, List[torch.Tensor]]] = [{} for _ in range(scheme.planes)]
        self.D1: List[Dict[str, List[torch.Tensor]]] = [{} for _ in range(scheme.planes)]
        in_range = {}
        for kind in ("E", "H"):
            rows = scheme._drude_rows(kind)
            if rows is None:
                continue
            tab, x0, y0 = rows
            X = torch.arange(B[0][0], B[1][0], device=tab.device) - x0
            Y = torch.arange(B[0][1], B[1][1], device=tab.device) - y0
            okx = (X >= 0) & (X < tab.shape[0])
            oky = (Y >= 0) & (Y < tab.shape[1])
            r = tab[X.clamp(0, tab.shape[0] - 1)][:, Y.clamp(0, tab.shape[1] - 1)]
            Z = torch.arange(B[0][2], B[1][2], device=tab.device)[None, None, :]
            in_range[kind] = ((okx[:, None] & oky[None, :])[..., None] & (Z >= r[..., 0:1]) & (Z < r[..., 1:2]))
        for c in scheme.comps:
            st = scheme.upml[c]
            if c not in boxes or c[0] not in in_range:
                continue
            own = torch.zeros(shp, dtype=torch.bool, device=dev)
            cb_ = boxes[c]
            own[tuple(slice(cb_[0][d] - B[0][d], cb_[1][d] - B[0][d]) for d in range(3))] = True
            use = own & in_range[c[0]].to(dev)
            scheme._drude_cells(c)
            M = torch.stack([st[n].cell[sl].reshape(-1) for n in ("b0", "b1", "b2", "ma1", "ma2")], 1)
            tab, inv = torch.unique(M, dim=0, return_inverse=True)
            if tab.shape[0] > self.MAX_LUT:
                raise ValueError("dispersive box: %d coefficient tuples (at most %d)" % (tab.shape[0], self.MAX_LUT))
            ids = torch.where(use.reshape(-1), inv + 1, torch.zeros_like(inv)).to(torch.uint8).reshape(shp)
            self.ids[c] = ids.contiguous()
            self.lut[c] = tab.to(dt).contiguous()
            pr = st["prof"]
            if pr["cell"] is not None:
                raise ValueError("dispersive box: per-cell material coefficients are not supported")
            aD, aA, aB = pr["axes"]

            def const(arr, a):
                v = arr[B[0][a]:B[1][a]]
                if not bool((v == v[0]).all()):
                    raise ValueError("dispersive box reaches an absorbing layer")
                return float(v[0])

            self.scal[c] = (const(pr["caD"], aD), const(pr["cbD"], aD), const(pr["caE"], aA),
                            float(pr["s"]) * const(pr["ica"], aA), const(pr["cbEa"], aB), const(pr["ccEa"], aB))
            for p in range(scheme.planes):
                self.D[p][c] = [torch.zeros(shp, dtype=dt, device=dev) for _ in range(3)]
                self.D1[p][c] = [torch.zeros(shp, dtype=dt, device=dev) for _ in range(3)]

    def cells(self) -> int:
        b = self.box
        return (b[1][0] - b[0][0]) * (b[1][1] - b[0][1]) * (b[1][2] - b[0][2])

    def host_table(self, p: int) -> torch.Tensor:
        """ShDrude block (csrc/yee3d_shell.hip) of plane ``p``, host bytes."""
        s = self.s
        comps = list(s.comps)
        key = (p,) + tuple(self.D[p][c][0].data_ptr() for c in comps if c in self.D[p])
        cache = self.__dict__.setdefault("_dev", {})
        if key in cache:
            return cache[key]
        B = self.box
        ints = list(B[0]) + list(B[1])
        ptr = []
        for arrs in (self.D[p], self.D1[p]):
            for c in comps:
                ptr += [t.data_ptr() for t in arrs[c]] if c in arrs else [0, 0, 0]
        ptr += [self.ids[c].data_ptr() if c in self.ids else 0 for c in comps]
        ptr += [self.lut[c].data_ptr() if c in self.lut else 0 for c in comps]
        fl = []
        for q in range(6):
            fl += [self.scal[c][q] if c in self.scal else 0.0 for c in comps]
        nl = [int(self.lut[c].shape[0]) if c in self.lut else 0 for c in comps]
        raw = struct.pack("<6i", *ints) + struct.pack("<48Q", *ptr) + struct.pack("<36f", *fl)
        raw += struct.pack("<6i", *nl)
        host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
        cache[key] = host
        return host

    def shell_arg(self, p: int, ops):
        return self.host_table(p) if ops.name == "hip" else (self, p)

    def rotate(self, p: int) -> None:
        """next -> cur -> prev (the stepped chain's level rotation)."""
        for arrs in (self.D[p], self.D1[p]):
            for c, L in arrs.items():
                L[0], L[1], L[2] = L[2], L[0], L[1]

    def named(self, p: int, sfx: str) -> Dict[str, torch.Tensor]:
        out = {}
        for c in self.s.comps:
            if c not in self.D[p]:
                continue
            k = "D" if c[0] == "E" else "B"
            for lv in range(2):
                out["%s%s-disp-lv%d%s" % (k, c[1], lv, sfx)] = self.D[p][c][lv]
                out["%s1%s-disp-lv%d%s" % (k, c[1], lv, sfx)] = self.D1[p][c][lv]
        return out
