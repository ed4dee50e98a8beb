"""Reference backend: every solver operation as vectorised torch ops.

This is the CPU oracle of the framework: it runs on
any torch device, is used by the CPU test-suite and is the numerics reference
the HIP kernels are compared against.  It implements exactly the same operation
interface as :class:`fdtd3d_amd.ops.hip_ops.HipOps`.

Operation semantics (shared by both backends):

* ``curl_update(kind, boxes, dst, src, cb)`` -- fast path
  ``dst[c] += cb[c] * curl(src)[c]`` on each component's local box.  ``curl``
  follows :data:`fdtd3d_amd.layout.yee.CURL_TERMS` (reference ``Kernels.h``).
* ``curl_general(kind, comp, box, out, inp, src, ca, cb)`` --
  ``out = ca*inp + cb*curl(src)`` (UPML D/B update, ``Scheme3D.cpp:266-324``).
* ``lincomb(out, box, terms)`` -- ``out = sum coef_i * x_i`` (Drude ADE and
  E-from-D, ``Kernels.h:80-107``).
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..layout.yee import UPML_AXES, YeeLayout
from ..models.regions import RegionLevel
from .coef import Coef

Box = Tuple[Tuple[int, int, int], Tuple[int, int, int]]


def box_slices(box: Box) -> Tuple[slice, slice, slice]:
    return tuple(slice(box[0][d], box[1][d]) for d in range(3))


def _shift(sl, axis, off):
    s = list(sl)
    s[axis] = slice(sl[axis].start + off, sl[axis].stop + off)
    return tuple(s)


def _empty(box: Box) -> bool:
    return any(box[1][d] <= box[0][d] for d in range(3))


def box_intersect_(a: Box, b: Box) -> Box:
    return (tuple(max(a[0][d], b[0][d]) for d in range(3)), tuple(min(a[1][d], b[1][d]) for d in range(3)))


def cb_pad(cb: Dict[str, Coef]) -> Dict[str, Coef]:
    """Coefficients re-indexed for fields padded by one zero layer per side."""
    def p1(t):
        return None if t is None else torch.nn.functional.pad(t, (1, 1))

    def p3(t):
        return None if t is None else torch.nn.functional.pad(t, (1, 1, 1, 1, 1, 1))
    return {c: Coef(k.scalar, p1(k.px), p1(k.py), p1(k.pz), p3(k.cell)) for c, k in cb.items()}


class TorchOps:
    name = "torch"
    chain_rows = True  # same launch plan as the HIP backend (row-range dispersive split)
    region_aux = True  # chain_update addresses region-local D / D1 levels (models/regions.py)

    def __init__(self, layout: YeeLayout, device, dtype):
        self.layout = layout
        self.device = torch.device(device)
        self.dtype = dtype

    # ------------------------------------------------------------------ curl
    def curl(self, kind: str, comp: str, sl, src: Dict[str, torch.Tensor]):
        acc = None
        for (s, axis, sign) in self.layout.curl_terms(comp):
            S = src[s]
            if kind == "E":
                d = S[sl] - S[_shift(sl, axis, -1)]
            else:
                d = S[_shift(sl, axis, +1)] - S[sl]
            if acc is None:
                acc = d if sign > 0 else -d
            else:
                acc = acc + d if sign > 0 else acc - d
        return acc

    def curl_update(self, kind: str, boxes: Dict[str, Box], dst: Dict[str, torch.Tensor],
                    src: Dict[str, torch.Tensor], cb: Dict[str, Coef]) -> None:
        for comp, box in boxes.items():
            if _empty(box):
                continue
            sl = box_slices(box)
            c = self.curl(kind, comp, sl, src)
            if c is None:
                continue
            dst[comp][sl] += cb[comp].materialize(sl) * c

    def fused_step(self, fin: Dict[str, torch.Tensor], fout: Dict[str, torch.Tensor], boxes: Dict[str, Box],
                   cb: Dict[str, Coef], source=None) -> None:
        """Reference semantics of the fused E+H kernel: E_new from (E_old,
        H_old) on the E boxes, the point source, then H_new from (H_old, E_new)
        on the H boxes, all written to ``fout``."""
        # like the kernel, only cells inside a component's box are written
        tmp = {c: fin[c].clone() for c in fin}
        e = {c: b for c, b in boxes.items() if c[0] == "E"}
        h = {c: b for c, b in boxes.items() if c[0] == "H"}
        self.curl_update("E", e, tmp, fin, cb)
        if source is not None:
            comp, idx, val = source
            tmp[comp][tuple(idx)] = val
        self.curl_update("H", h, tmp, tmp, cb)
        for c, b in boxes.items():
            if not _empty(b):
                sl = box_slices(b)
                fout[c][sl] = tmp[c][sl]

    def resident_1d_max_cells(self) -> int:
        return 1 << 30

    def resident_1d(self, F: Dict[str, torch.Tensor], boxes: Dict[str, Box], cb: Dict[str, Coef], nsteps: int,
                    src_i=None, vals=None) -> None:
        """Reference semantics of the register-resident 1D kernel
        (yee1d_res.hip): ``nsteps`` fused steps in place, hard Ez source
        ``vals[s]`` at cell ``src_i``.  CPU tensors run the native loop of
        the host library (csrc/host_yee1d.cpp); the torch ops below are the
        oracle it is tested against."""
        if self._res1d_native(F, boxes, cb, nsteps, src_i, vals):
            return
        for s in range(nsteps):
            nxt = {c: F[c].clone() for c in F}
            src = None if vals is None else ("Ez", (int(src_i), 0, 0), float(vals[s]))
            self.fused_step(F, nxt, boxes, cb, src)
            for c in F:
                F[c].copy_(nxt[c])

    native_1d = True  # CPU 1D runs take the host library's loop (False: the torch oracle)

    def _res1d_native(self, F, boxes, cb, nsteps, src_i, vals) -> bool:
        ez, hy = F["Ez"], F["Hy"]
        if (not self.native_1d or ez.device.type != "cpu" or ez.dtype not in (torch.float32, torch.float64)
                or not ez.is_contiguous() or not hy.is_contiguous() or hy.dtype != ez.dtype):
            return False
        try:
            from ..native import load_host_library
            lib = load_host_library(build_if_missing=False)
            fn = getattr(lib, "fdtd_res1d_cpu_%s" % ("f64" if ez.dtype == torch.float64 else "f32"))
        except (OSError, AttributeError):
            return False
        import ctypes
        n = ez.numel()
        whole = tuple(slice(0, d) for d in ez.shape)

        def cell(c):  # per-cell array of a coefficient with profiles / cells, None for a scalar
            if all(getattr(c, a) is None for a in ("cell", "px", "py", "pz")):
                return None
            v = c.materialize(whole)
            v = torch.as_tensor(v, dtype=ez.dtype).expand(ez.shape)
            return v.contiguous().reshape(-1)
        pe, ph = cell(cb["Ez"]), cell(cb["Hy"])
        lim = lambda b: (b[0][0], b[1][0]) if not _empty(b) else (0, 0)
        (elo, ehi), (hlo, hhi) = lim(boxes["Ez"]), lim(boxes["Hy"])
        v = None
        if vals is not None:
            v = vals.to("cpu", ez.dtype).contiguous()
        ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
        fn.restype = ctypes.c_int
        fn(ptr(ez), ptr(hy), ptr(pe), ptr(ph), ctypes.c_double(cb["Ez"].scalar if pe is None else 1.0),
           ctypes.c_double(cb["Hy"].scalar if ph is None else 1.0), ctypes.c_int(n),
           (ctypes.c_int * 4)(elo, ehi, hlo, hhi), ctypes.c_int(nsteps),
           ctypes.c_int(-1 if src_i is None else int(src_i)), ptr(v))
        return True

    def tb_step(self, fin: Dict[str, torch.Tensor], fout: Dict[str, torch.Tensor], boxes: Dict[str, Box],
                obox: Box, cb: Dict[str, Coef], steps: int, sources=None, tfsf=None) -> None:
        """Reference semantics of the temporally blocked kernel: ``steps``
        fused steps on the update boxes (reads outside the arrays count as
        zero, like the kernel's unloaded rows), then only ``obox`` ∩ each
        component's box is written to ``fout``.  ``tfsf`` = (TfsfSets, g
        table, first level): each level adds coef * g to the set's target
        cells after the curl update (the kernel adds g to the curl)."""
        pad = {c: torch.nn.functional.pad(fin[c], (1, 1, 1, 1, 1, 1)) for c in fin}
        shifted = {c: ((b[0][0] + 1, b[0][1] + 1, b[0][2] + 1), (b[1][0] + 1, b[1][1] + 1, b[1][2] + 1))
                   for c, b in boxes.items()}
        cbp = cb_pad(cb)
        e = {c: b for c, b in shifted.items() if c[0] == "E"}
        h = {c: b for c, b in shifted.items() if c[0] == "H"}
        cur = pad
        for l in range(steps):
            nxt = {c: cur[c].clone() for c in cur}
            self.curl_update("E", e, nxt, cur, cbp)
            if tfsf is not None:
                self._tfsf_level(nxt, tfsf, l, "E", shifted, cbp)
            if sources is not None and sources[l] is not None:
                # after the corrections, as the stepped path (and the kernel) does
                comp, idx, val = sources[l]
                nxt[comp][tuple(i + 1 for i in idx)] = val
            self.curl_update("H", h, nxt, nxt, cbp)
            if tfsf is not None:
                self._tfsf_level(nxt, tfsf, l, "H", shifted, cbp)
            cur = nxt
        for c, b in boxes.items():
            ob = box_intersect_(b, obox)
            if not _empty(ob):
                sl = box_slices(ob)
                sp = tuple(slice(s.start + 1, s.stop + 1) for s in sl)
                fout[c][sl] = cur[c][sp]

    tb_drude_max_steps = 5

    def tb_drude_step(self, fin: Dict[str, torch.Tensor], fout: Dict[str, torch.Tensor], boxes: Dict[str, Box],
                      obox: Box, cb: Dict[str, Coef], steps: int, sources, drude: dict) -> None:
        """Reference semantics of the Drude pass (csrc/tb3d_mr.h DrDev):
        :meth:`tb_step`'s fused steps, with the E components inside
        ``drude["box"]`` taking E' = (b0 cbd) curl - b2 delta + m1 E + m2 Ep
        from the state ``drude["sin"]`` (delta + ids, Ep; float4 per cell),
        whose advanced values go to ``drude["sout"]`` on the cells of
        ``obox`` inside the box."""
        B = drude["box"]
        pad = {c: torch.nn.functional.pad(fin[c], (1, 1, 1, 1, 1, 1)) for c in fin}
        shifted = {c: ((b[0][0] + 1, b[0][1] + 1, b[0][2] + 1), (b[1][0] + 1, b[1][1] + 1, b[1][2] + 1))
                   for c, b in boxes.items()}
        cbp = cb_pad(cb)
        unit = {c: Coef(1.0) for c in cb}
        e = {c: b for c, b in shifted.items() if c[0] == "E"}
        h = {c: b for c, b in shifted.items() if c[0] == "H"}
        E = ("Ex", "Ey", "Ez")
        bsl = tuple(slice(B[0][d] + 1, B[1][d] + 1) for d in range(3))
        s0, s1 = drude["sin"]
        ids = drude["ids"]  # int32 over B (the kernel reads the same bits from s0[..., 3] in fp32)
        lut = drude["lut"]
        k = [lut[q][((ids >> (8 * q)) & 0xff).long()] for q in range(3)]  # (bx, by, bz, 4) per component
        delta = [s0[..., q].clone() for q in range(3)]
        ep = [s1[..., q].clone() for q in range(3)]
        cbd = float(drude["cbd"])
        cur = pad
        for l in range(steps):
            nxt = {c: cur[c].clone() for c in cur}
            self.curl_update("E", e, nxt, cur, cbp)
            curl = {c: torch.zeros_like(cur[c]) for c in E}
            self.curl_update("E", e, curl, cur, unit)
            for q, c in enumerate(E):
                cu, ec = curl[c][bsl], cur[c][bsl]
                nxt[c][bsl] = k[q][..., 0] * cu - k[q][..., 1] * delta[q] + k[q][..., 2] * ec + k[q][..., 3] * ep[q]
                delta[q] = cbd * cu
                ep[q] = ec.clone()
            if sources is not None and sources[l] is not None:
                comp, idx, val = sources[l]
                nxt[comp][tuple(i + 1 for i in idx)] = val
            self.curl_update("H", h, nxt, nxt, cbp)
            cur = nxt
        for c, b in boxes.items():
            ob = box_intersect_(b, obox)
            if not _empty(ob):
                sl = box_slices(ob)
                sp = tuple(slice(s.start + 1, s.stop + 1) for s in sl)
                fout[c][sl] = cur[c][sp]
        ob = box_intersect_(B, obox)
        if not _empty(ob):
            o0, o1 = drude["sout"]
            sl = tuple(slice(ob[0][d] - B[0][d], ob[1][d] - B[0][d]) for d in range(3))
            for q in range(3):
                o0[sl + (q,)] = delta[q][sl]
                o1[sl + (q,)] = ep[q][sl]
            o0[sl + (3,)] = s0[sl + (3,)]
            o1[sl + (3,)] = 0.0

    tb_amp_max_steps = 3

    def tb_amp_step(self, fin: Dict[str, torch.Tensor], fout: Dict[str, torch.Tensor], boxes: Dict[str, Box],
                    obox: Box, cb: Dict[str, Coef], steps: int, line, vals, amps, aboxes, accuracy: float,
                    counts: torch.Tensor) -> None:
        """Reference semantics of the amplitude pass (csrc/tb3d_mr.h AmpDev):
        the fused steps of :meth:`tb_step` with, after each, the amplitude
        update (:meth:`amplitude_update`) of the cells of ``obox`` inside
        ``aboxes`` -- ``counts[l]`` += the changed cells of step l -- and the
        hard source on the z line ``line`` = (E component, i, j, k0, k1)."""
        pad = {c: torch.nn.functional.pad(fin[c], (1, 1, 1, 1, 1, 1)) for c in fin}
        shifted = {c: ((b[0][0] + 1, b[0][1] + 1, b[0][2] + 1), (b[1][0] + 1, b[1][1] + 1, b[1][2] + 1))
                   for c, b in boxes.items()}
        cbp = cb_pad(cb)
        e = {c: b for c, b in shifted.items() if c[0] == "E"}
        h = {c: b for c, b in shifted.items() if c[0] == "H"}
        comps = ("Ex", "Ey", "Ez", "Hx", "Hy", "Hz")
        cur = pad
        for l in range(steps):
            nxt = {c: cur[c].clone() for c in cur}
            self.curl_update("E", e, nxt, cur, cbp)
            if line is not None:
                comp, i, j, k0, k1 = line
                nxt[comp][i + 1, j + 1, k0 + 1:k1 + 1] = float(vals[l])
            self.curl_update("H", h, nxt, nxt, cbp)
            cur = nxt
            for c, a, ab in zip(comps, amps, aboxes):
                b = box_intersect_(ab, obox)
                if _empty(b):
                    continue
                view = {c: cur[c][tuple(slice(b[0][d] + 1, b[1][d] + 1) for d in range(3))]}
                n = self.amplitude_update(view[c], a[box_slices(b)], ((0, 0, 0), tuple(view[c].shape)), accuracy)
                counts[l] += n
        # the whole output box of every component, like the kernel (the line
        # source may sit outside its component's update box)
        sl = box_slices(obox)
        sp = tuple(slice(s_.start + 1, s_.stop + 1) for s_ in sl)
        for c in boxes:
            fout[c][sl] = cur[c][sp]

    def _tfsf_level(self, F, tfsf, l: int, kind: str, boxes, cb) -> None:
        """TF/SF corrections of level ``l`` of a blocked pass on fields padded
        by one cell: the E-form tables of the stepped path (``sets.tables``,
        models/scheme.py ``_init_tfsf``) applied from the incident line as it
        stood at that level (recorded by :meth:`tfsf_pass`), so a blocked
        pass is bit-for-bit the stepped arithmetic."""
        sets, g, level0 = tfsf
        hin, ein = g.lines[level0 + l]
        inc = hin if kind == "E" else ein
        shape = tuple(F["Ex"].shape)
        for c in (("Ex", "Ey", "Ez") if kind == "E" else ("Hx", "Hy", "Hz")):
            for tab in sets.tables.get(c, ()):
                if tab.n == 0:
                    continue
                off = tab.__dict__.setdefault("_pad_off", {}).get(shape)
                if off is None:
                    ijk = tab.ijk.long() + 1
                    off = tab._pad_off[shape] = (ijk[:, 0] * shape[1] + ijk[:, 1]) * shape[2] + ijk[:, 2]
                v = (inc[tab.i0] * tab.w0 + inc[tab.i0 + 1] * tab.w1) * tab.coef
                F[c].view(-1).index_add_(0, off, v.to(F[c].dtype))

    tfsf_sets_ok = True  # tb_step applies TfsfSets corrections (the blocked kernel's form)

    def tfsf_pass(self, einc: torch.Tensor, hinc: torch.Tensor, ce: float, ch: float, src_vals, reach: int,
                  sets, slot: int = 0, dry: bool = False) -> torch.Tensor:
        """Reference semantics of k_tfsf_pass (yee3d_tb.hip): the incident
        line advanced ``len(src_vals)`` steps, the per-level g table of the
        pass returned (levels x sets.ld).  ``dry``: the line is left as it was
        (the g table of a hybrid pass, whose shell steps the line itself)."""
        if dry:
            einc, hinc = einc.clone(), hinc.clone()
        T = len(src_vals)
        n = einc.numel()
        m = min(n, reach)
        ld = sets.ld
        g = torch.zeros(max(8, T) * max(1, ld), dtype=einc.dtype, device=einc.device)
        i0 = sets.i0.long()
        w0, w1, cc = sets.w0.to(einc.dtype), sets.w1.to(einc.dtype), sets.c.to(einc.dtype)
        ne = sets.n_e
        g.lines = []  # (H line before, E line after) each level's E half step: _tfsf_level
        for l in range(T):
            hin = hinc.clone()
            if ne:
                g[l * ld:l * ld + ne] = cc[:ne] * (w0[:ne] * hinc[i0[:ne]] + w1[:ne] * hinc[i0[:ne] + 1])
            if m > 0:
                new = einc[:m].clone()
                if m > 1:
                    new[1:m] = einc[1:m] + ce * (hinc[0:m - 1] - hinc[1:m])
                new[0] = src_vals[l]
                einc[:m] = new
            g.lines.append((hin, einc.clone()))
            if ld > ne:
                g[l * ld + ne:(l + 1) * ld] = cc[ne:] * (w0[ne:] * einc[i0[ne:]] + w1[ne:] * einc[i0[ne:] + 1])
            mh = min(m, n - 1)
            if mh > 0:
                hinc[:mh] += ch * (einc[:mh] - einc[1:mh + 1])
        return g

    def chain_update(self, kind: str, boxes: Dict[str, Box], F: Dict[str, torch.Tensor], upml: Dict[str, dict],
                     p: int, drude: bool, plain_form: bool = False, plain: Optional[Dict[str, Box]] = None,
                     cb: Optional[Dict[str, Coef]] = None, rows=None) -> None:
        """Reference semantics of the fused UPML/Drude chain kernel
        (chain_kernels.hip): D -> [D1] -> E per cell of each box, plus the
        plain Yee update on the folded ``plain`` boxes.  ``rows`` (dispersive
        launches): ``(table, lo0, lo1)``, per local row (x, y) the z range of
        the cells that run the chain; the other cells of the boxes take the
        plain update ``F += cb curl`` (their D / D1 levels are left alone)."""
        if plain:
            pb = {c: plain.get(c, ((0, 0, 0), (0, 0, 0))) for c in boxes}
            self.curl_update(kind, pb, F, F, cb)
        new = []
        for c, box in boxes.items():
            if _empty(box):
                continue
            st = upml[c]
            sl = box_slices(box)
            curl = self.curl(kind, c, sl, F)
            mask = None if rows is None else self._row_mask(rows, box)

            def lv(t, box=box, sl=sl):
                # full-grid level or region-local one (models/regions.py)
                return t.view(box) if isinstance(t, RegionLevel) else t[sl]
            D = st["D"][p]
            Dn = st["caD"].materialize(sl) * lv(D[0]) + st["cbD"].materialize(sl) * curl
            nw, old = Dn, lv(D[0])
            upd = [(lv(D[-1]), Dn)]
            if drude:
                D1 = st["D1"][p]
                D1n = (st["b0"].materialize(sl) * Dn + st["b1"].materialize(sl) * lv(D[0])
                       + st["b2"].materialize(sl) * lv(D[1]) + st["ma1"].materialize(sl) * lv(D1[0])
                       + st["ma2"].materialize(sl) * lv(D1[1]))
                upd.append((lv(D1[2]), D1n))
                nw, old = D1n, lv(D1[0])
            cbE, ccE = (st["plain"]["cbE"], st["plain"]["ccE"]) if plain_form else (st["cbE"], st["ccE"])
            En = st["caE"].materialize(sl) * F[c][sl] + cbE.materialize(sl) * nw + ccE.materialize(sl) * old
            if mask is not None:
                En = torch.where(mask, En, F[c][sl] + cb[c].materialize(sl) * curl)
                upd = [(t, torch.where(mask, v, t)) for t, v in upd]
            new.append((c, sl, En, upd))
        # every component reads the other kind only: the stores can follow in any order
        for c, sl, En, upd in new:
            for t, v in upd:
                t.copy_(v)
            F[c][sl] = En

    @staticmethod
    def _row_mask(rows, box: Box) -> torch.Tensor:
        """Boolean mask over ``box``: z inside the row's dispersive range."""
        tab, lo0, lo1 = rows
        nx, ny = tab.shape[0], tab.shape[1]
        X = torch.arange(box[0][0], box[1][0], device=tab.device) - lo0
        Y = torch.arange(box[0][1], box[1][1], device=tab.device) - lo1
        okx = (X >= 0) & (X < nx)
        oky = (Y >= 0) & (Y < ny)
        r = tab[X.clamp(0, nx - 1)][:, Y.clamp(0, ny - 1)]  # (bx, by, 2)
        ok = (okx[:, None] & oky[None, :])[..., None]
        Z = torch.arange(box[0][2], box[1][2], device=tab.device)[None, None, :]
        return ok & (Z >= r[..., 0:1]) & (Z < r[..., 1:2])

    def curl_general(self, kind: str, comp: str, box: Box, out: torch.Tensor, inp: torch.Tensor,
                     src: Dict[str, torch.Tensor], ca: Coef, cb: Coef) -> None:
        if _empty(box):
            return
        sl = box_slices(box)
        c = self.curl(kind, comp, sl, src)
        v = ca.materialize(sl) * inp[sl]
        if c is not None:
            v = v + cb.materialize(sl) * c
        out[sl] = v

    def lincomb(self, out: torch.Tensor, box: Box, terms: Sequence[Tuple[Coef, torch.Tensor]]) -> None:
        if _empty(box):
            return
        sl = box_slices(box)
        v = None
        for coef, x in terms:
            t = coef.materialize(sl) * x[sl]
            v = t if v is None else v + t
        out[sl] = v

    def cpml_apply(self, kind: str, target: torch.Tensor, src: torch.Tensor, axis: int, sign: int,
                   psi: torch.Tensor, psi_box: Box, box: Box, b: torch.Tensor, c: torch.Tensor,
                   kinv_m1: torch.Tensor, cb: Coef) -> None:
        """CPML slab correction (models/cpml.py)."""
        if _empty(box):
            return
        sl = box_slices(box)
        if kind == "E":
            diff = src[sl] - src[_shift(sl, axis, -1)]
        else:
            diff = src[_shift(sl, axis, +1)] - src[sl]
        psl = tuple(slice(box[0][d] - psi_box[0][d], box[1][d] - psi_box[0][d]) for d in range(3))
        view = [1, 1, 1]
        view[axis] = -1
        bb = b[sl[axis]].view(view)
        cc = c[sl[axis]].view(view)
        kk = kinv_m1[sl[axis]].view(view)
        psi[psl] = bb * psi[psl] + cc * diff
        corr = kk * diff + psi[psl]
        if sign < 0:
            corr = -corr
        target[sl] += cb.materialize(sl) * corr

    # --------------------------------------------------------------- sources
    def set_value(self, t: torch.Tensor, idx: Sequence[int], value: float) -> None:
        t[tuple(idx)] = value

    def set_values(self, t: torch.Tensor, flat_idx: torch.Tensor, value: float) -> None:
        t.view(-1)[flat_idx] = value

    # ------------------------------------------------------------------ halo
    def pack(self, tensors: Sequence[torch.Tensor], box: Box, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        sl = box_slices(box)
        parts = [t[sl].reshape(-1) for t in tensors]
        buf = torch.cat(parts)
        if out is not None:
            out.copy_(buf)
            return out
        return buf

    def unpack(self, tensors: Sequence[torch.Tensor], box: Box, buf: torch.Tensor) -> None:
        sl = box_slices(box)
        n = 1
        for d in range(3):
            n *= box[1][d] - box[0][d]
        for c, t in enumerate(tensors):
            t[sl] = buf[c * n:(c + 1) * n].view(t[sl].shape)

    def copy_box(self, src: Sequence[torch.Tensor], dst: Sequence[torch.Tensor], box: Box) -> None:
        """dst[c][box] = src[c][box] for every component pair."""
        sl = box_slices(box)
        for a, b in zip(src, dst):
            b[sl] = a[sl]

    # ------------------------------------------------------------ reductions
    def maxabs(self, t: torch.Tensor, box: Box) -> float:
        if _empty(box):
            return 0.0
        v = t[box_slices(box)].abs()
        if torch.isnan(v).any():
            return float("inf")
        return float(v.max())

    def amplitude_update_many(self, fields, amps, boxes, accuracy: float, counter: torch.Tensor) -> None:
        """Several components' amplitude updates; the changed count is added
        to ``counter`` (semantics of the HIP kernel)."""
        for f, a, b in zip(fields, amps, boxes):
            counter += self.amplitude_update(f, a, b, accuracy)

    def amplitude_update(self, f: torch.Tensor, amp: torch.Tensor, box: Box, accuracy: float) -> int:
        """Running max-|f| with the reference's convergence test
        (``Scheme3D::updateAmplitude``, Scheme3D.cpp:3294-3333): the stored
        amplitude is raised only when it grows by more than ``accuracy``
        (relative); returns the number of such cells."""
        if _empty(box):
            return 0
        sl = box_slices(box)
        v = f[sl].abs()
        a = amp[sl]
        ge = v >= a
        diff = v - a
        denom = torch.where(a != 0, a, torch.where(v != 0, v, torch.ones_like(v)))
        acc = diff / denom
        upd = ge & (acc > accuracy)
        amp[sl] = torch.where(upd, v, a)
        return int(upd.sum())

    # ----------------------------------------------------------------- TF/SF
    def inc_step_e(self, einc: torch.Tensor, hinc: torch.Tensor, coef: float, source: float) -> None:
        """1D incident line, E half step (Scheme3D.cpp:25-59)."""
        einc[1:] = einc[1:] + coef * (hinc[:-1] - hinc[1:])
        einc[0] = source

    def inc_step_h(self, einc: torch.Tensor, hinc: torch.Tensor, coef: float) -> None:
        """1D incident line, H half step (Scheme3D.cpp:62-82)."""
        hinc[:-1] = hinc[:-1] + coef * (einc[:-1] - einc[1:])

    def tfsf_apply(self, target: torch.Tensor, table: "TfsfTable", inc: torch.Tensor, box: Box) -> None:
        """``target[cell] += coef * (w0 inc[i0] + w1 inc[i0+1])`` for the
        table's cells inside ``box`` (local)."""
        if table.n == 0 or _empty(box):
            return
        ijk = table.ijk
        m = torch.ones(table.n, dtype=torch.bool, device=ijk.device)
        for d in range(3):
            m &= (ijk[:, d] >= box[0][d]) & (ijk[:, d] < box[1][d])
        v = (inc[table.i0] * table.w0 + inc[table.i0 + 1] * table.w1) * table.coef
        v = torch.where(m, v, torch.zeros_like(v))
        flat = target.view(-1)
        flat.index_add_(0, table.off, v.to(target.dtype))


class TfsfTable:
    """Per-component TF/SF correction list: ``target[off] += coef *
    (w0*inc[i0] + w1*inc[i0+1])`` (built by :mod:`fdtd3d_amd.models.tfsf`).
    Target cells within one table are unique."""

    def __init__(self, off, i0, w0, w1, coef, ijk):
        self.off = off
        self.i0 = i0
        self.w0 = w0
        self.w1 = w1
        self.coef = coef
        self.ijk = ijk
        # host-side bounds, so the HIP op validates without a device sync
        # (required inside HIP graph capture)
        self.max_off = int(off.max()) if off.numel() else -1
        self.max_inc = int(i0.max()) + 1 if i0.numel() else -1

    @property
    def n(self) -> int:
        return int(self.off.numel())
