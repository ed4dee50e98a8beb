"""Temporal blocking of the 3D leapfrog (mixed into :class:`YeeScheme`).

* ``_tb_step``: T leapfrog steps of plain 3D runs in ONE HBM pass through the
  blocked kernels (``csrc/yee3d_tb.hip`` fp32, ``csrc/yee3d_tb64.hip`` fp64).
  Decomposed runs exchange T-deep ghosts (faces, edges, corners) once per pass
  on a high-priority side stream, overlapped with the interior pass, then
  update the T-thick shells.
* ``_hybrid_step``: runs with PML / TF-SF / dispersive media -- the blocked
  kernel advances the core, the per-step kernels the shell plus a band.

The reference has no counterpart: its only communication-avoiding scheme is
the deep halo of ``--buffer-size`` (``Source/Grid/ParallelGrid.cpp:2161-2194,
2365-2489``) with per-step CPU updates, and its CUDA path launches one kernel
per component and step (``Source/Cuda/CudaInterface.cu:583-812``).
"""

from __future__ import annotations

from typing import Tuple

import torch

from ..parallel.domain import box_empty, box_intersect, box_subtract, box_volume

Box = Tuple[Tuple[int, int, int], Tuple[int, int, int]]

# automatic steps per pass of the fp64 blocked kernel (yee3d_tb64.hip);
# 512^3: T=1 42.6k, 2 75.7k, 3 99.0k, 4 110k Mcells/s
F64_AUTO_STEPS = 4
# automatic steps per hybrid pass (fp32): 512^3 CPML + TF/SF 79.2k / 75.5k /
# 74.5k Mcells/s at T = 5 / 4 / 3, UPML + TF/SF 70.9k / 67.9k / 66.6k, Drude
# sphere 53.5k / 52.1k / 49.3k, CPML point 99.4k / 95.0k / 80.2k: the faster
# T = 5 core outweighs the one-cell deeper band
HYBRID_AUTO_STEPS = 5
# automatic steps per pass of the 2D TMz / TEz blocked kernel (yee2d_tb.hip);
# 16384^2 fp32 TMz: T=1 119k, 5 851k, 6 1.01M, 7 1.11M, 8 1.06M Mcells/s
TB2D_AUTO_STEPS = 7
# fp64: T=1 67k, 4 361k, 6 521k-638k, 7 701k, 8 630k Mcells/s
TB2D_AUTO_STEPS_F64 = 7


# automatic steps per pass of the fp32 3D blocked kernel: uniform media
# (1024^3: T=5 281-289k vs T=4 260-263k Mcells/s on one GPU; decomposed over
# more than two ranks T=4, whose ghosts and shells are thinner:
# tools/decomp_cost.py 8 ranks T=4 229k vs T=5 221k per GPU).  Per-cell
# coefficients of one kind (dielectric or magnetic scenes) run the sparse
# multi-row kernel with an LDS ring of coefficient planes (512^3 eps sphere:
# T=3 160k, 4 188k, 5 203k Mcells/s); per-cell E AND H keep the planes in
# registers, spill-free only to T=2.
F32_AUTO_STEPS = 5
F32_AUTO_STEPS_MANY_RANKS = 4
F32_AUTO_STEPS_PERCELL_BOTH = 2
# plain runs with in-kernel TF/SF (TfsfSets): 512^3 vacuum + TF/SF T=4 127k,
# T=5 86k Mcells/s (the TF/SF variant spills at T=5)
F32_AUTO_STEPS_TFSF = 4


# hybrid_shell modes that take the blocked shell (_hybrid3_plan) when the run fits it
BLOCKED_SHELL_MODES = ("blocked", "mixed")


def auto_time_block(scheme: str, dtype_name: str, backend: str, percell, world: int = 1, tfsf: bool = False) -> int:
    """Steps per pass of a plain (no PML / TF-SF / dispersion) run in
    automatic mode -- ONE rule for the serial scheme, the decomposed driver
    (which must size the ghost layers before the scheme exists) and bench.py.
    ``percell``: number of field kinds (E, H) with per-cell coefficients
    (a bool counts as one)."""
    if backend != "hip":
        return 1
    if scheme in ("tmz", "tez"):
        return TB2D_AUTO_STEPS if dtype_name == "f32" else TB2D_AUTO_STEPS_F64
    if scheme != "3d":
        return 1
    if dtype_name != "f32":
        return F64_AUTO_STEPS
    if int(percell) >= 2:
        return F32_AUTO_STEPS_PERCELL_BOTH
    if tfsf:
        return F32_AUTO_STEPS_TFSF
    return F32_AUTO_STEPS if world <= 2 else F32_AUTO_STEPS_MANY_RANKS


def _cut_pieces(b: Box, cuts, keep=()):
    """``b`` split at the absorbing-slab cuts of every axis: [(box, axes
    bits)], bit a set when the piece may touch a slab along axis a.  The
    high-side cut moves one cell down: a tile recomputes its halo cells with
    its own specialisation, and the H update of the last cell below a high
    slab reads the new E of the first slab cell (H^{n+1} needs E^{n+1} at
    +1 along every axis; E^{n+1} needs only H^n, so the low side is exact).
    Axes in ``keep`` are not cut (the piece keeps its slab cells and the band
    beyond them in one box: a thin face of the shell stays one tile deep
    instead of two part-filled ones); their bit is set when ``b`` reaches a
    slab."""
    pieces = [(b, 0)]
    for a in range(3):
        if cuts[a] is None:
            continue
        lo_c, hi_c = cuts[a][0], cuts[a][1] - 1
        if a in keep:
            if b[0][a] < lo_c or b[1][a] > hi_c:
                pieces = [(pb, ax | (1 << a)) for pb, ax in pieces]
            continue
        nxt = []
        for pb, ax in pieces:
            for s_lo, s_hi, slab in ((None, lo_c, True), (lo_c, hi_c, False), (hi_c, None, True)):
                l0 = pb[0][a] if s_lo is None else max(pb[0][a], s_lo)
                h0 = pb[1][a] if s_hi is None else min(pb[1][a], s_hi)
                if h0 <= l0:
                    continue
                lo, hi = list(pb[0]), list(pb[1])
                lo[a], hi[a] = l0, h0
                nxt.append(((tuple(lo), tuple(hi)), ax | ((1 << a) if slab else 0)))
        pieces = nxt
    return [(pb, ax) for pb, ax in pieces if not box_empty(pb)]


def _cut_box(b: Box, box: Box):
    """``b`` split at a dispersive box: [(piece, 8)] for the part within
    [box.lo - 1, box.hi) on every axis (the cell below the box's low face
    updates H from the box's new E), [(piece, 0)] for the rest."""
    lo = tuple(box[0][d] - 1 for d in range(3))
    inner = (tuple(max(b[0][d], lo[d]) for d in range(3)), tuple(min(b[1][d], box[1][d]) for d in range(3)))
    if box_empty(inner):
        return [(b, 0)]
    return [(inner, 8)] + [(r, 0) for r in box_subtract(b, inner) if not box_empty(r)]


def _merge_pieces(pieces):
    """Merge pieces of the same CPML class whose union is a box (fewer,
    larger boxes per shell launch)."""
    out = list(pieces)
    changed = True
    while changed:
        changed = False
        for i in range(len(out)):
            for j in range(i + 1, len(out)):
                (a, ca), (b, cb_) = out[i], out[j]
                if ca != cb_:
                    continue
                for d in range(3):
                    same = all(a[0][e] == b[0][e] and a[1][e] == b[1][e] for e in range(3) if e != d)
                    if same and (a[1][d] == b[0][d] or b[1][d] == a[0][d]):
                        lo = tuple(min(a[0][e], b[0][e]) for e in range(3))
                        hi = tuple(max(a[1][e], b[1][e]) for e in range(3))
                        out[i] = ((lo, hi), ca)
                        del out[j]
                        changed = True
                        break
                if changed:
                    break
            if changed:
                break
    return out


class PassTimer:
    """Per-pass breakdown of decomposed blocked / hybrid passes on the main
    stream: ``interior`` (the pass part that needs no fresh ghost, issued
    while the exchange runs on the side stream), ``exchange_wait`` (main
    stream blocked on the side stream after the interior: the part of the
    exchange the interior did not hide) and ``shell`` (the parts that read
    the fresh ghosts).  HIP events on the GPU, wall clock on the CPU (where
    the gloo exchange is synchronous and lands in ``exchange_wait``)."""

    def __init__(self, device):
        self.cuda = getattr(device, "type", str(device)) == "cuda"
        self.passes: list = []
        self._cur = None

    def mark(self, name: str) -> None:
        if name == "start":
            self._cur = []
            self.passes.append(self._cur)
        if self._cur is None:
            return
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._cur.append((name, ev))
        else:
            import time
            self._cur.append((name, time.perf_counter()))

    def summary(self) -> dict:
        """Totals in ms over the recorded passes (synchronises the device)."""
        out = {"passes": len(self.passes), "interior_ms": 0.0, "exchange_wait_ms": 0.0, "shell_ms": 0.0}
        keys = {"interior": "interior_ms", "wait": "exchange_wait_ms", "end": "shell_ms"}
        for marks in self.passes:
            for (_, a), (name, b) in zip(marks, marks[1:]):
                if self.cuda:
                    b.synchronize()
                    ms = a.elapsed_time(b)
                else:
                    ms = (b - a) * 1e3
                if name in keys:
                    out[keys[name]] += ms
        return out


class BlockedStepping:
    """Blocked and hybrid passes of :class:`fdtd3d_amd.models.scheme.YeeScheme`
    (uses its fields, ops, domain, halo, layout and per-step update methods)."""

    _tfsf_once = False
    pass_timer = None  # PassTimer of decomposed passes (bench.py / --json), None: off
    _skip_side_wait = False  # tests only: drop the main stream's wait on the exchange (negative control)

    def _mark(self, name: str) -> None:
        if self.pass_timer is not None:
            self.pass_timer.mark(name)

    def _join_side(self, side) -> None:
        """Main stream waits for the ghost exchange issued on ``side``."""
        if side is not None and not self._skip_side_wait:
            torch.cuda.current_stream(self.device).wait_stream(side)

    def _fork_side_stream(self):
        """High-priority side stream for the ghost exchange, ordered after
        everything issued so far on the current stream (the pack must see the
        previous pass's results) but NOT after the interior pass launched
        next: that pass reads owned cells only (the ghosts it may touch lie
        beyond its dependency cone) and writes the other buffer, so the
        exchange runs concurrently with it.  None on the CPU."""
        if self.device.type != "cuda":
            return None
        side = getattr(self, "_side_stream", None)
        if side is None:
            # high priority: its pack / unpack kernels get CUs next to the interior pass
            side = torch.cuda.Stream(device=self.device, priority=-1)
            self._side_stream = side
        side.wait_stream(torch.cuda.current_stream(self.device))
        return side

    # ------------------------------------------------------ hybrid blocking
    def _init_hybrid(self) -> None:
        """Blocked core + stepped shell for 3D and 2D runs with absorbing
        layers, TF/SF injection or dispersive media (serial HIP runs by
        default; the 2D core runs the yee2d_tb.hip kernel).

        Every ``T`` steps: (1) the temporally blocked kernel advances the
        *core* -- cells at least ``T + 2`` away from any PML / CPML slab,
        TF/SF target cell and dispersive box -- by ``T`` steps in one HBM pass
        (F -> F_alt); (2) the regular per-step kernels (UPML/Drude chain,
        CPML, TF/SF corrections, sources) advance the *shell* (everything
        else) plus a ``T + 1`` deep band into the core, in place in F: stale
        values beyond the band corrupt at most ``T`` cells of it, all inside
        the core, so the shell itself is exact; (3) the shell is copied into
        F_alt and the buffers swap.  Bit-for-bit the same arithmetic as the
        stepped run in both regions (the core's plain Yee update is what the
        step kernels do there)."""
        cfg = self.cfg
        two_d = cfg.scheme in ("tmz", "tez")
        H = int(cfg.hybrid_block)
        if H <= 0:
            if self.ops.name != "hip":
                H = 1
            elif two_d:
                H = TB2D_AUTO_STEPS if self.dtype == torch.float32 else TB2D_AUTO_STEPS_F64
            else:
                H = HYBRID_AUTO_STEPS if self.dtype == torch.float32 else F64_AUTO_STEPS
        hmax = getattr(self.ops, "tb2d_max_steps" if two_d else "tb_max_steps", 8 if two_d else 6)
        if (H <= 1 or self.fused or self.tb > 1 or cfg.scheme not in ("3d", "tmz", "tez")
                or not hasattr(self.ops, "tb_step") or cfg.use_amp_mode or self.graph_mode
                or not (cfg.use_pml or cfg.use_tfsf or cfg.use_metamaterials) or H > hmax):
            return
        if self.halo is not None and (cfg.scheme != "3d" or self.domain.buffer_size != H):
            # decomposed: one T-deep exchange per pass feeds both the core and
            # the deep-halo stepped shell, so the ghosts must be exactly T deep
            return
        if (two_d and int(cfg.hybrid_block) <= 0 and self.use_upml_chain and self.dtype == torch.float32
                and self.ops.name == "hip"):
            # measured 8192^2 TMz UPML + TF/SF fp32: stepped 88.7k > hybrid 77.1k
            # Mcells/s (the thin shell's per-window launches cost as much as the
            # whole stepped grid); fp64 and CPML gain (52.5k -> 72.9k, 106k -> 116k)
            return
        # fp32 3D rows are float4 along z, 2D rows 16-byte lanes along y
        if self.ops.name == "hip":
            if two_d and self.domain.shape[1] % (16 // self.dtype.itemsize) != 0:
                return
            if not two_d and self.dtype == torch.float32 and self.domain.shape[2] % 4 != 0:
                return
        if self._hybrid3_ok():
            # automatic T: 4, where the face classes hand psi through LDS
            # (csrc/tb3d_mr.h LPS) in the plain kernel's tile
            T3 = H if int(cfg.hybrid_block) > 0 or not self.use_cpml else 4
            plan = self._hybrid3_plan(T3)
            if plan is not None and getattr(cfg, "hybrid_shell", "auto") == "mixed" and self.use_cpml:
                plan = self._hybrid4_plan(plan)
            if plan is not None:
                if not hasattr(self, "F_alt"):
                    self.F_alt = [{c: self._zeros() for c in self.comps} for _ in range(self.planes)]
                self.hybrid = plan
                return
        if self._hybrid2_ok() and self._hybrid2_regions():
            plan = self._hybrid2_plan(H)
            if plan is None:
                self.upml_regions = None
                self.drude_box = None
            else:
                if not hasattr(self, "F_alt"):
                    self.F_alt = [{c: self._zeros() for c in self.comps} for _ in range(self.planes)]
                self.F_3 = [{c: self._zeros() for c in self.comps} for _ in range(self.planes)]
                self.hybrid = plan
                return
        plan = self._hybrid_plan(H)
        if plan is None:
            return
        if int(cfg.hybrid_block) <= 0 and plan["cut_cells"] > 0.5 * self.cells():
            # automatic mode: a dispersive box over half the grid leaves too
            # little core.  (512^3 Drude sphere r=128, the box an eighth of
            # the grid: hybrid 51.7k vs stepped 45.7k Mcells/s once the Drude
            # chain reads its coefficients through the material LUT; 37.8k vs
            # 42k before)
            return
        if not hasattr(self, "F_alt"):
            self.F_alt = [{c: self._zeros() for c in self.comps} for _ in range(self.planes)]
        self.hybrid = plan

    # ------------------------------------------------ hybrid, blocked shell
    def _hybrid3_ok(self) -> bool:
        """Runs whose shell takes blocked passes too (``hybrid_shell`` auto or
        blocked): serial fp32 3D HIP runs with CPML absorbing layers and / or
        TF/SF plane waves along x or y (in-kernel TfsfSets), uniform media.
        The CPML variant of the blocked kernel carries psi through the pass's
        levels (csrc/yee3d_tb.hip, thread-private hand-off)."""
        cfg = self.cfg
        mode = getattr(cfg, "hybrid_shell", "auto")
        if mode not in BLOCKED_SHELL_MODES or self.ops.name != "hip" or not hasattr(self.ops, "tb_step"):
            return False
        if cfg.scheme != "3d" or self.halo is not None or cfg.use_amp_mode or cfg.use_metamaterials:
            return False
        if self.dtype != torch.float32 or self.domain.shape[2] % 4 != 0:
            return False
        if cfg.use_pml and (not self.use_cpml or self.use_upml_chain):
            return False
        if cfg.use_tfsf and getattr(self, "tfsf_sets", None) is None:
            return False
        if not (self.use_cpml or cfg.use_tfsf):
            return False
        return not any(getattr(self.cb[c], "cell", None) is not None for c in self.comps)

    def _hybrid3_plan(self, T: int):
        """Every cell advances ``T`` steps per pass in ONE blocked launch per
        box, all reading ``F`` and writing ``F_alt``: the plain kernel on the
        core (cells at least ``T + 1`` -- ``T + 2`` when staggering needs it --
        from every CPML slab cell and TF/SF target, so its dependency cone
        holds only plain cells) and the CPML + TF/SF variant on the six shell
        boxes around it.  No stepped band, no shell copy: a shell box's cone
        reaches into the core, where the variant's update is the plain one."""
        cfg = self.cfg
        size = cfg.size
        dom = self.domain
        alloc = dom.allocated_global()

        def grow(b, n):
            return (tuple(b[0][d] - n for d in range(3)), tuple(b[1][d] + n for d in range(3)))

        K = None
        for m in (T + 1, T + 2):
            lo, hi = [0, 0, 0], list(size)
            for a in range(3):
                edge = 0
                if cfg.use_pml:
                    edge = max(edge, self.layout.pml_size[a])
                if cfg.use_tfsf:
                    edge = max(edge, cfg.tfsf_size[a] + 1)
                if edge > 0:
                    lo[a], hi[a] = edge + m, size[a] - edge - m
            cand = (tuple(lo), tuple(hi))
            if box_empty(cand):
                return None
            g = grow(cand, T + 1)
            if self.use_cpml and any(not box_empty(box_intersect(g, sl.gbox))
                                     for slabs in self.cpml.slabs.values() for sl in slabs):
                continue
            if cfg.use_tfsf and self._tfsf_targets_in(dom.to_local(g)):
                continue
            K = cand
            break
        if K is None:
            return None
        if self.use_cpml and T not in getattr(self.ops, "tb_cpml_steps", ()):
            return None
        # shell pieces by class: the CPML axes whose slabs a piece's
        # dependency cone reaches (cuts T + 1 beyond each slab), and whether
        # it reaches a TF/SF target -- each class is its own kernel variant
        slabs = [sl for sls in (self.cpml.slabs.values() if self.use_cpml else ()) for sl in sls]
        cuts = []
        for a in range(3):
            lo_e = max([sl.gbox[1][a] for sl in slabs if sl.axis == a and sl.side == 0], default=None)
            hi_s = min([sl.gbox[0][a] for sl in slabs if sl.axis == a and sl.side == 1], default=None)
            cuts.append([c for c in ((lo_e + T + 1) if lo_e is not None else None,
                                     (hi_s - T - 1) if hi_s is not None else None) if c is not None])
        pieces = [b for b in box_subtract(alloc, K) if not box_empty(b)]
        for a in range(3):
            nxt = []
            for b in pieces:
                edges = sorted({b[0][a], b[1][a]} | {c for c in cuts[a] if b[0][a] < c < b[1][a]})
                for lo_, hi_ in zip(edges, edges[1:]):
                    lo, hi = list(b[0]), list(b[1])
                    lo[a], hi[a] = lo_, hi_
                    nxt.append((tuple(lo), tuple(hi)))
            pieces = nxt
        classed = []
        for b in pieces:
            g = grow(b, T + 1)
            ax = 0
            for sl in slabs:
                if not box_empty(box_intersect(g, sl.gbox)):
                    ax |= 1 << sl.axis
            tf = bool(cfg.use_tfsf and self._tfsf_targets_in(dom.to_local(g)))
            classed.append((b, ax | (8 if tf else 0)))
        shell = [(dom.to_local(b), c) for b, c in _merge_pieces(classed)]
        upd = {c: self.local_box(c, alloc) for c in self.comps}
        return {"T": T, "v3": True, "core": [dom.to_local(K)], "shell": shell, "upd": upd,
                "core_cells": box_volume(K)}

    def _hybrid4_plan(self, p3):
        """Mixed shell: the core and the x / y faces (one CPML axis in their
        cone: psi through LDS, csrc/tb3d_mr.h LPS, + in-kernel TF/SF) take
        blocked launches; the rest -- the z slabs over the whole x / y
        extent and the x-y edge columns -- is stepped in place in F over
        windows grown ``T - s`` cells into the blocked pieces at step ``s``
        (the band rule of ``_hybrid_plan``), then copied to F_alt.  The
        blocked faces' psi (written to the other copy) is copied back over
        the band's in-place psi afterwards."""
        T = p3["T"]
        dom = self.domain
        alloc = dom.allocated_global()
        # geometry: the x faces (x outside the core's range, y / z inside it)
        # and the y faces (x / z inside, y outside) are blocked; the z slabs
        # (whole x / y extent) and the x-y edge columns are stepped -- few,
        # large stepped windows
        K = dom.to_global(p3["core"][0])
        faces = []
        for a in (0, 1):
            for lo_, hi_ in ((alloc[0][a], K[0][a]), (K[1][a], alloc[1][a])):
                if hi_ <= lo_:
                    continue
                lo, hi = list(K[0]), list(K[1])
                lo[a], hi[a] = lo_, hi_
                if a == 1:
                    lo[0], hi[0] = K[0][0], K[1][0]
                faces.append(((tuple(lo), tuple(hi)), a))
        slabs = [sl for sls in self.cpml.slabs.values() for sl in sls]
        blocked = []
        for b, a in faces:
            g = (tuple(b[0][d] - T - 1 for d in range(3)), tuple(b[1][d] + T + 1 for d in range(3)))
            ax = 0
            for sl in slabs:
                if not box_empty(box_intersect(g, sl.gbox)):
                    ax |= 1 << sl.axis
            if ax != 1 << a:
                return p3  # a face's cone reaches another axis's slab: the blocked plan
            tf = bool(self.cfg.use_tfsf and self._tfsf_targets_in(dom.to_local(g)))
            blocked.append((dom.to_local(b), ax | (8 if tf else 0)))
        rest = [alloc]
        for b in [K] + [dom.to_global(f) for f, _ in blocked]:
            rest = [r for q in rest for r in (box_subtract(q, b) if not box_empty(box_intersect(q, b)) else [q])
                    if not box_empty(r)]
        stepped = [(dom.to_local(r), 7) for r in rest]
        if not stepped:
            return p3

        def grow(b, n):
            return (tuple(b[0][d] - n for d in range(3)), tuple(b[1][d] + n for d in range(3)))

        def disjoint_union(boxes):
            out = []
            for b in boxes:
                pieces = [box_intersect(b, alloc)]
                for o in out:
                    nxt = []
                    for q in pieces:
                        nxt += [r for r in box_subtract(q, o) if not box_empty(r)] if not box_empty(
                            box_intersect(q, o)) else [q]
                    pieces = nxt
                out += [q for q in pieces if not box_empty(q)]
            return out

        sg = [dom.to_global(b) for b, _ in stepped]
        # step s (0-based) advances the stepped pieces plus a band T - s deep
        windows = [disjoint_union([grow(b, T - s) for b in sg]) for s in range(T)]
        fixes = []
        for b, cls in blocked:
            a = {1: 0, 2: 1}.get(cls & 7)
            if a is None:
                continue
            for c in self.comps:
                for sl in self.cpml.slabs[c]:
                    if sl.axis != a:
                        continue
                    i = box_intersect(b, sl.lbox)
                    if not box_empty(i):
                        fixes.append((sl, tuple(slice(i[0][d] - sl.lbox[0][d], i[1][d] - sl.lbox[0][d])
                                                for d in range(3))))
        self._tfsf_once = bool(self.cfg.use_tfsf)
        return dict(p3, v3=False, v4=True, shell=blocked, windows=windows, copy=[b for b, _ in stepped],
                    psi_fix=fixes)

    def _hybrid4_step(self, T: int) -> None:
        hp = self.hybrid
        if T != hp["T"]:
            for _ in range(T):
                self.step()
            return
        srcs = self._pass_sources(self.t, T)
        for p in range(self.planes):
            line0 = None
            if self.cfg.use_tfsf:
                # the blocked launches' g tables advance the incident line T
                # steps; the stepped windows advance it again from here
                line0 = (self.einc[p].clone(), self.hinc[p].clone())
            tf = self._tfsf_pass(p, T)
            cp = self.cpml.host_table(p)
            P, Q = self.F[p], self.F_alt[p]
            with self.prof.phase("blocked-core"):
                for ob in hp["core"]:
                    self.ops.tb_step(P, Q, hp["upd"], ob, self.cb, T, srcs[p])
                for ob, cls in hp["shell"]:
                    cax = cls & 7
                    self.ops.tb_step(P, Q, hp["upd"], ob, self.cb, T, srcs[p], tfsf=tf if cls & 8 else None,
                                     cpml=cp if cax else None, cpml_axes=cax)
            if line0 is not None:
                self.einc[p].copy_(line0[0])
                self.hinc[p].copy_(line0[1])
        for s in range(T):
            self.step(hp["windows"][s])
        with self.prof.phase("shell-copy"):
            for p in range(self.planes):
                src = [self.F[p][c] for c in self.comps]
                dst = [self.F_alt[p][c] for c in self.comps]
                for b in hp["copy"]:
                    self.ops.copy_box(src, dst, b)
                # the blocked face pieces' psi (level T, other copy) over the
                # stepped band's in-place values
                for sl, sub in hp["psi_fix"]:
                    sl.psi[p][sub] = sl.psi_alt[p][sub]
        for p in range(self.planes):
            self.F[p], self.F_alt[p] = self.F_alt[p], self.F[p]

    def _hybrid3_step(self, T: int) -> None:
        hp = self.hybrid
        if T != hp["T"]:
            tails = self.__dict__.setdefault("_hybrid3_tails", {})
            if T not in tails:
                tails[T] = self._hybrid3_plan(T)
            hp = tails[T]
            if hp is None:
                for _ in range(T):
                    self.step()
                return
        srcs = self._pass_sources(self.t, T)
        for p in range(self.planes):
            tf = self._tfsf_pass(p, T)
            cp = self.cpml.host_table(p) if self.use_cpml else None
            P, Q = self.F[p], self.F_alt[p]
            with self.prof.phase("blocked-core"):
                for ob in hp["core"]:
                    self.ops.tb_step(P, Q, hp["upd"], ob, self.cb, T, srcs[p])
            with self.prof.phase("blocked-shell"):
                for ob, cls in hp["shell"]:
                    cax = cls & 7
                    self.ops.tb_step(P, Q, hp["upd"], ob, self.cb, T, srcs[p], tfsf=tf if cls & 8 else None,
                                     cpml=cp if cax else None, cpml_axes=cax)
            if self.use_cpml:
                self.cpml.flip(p)
            self.F[p], self.F_alt[p] = Q, P
        self.t += T
        if self.cfg.check_finite and (self.t // max(1, self.cfg.finite_check_step)
                                      != (self.t - T) // max(1, self.cfg.finite_check_step)):
            self.check_finite()

    # ------------------------------------------------ hybrid, single-pass shell
    def _hybrid2_ok(self) -> bool:
        """Runs whose shell the fused single-step shell kernel can advance
        (csrc/yee3d_shell.hip): 3D serial runs with CPML, UPML (D/B form),
        dispersive (Drude / Lorentz) boxes inside the all-sigma-zero core, or
        plane waves in an open box; uniform background media (scalar
        coefficients); plane waves through the TF/SF tables.  Opt-in
        (``hybrid_shell`` = single-pass): measured at 512^3 (round 3,
        ``tools/shell_micro.py``, ``profiles/configs_r3.md``) the fused
        single-step shell kernel is issue-bound on the thin shell faces
        (20-54 Gcells/s, a 0.2 ms floor per two-axis edge launch) and the whole
        runs are 1.7-1.9x slower than the stepped shell (CPML + TF/SF 48.5k
        vs 84.7k Mcells/s), so ``auto`` keeps the stepped shell."""
        cfg = self.cfg
        mode = getattr(cfg, "hybrid_shell", "auto")
        if mode != "single-pass" or not hasattr(self.ops, "shell_step"):
            return False
        if cfg.scheme != "3d" or self.halo is not None or cfg.use_amp_mode:
            return False
        upml = cfg.use_pml and self.use_upml_chain
        if not ((cfg.use_pml and self.use_cpml) or upml or (not cfg.use_pml and (cfg.use_tfsf or
                                                                               cfg.use_metamaterials))):
            return False
        if self.use_upml_chain:
            for c in self.comps:
                st = self.upml[c]
                if st["prof"]["cell"] is not None or ("plain" in st and st["plain"]["prof"]["cell"] is not None):
                    return False
        if self.ops.name == "hip" and (self.dtype != torch.float32 or self.domain.shape[2] % 4 != 0):
            return False
        if any(getattr(self.cb[c], "cell", None) is not None for c in self.comps):
            return False  # per-cell coefficients: the stepped shell
        # the kernel shares one slab geometry per (kind, axis): the terms of
        # a kind along y / z must have the same psi slab ranges
        by = {}
        for c, slabs in (self.cpml.slabs.items() if self.use_cpml else ()):
            for sl in slabs:
                key = (c[0], sl.axis, sl.side)
                rng = (sl.lbox[0][sl.axis], sl.lbox[1][sl.axis])
                if by.setdefault(key, rng) != rng:
                    return False
        return True

    def _hybrid2_regions(self) -> bool:
        """Region-local UPML / dispersive state of the single-pass shell
        (models/upml.py); False when the run does not fit it."""
        cfg = self.cfg
        self.upml_regions = None
        self.drude_box = None
        try:
            if cfg.use_pml and self.use_upml_chain:
                from .upml import UPMLRegions
                self.upml_regions = UPMLRegions(self)
            if cfg.use_metamaterials:
                from .upml import DrudeBox
                self.drude_box = DrudeBox(self)
                if self.upml_regions is not None:
                    I, B = self.upml_regions.core, self.drude_box.box
                    if box_intersect(I, B) != B:
                        raise ValueError("dispersive box reaches an absorbing layer")
        except ValueError:
            self.upml_regions = None
            self.drude_box = None
            return False
        return True

    def _hybrid2_plan(self, T: int):
        """Blocked core + single-pass shell with shrinking windows.

        The core -- cells at least ``T + 2`` from every absorbing-layer cell,
        TF/SF target and dispersive cell -- takes one ``T``-step blocked pass
        of the plain kernel (``K``, minus the dispersive box grown by
        ``T + 2``).  The shell -- everything else -- takes ``T`` fused single
        steps (``ops.shell_step``), step ``s`` over ``alloc`` minus the core
        shrunk by ``T - s`` on its inner sides: each step's window is one cell
        deeper into the core than the next needs, so every shell value is
        exact without a stale band (the deep-halo rule, reference
        ``ParallelGrid.cpp:2365-2489``).  Single-step passes read one buffer
        and write another, so the shell ping-pongs between ``F_alt`` and a
        third buffer while the core reads the untouched ``F``.  Each window
        is cut at the absorbing-slab and dispersive-box boundaries into boxes
        tagged with the kernel's specialisation (axes bits; 8 = dispersive)."""
        cfg = self.cfg
        size = cfg.size
        m = T + 2
        lo, hi = [0, 0, 0], list(size)
        for a in range(3):
            edge = self.layout.pml_size[a] if cfg.use_pml else 0
            if cfg.use_tfsf:
                edge = max(edge, cfg.tfsf_size[a] + 1)
            if edge > 0:
                lo[a], hi[a] = edge + m, size[a] - edge - m
        K = (tuple(lo), tuple(hi))
        if box_empty(K):
            return None
        dom = self.domain
        alloc = dom.allocated_global()
        dbox = getattr(self, "drude_box", None)
        Dm = None
        couts = [K]
        if dbox is not None:
            B = dom.to_global(dbox.box)
            Dm = box_intersect((tuple(B[0][d] - m for d in range(3)), tuple(B[1][d] + m for d in range(3))), K)
            if not box_empty(Dm):
                couts = [b for b in box_subtract(K, Dm) if not box_empty(b)]
        core_cells = sum(box_volume(b) for b in couts)
        if core_cells < 0.25 * size[0] * size[1] * size[2]:
            return None

        def grow(b, n):
            return (tuple(b[0][d] - n for d in range(3)), tuple(b[1][d] + n for d in range(3)))

        # every irregular cell must stay T + 1 clear of the core (its
        # dependency cone; also keeps the host-side TF/SF additions to the
        # shell's input buffer out of what the core pass reads)
        ureg = getattr(self, "upml_regions", None)
        for ob in couts:
            g = grow(ob, T + 1)
            for slabs in (self.cpml.slabs.values() if self.use_cpml else ()):
                for sl in slabs:
                    if not box_empty(box_intersect(g, sl.gbox)):
                        return None
            lg = dom.to_local(g)
            if ureg is not None and box_intersect(lg, ureg.core) != box_intersect(lg, dom.to_local(alloc)):
                return None  # the core's cone must see no UPML cell
            if dbox is not None and not box_empty(box_intersect(lg, dbox.box)):
                return None
            if cfg.use_tfsf and self._tfsf_targets_in(lg):
                return None
        if cfg.use_tfsf and (ureg is not None or dbox is not None):
            # E-form corrections only where the update is the plain one
            if ureg is not None and self._tfsf_targets_in(ureg.core, outside=True):
                return None
            if dbox is not None and self._tfsf_targets_in(grow(dbox.box, 1)):
                return None
        cuts = self._cpml_cuts()

        def shrink_inner(b, n):
            return (tuple(b[0][d] + (n if b[0][d] > 0 else 0) for d in range(3)),
                    tuple(b[1][d] - (n if b[1][d] < size[d] else 0) for d in range(3)))

        windows = []
        for st in range(1, T + 1):
            d = T - st
            Kd = shrink_inner(K, d)
            pieces = []
            for b in box_subtract(alloc, Kd):
                if not box_empty(b):
                    # the face normal of this part of the shell (the axes
                    # along which it lies wholly outside the hole) is not cut
                    normal = [a for a in range(3) if b[1][a] <= Kd[0][a] or b[0][a] >= Kd[1][a]]
                    pieces += _cut_pieces(dom.to_local(b), cuts, keep=normal)
            if Dm is not None and not box_empty(Dm):
                inner = box_intersect(grow(Dm, d), Kd)
                if not box_empty(inner):
                    pieces += _cut_box(dom.to_local(inner), dbox.box)
            windows.append(_merge_pieces(pieces))
        upd = {c: self.local_box(c, alloc) for c in self.comps}
        return {"T": T, "v2": True, "core": [dom.to_local(b) for b in couts], "windows": windows, "upd": upd,
                "core_cells": core_cells}

    def _tfsf_targets_in(self, lbox: Box, outside: bool = False) -> bool:
        """True when some TF/SF target lies inside the local box (``outside``:
        outside it)."""
        for c in self.comps:
            for tab in self.tfsf[c]:
                if tab.n == 0:
                    continue
                ijk = tab.ijk.view(-1, 3)
                inside = torch.ones(ijk.shape[0], dtype=torch.bool, device=ijk.device)
                for d in range(3):
                    inside &= (ijk[:, d] >= lbox[0][d]) & (ijk[:, d] < lbox[1][d])
                if bool((~inside if outside else inside).any()):
                    return True
        return False

    def _cpml_cuts(self):
        """Per axis (low cut, high cut) of the CPML slabs, local indices:
        cells below the low cut or at / above the high cut may carry that
        axis's psi terms (None: no slab along the axis)."""
        cuts = [None, None, None]
        n = self.domain.shape
        ureg = getattr(self, "upml_regions", None)
        if ureg is not None:
            # the D boxes: everything outside the all-sigma-zero core
            I = ureg.core
            return [(I[0][a], I[1][a]) if (I[0][a] > 0 or I[1][a] < n[a]) else None for a in range(3)]
        for slabs in (self.cpml.slabs.values() if self.use_cpml else ()):
            for sl in slabs:
                a = sl.axis
                b = self.domain.to_local(sl.gbox)
                lo_c, hi_c = cuts[a] if cuts[a] is not None else (0, n[a])
                if sl.side == 0:
                    lo_c = max(lo_c, b[1][a])
                else:
                    hi_c = min(hi_c, b[0][a])
                cuts[a] = (lo_c, hi_c)
        return cuts

    def _tfsf_kind(self, kind: str, p: int, F) -> None:
        """Every TF/SF correction of ``kind`` on plane ``p``'s fields ``F``
        (coefficient Cb / Db, incident H for E targets, E for H targets), in
        as few launches as the backend allows."""
        comps = self.e_comps if kind == "E" else self.h_comps
        inc = self.hinc[p] if kind == "E" else self.einc[p]
        whole = ((0, 0, 0), tuple(self.domain.shape))
        if hasattr(self.ops, "tfsf_apply_many"):
            self.ops.tfsf_apply_many([(F[c], tab) for c in comps for tab in self.tfsf[c]], inc)
        else:
            for c in comps:
                for tab in self.tfsf[c]:
                    self.ops.tfsf_apply(F[c], tab, inc, whole)

    def _hybrid2_step(self, T: int) -> None:
        hp = self.hybrid
        if T != hp["T"]:
            # a short tail pass: its own (shallower) windows
            hp = self.__dict__.setdefault("_hybrid2_tails", {}).get(T)
            if hp is None:
                hp = self._hybrid2_plan(T)
                self._hybrid2_tails[T] = hp
            if hp is None:
                for _ in range(T):
                    self.step()
                return
        srcs = self._pass_sources(self.t, T)
        tfsf = self.cfg.use_tfsf
        kappa = getattr(self.cfg, "cpml_kappa_max", 1.0) != 1.0
        for p in range(self.planes):
            P, Q, Z = self.F[p], self.F_alt[p], self.F_3[p]
            cur = P
            with self.prof.phase("shell"):
                for st in range(1, T + 1):
                    out = Q if st % 2 == 1 else Z
                    t = self.t + st - 1
                    if tfsf:
                        # incident line E half step, then the E corrections
                        # added to the INPUT (additive: E + Cb g + Cb curl)
                        self.ops.inc_step_e(self.einc[p], self.hinc[p], self.inc_ce, self.source_value(t, p))
                        self._tfsf_kind("E", p, cur)
                    sv = None if srcs[p] is None else srcs[p][st - 1]
                    cp = self.cpml.shell_arg(p, self.ops) if self.use_cpml else None
                    ureg = getattr(self, "upml_regions", None)
                    pieces = hp["windows"][st - 1]
                    dbox = getattr(self, "drude_box", None)
                    self.ops.shell_step(cur, out, hp["upd"], [b for b, _ in pieces], [a for _, a in pieces],
                                        self.cb, sv, cpml=cp, kappa=kappa,
                                        upml=None if ureg is None else ureg.shell_arg(p, self.ops),
                                        drude=None if dbox is None else dbox.shell_arg(p, self.ops))
                    if self.use_cpml:
                        self.cpml.flip(p)
                    if ureg is not None:
                        ureg.flip(p)
                    if dbox is not None:
                        dbox.rotate(p)
                    if tfsf:
                        # incident line H half step, H corrections on the OUTPUT
                        self.ops.inc_step_h(self.einc[p], self.hinc[p], self.inc_ch)
                        self._tfsf_kind("H", p, out)
                    cur = out
            with self.prof.phase("blocked-core"):
                for ob in hp["core"]:
                    self.ops.tb_step(P, cur, hp["upd"], ob, self.cb, T, srcs[p])
            rest = [b for b in (Q, Z) if b is not cur]
            self.F[p], self.F_alt[p], self.F_3[p] = cur, P, rest[0]
        self.t += T
        if self.cfg.check_finite and (self.t // max(1, self.cfg.finite_check_step)
                                      != (self.t - T) // max(1, self.cfg.finite_check_step)):
            self.check_finite()

    def _hybrid_plan(self, T: int):
        dom = self.domain
        cfg = self.cfg
        size = cfg.size
        alloc = dom.allocated_global()
        # core margin to every irregular cell: T + 1 clears the stencil reach
        # of a T-step pass (checked below; T + 2 when a staggered component's
        # irregular box sticks out one cell further)
        for m in (T + 1, T + 2):
            plan = self._hybrid_plan_m(T, m)
            if plan is not None:
                return plan
        return None

    def _hybrid_plan_m(self, T: int, m: int):
        dom = self.domain
        cfg = self.cfg
        size = cfg.size
        alloc = dom.allocated_global()
        # TF/SF faces stay in the stepped shell: the blocked kernel's TF/SF
        # variant runs at about half the plain kernel's rate
        # (profiles/tfsf_cpml_r2.md), more than the shell it would save
        in_kernel_tfsf = False
        lo, hi = [0, 0, 0], list(size)
        act = [self.layout.active(a) for a in range(3)]  # 2D: z is one cell, never cut
        for a in range(3):
            if not act[a]:
                continue
            edge = 0
            if cfg.use_pml:
                edge = max(edge, self.layout.pml_size[a])
            if cfg.use_tfsf and not in_kernel_tfsf:
                edge = max(edge, cfg.tfsf_size[a] + 1)
            if edge > 0:
                lo[a], hi[a] = edge + m, size[a] - edge - m
            # else: nothing irregular along this axis but the domain border,
            # which the blocked kernel handles itself (a Drude sphere in
            # vacuum without PML: the core reaches the faces)
        K = (tuple(lo), tuple(hi))
        if box_empty(K):
            return None
        # dispersive boxes (chain boxes off the domain border) are cut out of the core
        disp = []
        if cfg.use_metamaterials and self.use_upml_chain:
            for c in self.comps:
                b = self._bbox_global(self.upml[c].get("drude_active"))
                if not box_empty(b):
                    disp.append(b)
        D = None
        for b in disp:
            D = b if D is None else (tuple(min(D[0][d], b[0][d]) for d in range(3)),
                                     tuple(max(D[1][d], b[1][d]) for d in range(3)))

        def grow(b, n):
            return (tuple(b[0][d] - (n if act[d] else 0) for d in range(3)),
                    tuple(b[1][d] + (n if act[d] else 0) for d in range(3)))

        if D is not None:
            Dm = box_intersect(grow(D, m), K)
            couts = [b for b in box_subtract(K, Dm) if not box_empty(b)] if not box_empty(Dm) else [K]
        else:
            Dm = None
            couts = [K]
        couts = [b for b in couts if not box_empty(b)]
        core_cells = sum(box_volume(b) for b in couts)
        if core_cells < 0.25 * size[0] * size[1] * size[2]:
            return None
        # verify: no irregular cell within T + 1 of an output box
        irregular = []
        if getattr(self, "chain_regions", None) is not None:
            for kind in ("E", "H"):
                for r, _ in self.chain_regions[kind]["chain"]:
                    irregular += [b for b in r.values() if not box_empty(b)]
        if self.use_cpml:
            for slabs in self.cpml.slabs.values():
                irregular += [sl.gbox for sl in slabs if not box_empty(sl.gbox)]
        if self.use_upml_chain and getattr(self, "chain_regions", None) is None:
            if cfg.scheme == "3d":
                return None  # 3D UPML without region split: every cell runs the chain
            # 2D: the per-component UPML update runs on every cell; away from
            # the PML slabs (sigma = 0) it reduces to the plain Yee update to
            # round-off, and the core is cut T + 2 clear of the slabs above
            for a in range(3):
                if act[a] and cfg.use_pml and self.layout.pml_size[a] > 0:
                    n = self.layout.pml_size[a]
                    irregular.append(((0, 0, 0), tuple(n if d == a else size[d] for d in range(3))))
                    irregular.append((tuple(size[a] - n if d == a else 0 for d in range(3)), tuple(size)))
        for ob in couts:
            g = grow(ob, T + 1)
            if any(not box_empty(box_intersect(g, b)) for b in irregular):
                return None
            if cfg.use_tfsf and not in_kernel_tfsf:
                lg = dom.to_local(g)
                for c in self.comps:
                    for tab in self.tfsf[c]:
                        if tab.n == 0:
                            continue
                        ijk = tab.ijk.view(-1, 3)
                        inside = torch.ones(ijk.shape[0], dtype=torch.bool, device=ijk.device)
                        for d in range(3):
                            inside &= (ijk[:, d] >= lg[0][d]) & (ijk[:, d] < lg[1][d])
                        if bool(inside.any()):
                            return None
        if self.halo is not None:
            # decomposed: each rank's core is its owned part of the global core
            couts = [box_intersect(b, dom.owned_global()) for b in couts]
            couts = [b for b in couts if not box_empty(b)]
        def shrink_inner(b, n):
            # shrink by n only the sides that lie inside the domain (a side
            # on the domain border has no shell beyond it)
            return (tuple(b[0][d] + (n if act[d] and b[0][d] > 0 else 0) for d in range(3)),
                    tuple(b[1][d] - (n if act[d] and b[1][d] < size[d] else 0) for d in range(3)))

        def shell_windows(d):
            # everything but the core cells deeper than d inside it
            Kd = shrink_inner(K, d)
            if box_empty(Kd):
                return None
            ws = [b for b in box_subtract(alloc, Kd) if not box_empty(b)]
            if Dm is not None and not box_empty(Dm):
                inner = box_intersect(grow(Dm, d), Kd)
                if not box_empty(inner):
                    ws.append(inner)
            return ws

        # step s of the pass (0-based) advances the shell plus a band T - s
        # deep into the core: the stale core beyond the band corrupts one
        # more band cell per step, so after step s the band is exact to depth
        # T - 1 - s, and after the last step the shell itself (depth 0)
        shells = [shell_windows(T - s) for s in range(T)]
        if shells[0] is None:
            return None
        copy_boxes = [b for b in box_subtract(alloc, K) if not box_empty(b)]
        if Dm is not None and not box_empty(Dm):
            # (a decomposed run's dispersive box can reach past this rank's
            # allocation: clip before turning it into local slices)
            dma = box_intersect(Dm, alloc)
            if not box_empty(dma):
                copy_boxes.append(dma)
        # TF/SF corrections once per half step, unless a component's TF/SF
        # targets reach into a UPML chain box (D-form corrections there)
        self._tfsf_once = bool(cfg.use_tfsf)
        if self.use_upml_chain and getattr(self, "chain_regions", None) is None:
            self._tfsf_once = False  # 2D UPML: the per-window chain applies its D-form corrections
        if cfg.use_tfsf and getattr(self, "chain_regions", None) is not None:
            for kind in ("E", "H"):
                for r, _ in self.chain_regions[kind]["chain"]:
                    for c, b in r.items():
                        tb = self.tfsf_bbox.get(c)
                        if tb is not None and not box_empty(b) and not box_empty(box_intersect(dom.to_local(b), tb)):
                            self._tfsf_once = False
        upd = {c: self.local_box(c, alloc) for c in self.comps}
        return {"T": T, "core": [dom.to_local(b) for b in couts], "shell": shells[0], "shells": shells,
                "copy": [dom.to_local(b) for b in copy_boxes], "upd": upd, "core_cells": core_cells,
                "cut_cells": box_volume(Dm) if Dm is not None else 0}

    def _tfsf_pass(self, p: int, T: int, level0: int = 0):
        """In-kernel TF/SF of a blocked pass starting at step ``self.t`` on
        plane ``p``: advances the plane's incident line ``T`` steps and returns
        the ``tfsf`` argument of ``ops.tb_step`` (None without in-kernel
        TF/SF)."""
        sets = getattr(self, "tfsf_sets", None)
        if not self.cfg.use_tfsf or sets is None:
            return None
        vals = [self.source_value(self.t + l, p) for l in range(T)]
        g = self.ops.tfsf_pass(self.einc[p], self.hinc[p], self.inc_ce, self.inc_ch, vals, self.t + T + 2, sets,
                               slot=p)
        return (sets, g, level0)

    def _pass_sources(self, t: int, T: int):
        """Per plane: the hard point source's value at each of the pass's T
        E half steps (None without a point source on this rank)."""
        srcs = []
        for p in range(self.planes):
            sp = None
            if self.point_source is not None and self.point_source[1] is not None:
                comp, li, _ = self.point_source
                sp = [(comp, li, self.source_value(t + l, p)) for l in range(T)]
            srcs.append(sp)
        return srcs

    def _hybrid_step(self, T: int) -> None:
        if self.hybrid.get("v4"):
            self._hybrid4_step(T)
            return
        if self.hybrid.get("v3"):
            self._hybrid3_step(T)
            return
        if self.hybrid.get("v2"):
            self._hybrid2_step(T)
            return
        hp = self.hybrid
        srcs = self._pass_sources(self.t, T)
        side = None
        core_now, core_later = hp["core"], []
        if self.halo is not None:
            # one T-deep exchange of every state array (aux included) feeds the
            # core pass and the deep-halo shell steps; step() skips its own.
            # It runs on the side stream while the core cells at least T from
            # every neighbour (no fresh ghost in their dependency cone) are
            # advanced; the rest of the core and the stepped shell follow.
            core_now, core_later = self._hybrid_core_split(T)
            side = self._fork_side_stream()
            self._mark("start")
            with self.prof.phase("halo-deep"):
                self.halo.exchange_all(self, stream=side)
            self._deep_fresh = True
            # the fresh ghosts are T deep: the shell steps of this pass use
            # the deep-halo windows from sub-step 0, whatever an earlier
            # shorter pass (periodic work, a tail) left behind
            self.sub_step = 0
        tfs = []
        for p in range(self.planes):
            tf = None
            if self.cfg.use_tfsf and self.hybrid.get("tfsf_in_core"):
                # the pass kernel advances the incident line for the core;
                # the stepped shell advances it again from the same state
                line0 = (self.einc[p].clone(), self.hinc[p].clone())
                tf = (self._tfsf_pass(p, T), line0)
            tfs.append(tf)

        def core(boxes):
            for p in range(self.planes):
                tf = tfs[p][0] if tfs[p] is not None else None
                for ob in boxes:
                    if tf is not None:
                        self.ops.tb_step(self.F[p], self.F_alt[p], hp["upd"], ob, self.cb, T, srcs[p], tfsf=tf)
                    else:
                        self.ops.tb_step(self.F[p], self.F_alt[p], hp["upd"], ob, self.cb, T, srcs[p])

        with self.prof.phase("blocked-core"):
            core(core_now)
        if self.halo is not None:
            self._mark("interior")
            self._join_side(side)
            self._mark("wait")
            with self.prof.phase("blocked-core"):
                core(core_later)
        for p in range(self.planes):
            if tfs[p] is not None:
                self.einc[p].copy_(tfs[p][1][0])
                self.hinc[p].copy_(tfs[p][1][1])
        for s in range(T):
            self.step(hp["shells"][s])
        if self.halo is not None:
            self._mark("end")
        with self.prof.phase("shell-copy"):
            for p in range(self.planes):
                src = [self.F[p][c] for c in self.comps]
                dst = [self.F_alt[p][c] for c in self.comps]
                for b in hp["copy"]:
                    self.ops.copy_box(src, dst, b)
        for p in range(self.planes):
            self.F[p], self.F_alt[p] = self.F_alt[p], self.F[p]

    def _hybrid_core_split(self, T: int):
        """(core boxes that need no fresh ghost, the rest) of a decomposed
        hybrid pass, local indices: the interior is the owned box shrunk by
        ``T`` on every side with a neighbour (a T-step pass reads T cells
        beyond its output box), the rest are the slabs between it and the
        rank border, which wait for the exchange."""
        cache = self.__dict__.setdefault("_hybrid_split_cache", {})
        if T in cache:
            return cache[T]
        dom = self.domain
        lo, hi = list(dom.lo), list(dom.hi)
        for a in range(3):
            if dom.has_low(a):
                lo[a] += T
            if dom.has_high(a):
                hi[a] -= T
        inner = dom.to_local((tuple(lo), tuple(hi)))
        now, later = [], []
        for b in self.hybrid["core"]:
            i = box_intersect(b, inner)
            if not box_empty(i):
                now.append(i)
                later += [r for r in box_subtract(b, i) if not box_empty(r)]
            else:
                later.append(b)
        cache[T] = (now, later)
        return cache[T]

    # ----------------------------------------------------- plain blocking
    def _tb_regions(self, T: int):
        """(update boxes, [output boxes]) of a blocked pass, local indices.
        Serial: one output box (the whole domain).  Decomposed: first the
        interior (owned cells at least ``T`` from every neighbour -- needs no
        fresh ghost), then the ``T``-thick shell slabs peeled off axis by axis
        (disjoint), which run once the ghosts have arrived."""
        cache = self.__dict__.setdefault("_tb_regions_cache", {})
        if T in cache:
            return cache[T]
        dom = self.domain
        upd = {c: self.local_box(c, dom.allocated_global()) for c in self.comps}
        lo, hi = list(dom.lo), list(dom.hi)
        shells = []
        for a in range(3):
            if dom.has_low(a):
                slo, shi = list(lo), list(hi)
                shi[a] = lo[a] + T
                shells.append((tuple(slo), tuple(shi)))
                lo[a] += T
            if dom.has_high(a):
                slo, shi = list(lo), list(hi)
                slo[a] = hi[a] - T
                shells.append((tuple(slo), tuple(shi)))
                hi[a] -= T
        outs = [dom.to_local((tuple(lo), tuple(hi)))] + [dom.to_local(b) for b in shells if not box_empty(b)]
        cache[T] = (upd, outs)
        return cache[T]

    def _tb_step(self, T: int) -> None:
        """``T`` steps in one blocked pass.  Decomposed runs overlap the
        T-deep ghost exchange (side stream) with the interior pass and run the
        shell slabs after it."""
        upd, outs = self._tb_regions(T)
        srcs = self._pass_sources(self.t, T)
        side = self._fork_side_stream() if self.halo is not None else None
        tfs = [self._tfsf_pass(p, T) for p in range(self.planes)] if self.cfg.use_tfsf else [None] * self.planes
        if self.halo is not None:
            self._mark("start")
        for p in range(self.planes):
            if not box_empty(outs[0]):
                with self.prof.phase("blocked-interior" if self.halo is not None else "blocked"):
                    if tfs[p] is not None:
                        self.ops.tb_step(self.F[p], self.F_alt[p], upd, outs[0], self.cb, T, srcs[p], tfsf=tfs[p])
                    else:
                        self.ops.tb_step(self.F[p], self.F_alt[p], upd, outs[0], self.cb, T, srcs[p])
        if self.halo is not None:
            self._mark("interior")
            if side is not None and self.prof.enabled:
                with torch.cuda.stream(side):
                    with self.prof.phase("halo-overlapped"):
                        self.halo.exchange_all(self)
            else:
                with self.prof.phase("halo-overlapped"):
                    self.halo.exchange_all(self, stream=side)
            self._join_side(side)
            self._mark("wait")
            with self.prof.phase("blocked-shells"):
                for ob in outs[1:]:
                    for p in range(self.planes):
                        if tfs[p] is not None:
                            self.ops.tb_step(self.F[p], self.F_alt[p], upd, ob, self.cb, T, srcs[p], tfsf=tfs[p])
                        else:
                            self.ops.tb_step(self.F[p], self.F_alt[p], upd, ob, self.cb, T, srcs[p])
            self._mark("end")
        for p in range(self.planes):
            self.F[p], self.F_alt[p] = self.F_alt[p], self.F[p]
        self.t += T
        if self.cfg.check_finite and (self.t // max(1, self.cfg.finite_check_step)
                                      != (self.t - T) // max(1, self.cfg.finite_check_step)):
            self.check_finite()
