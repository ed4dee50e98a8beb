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

import os

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
# (1024^3: T=5 281-289k vs T=4 260-263k Mcells/s on one GPU; decomposed
# T=4, whose ghosts and shells are thinner: tools/decomp_cost.py at 1024^3,
# profiles/decomp_r6.md -- 2 ranks 266-298k vs 261-263k, 4 ranks 232-249k vs
# 225-238k, 8 ranks 240-246k vs 202-207k per GPU).  Per-cell
# coefficients of one kind (dielectric or magnetic scenes) run the sparse
# multi-row kernel with an LDS ring of coefficient planes (512^3 eps sphere:
# T=3 160k, 4 188k, 5 203k Mcells/s); per-cell E AND H keep the planes in
# registers, spill-free only to T=2.
F32_AUTO_STEPS = 5
F32_AUTO_STEPS_MANY_RANKS = 4
F32_AUTO_STEPS_PERCELL_BOTH = 2
# plain runs with in-kernel TF/SF (TfsfSets): 512^3 vacuum + TF/SF T=4 127k,
# T=5 86k Mcells/s with the round-4 slot form (the TF/SF variant spilled at T=5)
F32_AUTO_STEPS_TFSF = 4
# longest pass of the TF/SF variant (yee3d_tb.hip launch_tb_mr_sel: T <= 5)
TFSF_MAX_STEPS = 5
# steps per pass with the Drude box inside the blocked passes (its variant
# holds T - 1 levels of dispersive state in registers: T <= 5).  512^3 Drude
# sphere r = 128 (profiles/drude_blk_r5.md): T = 3 / 4 / 5 131.6k / 165-170k /
# 155-157k Mcells/s without PML, 66.6k / 73.6-75.3k / 74.6-75.4k with UPML
DRUDE_AUTO_STEPS = 4



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
    return F32_AUTO_STEPS if world <= 1 else F32_AUTO_STEPS_MANY_RANKS


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
    drude_blk = None   # the Drude box inside the blocked passes (_plan_drude_blk), None: off
    _drude_plan = None
    _drude_glob = None
    # the Drude pass of a serial hybrid pass on a stream of its own, next to the shell steps (when its
    # cone is clear of the shell); FDTD3D_DRUDE_SIDE=0: in order (A/B)
    drude_side = os.environ.get("FDTD3D_DRUDE_SIDE", "1") != "0"  # (T, global Drude box) of the pass form every rank takes (None: off)
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

    # ------------------------------------------------- Drude box, blocked
    def _plan_drude_blk(self):
        """The dispersive box inside the blocked passes (csrc/tb3d_mr.h
        DrDev): every pass runs the plain blocked kernel over the core, then
        the Drude variant over the box grown by T (its halo cells ran the plain
        update in the first launch), reading and writing the box's dispersive
        state -- (delta = D - Dp, Ep) per E component -- once per pass.  The
        stepped chain never runs on the box (the hybrid's shell keeps the
        absorbing layers only).  Returns the plan (T, box, tables) or None:
        3D runs of an electric Drude medium with uniform eps / gamma
        (coefficient tuples in a table of <= 256 rows per component), the box
        in the sigma = 0 region, TF/SF targets (if any) clear of the Drude
        launch's cone, no amplitude mode or complex fields;
        ``--blocked-drude off`` (or one step per pass) keeps the stepped
        dispersive box.  Decomposed runs: T is the ghost depth, every rank
        plans the global box clipped to its allocation (its state joins the
        deep exchange), and the ranks vote -- one rank's refusal keeps the
        stepped box everywhere.  Reference: Scheme3D.cpp:266-416,
        Kernels.h:103-107; the MPI counterpart shares D1 / B1 on
        nextTimeStep, Scheme3D.h:161-222."""
        cfg = self.cfg
        mode = getattr(cfg, "blocked_drude", "auto")
        if (mode == "off" or not cfg.use_metamaterials or cfg.scheme != "3d" or not hasattr(self.ops, "tb_drude_step")
                or (self.ops.name != "hip" and mode != "on")):
            return None
        if (self.planes != 1 or cfg.use_amp_mode or self.graph_mode
                or not self.use_upml_chain or getattr(self, "chain_regions", None) is None or self.use_cpml
                or getattr(cfg, "dispersion", "drude") != "drude" or self.hooks):
            return None
        if any("D1" in self.upml[c] for c in self.h_comps) or not any("D1" in self.upml[c] for c in self.e_comps):
            return None
        T = int(cfg.hybrid_block) if int(cfg.hybrid_block) > 0 else int(cfg.time_block)
        if T <= 0:
            T = DRUDE_AUTO_STEPS
        if self.halo is not None:
            T = self.domain.buffer_size  # one T-deep exchange per pass
        T = min(T, int(getattr(self.ops, "tb_drude_max_steps", 5)))
        if T <= 1 or (self.halo is not None and T != self.domain.buffer_size):
            return None
        G = self._drude_gbox()
        if G is None:
            return None
        # (checks on this rank's arrays refuse through the vote below: every rank reaches it)
        local_ok = (not (self.ops.name == "hip" and self.dtype == torch.float32 and self.domain.shape[2] % 4 != 0)
                    and all(self.cb[c].is_scalar for c in self.comps))
        plan = self._plan_drude_local(T, G) if local_ok else False
        if self.halo is not None:
            # every rank takes the pass or none does (False: this rank refused); a rank whose
            # allocation misses the box (None) runs the same pass plan without a Drude launch
            if self.halo.allreduce_max(1.0 if plan is False else 0.0) > 0:
                return None
        elif not plan:
            return None
        self._drude_glob = (T, G)
        return plan if plan else None

    def _drude_gbox(self):
        """Bounding box of the E components' global dispersive boxes (the
        same on every rank), None without one."""
        G = None
        for c in self.e_comps:
            if "D1" in self.upml[c] and not box_empty(self._disp_box(c)):
                g = self._disp_box(c)
                G = g if G is None else (tuple(min(G[0][d], g[0][d]) for d in range(3)),
                                         tuple(max(G[1][d], g[1][d]) for d in range(3)))
        return G

    def _plan_drude_local(self, T: int, G):
        """This rank's part of :meth:`_plan_drude_blk` for the global box
        ``G``: the plan, None (``G`` misses this rank's allocation) or False
        (refused).  The rank's box is ``G`` clipped to its allocation, so the
        boxed state messages of two neighbours cover the same cells."""
        cfg = self.cfg
        dom = self.domain
        alloc = dom.allocated_global()
        B = box_intersect(G, alloc)
        if box_empty(B):
            return None
        store = {}
        for c in self.e_comps:
            S = box_intersect(self._disp_box(c), alloc) if "D1" in self.upml[c] else None
            if S is not None and box_empty(S):
                S = None
            store[c] = S
        for c in self.e_comps:
            sig0 = self._chain_sigma0.get(c)
            ub = self._global_box(c)
            for d in range(3):
                if sig0 is None or B[0][d] < sig0[0][d] or B[1][d] > sig0[1][d]:
                    return False  # the box reaches into an absorbing layer
                if B[0][d] < ub[0][d] or B[1][d] > ub[1][d]:
                    return False
        Bl = dom.to_local(B)
        if cfg.use_tfsf:
            # a scattering scene (reference Scheme3D.cpp:3452-3492 with :138-208): the Drude launch
            # recomputes the box grown by T from the pass-start fields, its halo cells on the plain
            # update without TF/SF fixes, so every TF/SF target must lie outside the launch's cone
            # (the box grown by 2T, one more cell for the staggering); the core pass / stepped shell
            # correct the faces as without the Drude box
            reach = 2 * T + 2
            cone = (tuple(Bl[0][d] - reach for d in range(3)), tuple(Bl[1][d] + reach for d in range(3)))
            if getattr(self, "tfsf", None) is None or self._tfsf_targets_in(cone):
                return False
        bshape = tuple(Bl[1][d] - Bl[0][d] for d in range(3))
        # D coefficient where sigma = 0 (the chain's cbD profile), the same for the three components
        cbd = None
        for c in self.e_comps:
            pr = self.upml[c]["prof"]
            aD = pr["axes"][0]
            v = pr["cbD"][Bl[0][aD]:Bl[1][aD]].double()
            if bool((v != v[0]).any()):
                return False
            if cbd is None:
                cbd = float(v[0])
            elif abs(float(v[0]) - cbd) > 1e-6 * abs(cbd):
                return False
        # per component: material index over B into (b0 cbd, b2, m1, m2) rows; cells outside the
        # component's own dispersive box take the plain row (cb, 0, 1, 0): E' = E + cb curl
        ids4 = torch.zeros(bshape, dtype=torch.int32, device=self.device)
        rows = []
        for q, c in enumerate(self.e_comps):
            st = self.upml[c]
            plain = [float(self.cb[c].scalar), 0.0, 1.0, 0.0]
            S = store[c]
            if S is None:
                rows.append(torch.tensor([plain], dtype=torch.float64))
                continue
            Sl = dom.to_local(S)
            ssl = tuple(slice(Sl[0][d], Sl[1][d]) for d in range(3))
            lut = st.get("_drude_lut")
            if lut is not None and lut[0] is not None:
                ids_s = lut[0][ssl].to(torch.int32)
                tab = lut[1].double().cpu()
            else:
                cells = [st[n].materialize(ssl) for n in ("b0", "b1", "b2", "ma1", "ma2")]
                cells = torch.stack([torch.as_tensor(x, dtype=torch.float64).expand(Sl[1][0] - Sl[0][0],
                                     Sl[1][1] - Sl[0][1], Sl[1][2] - Sl[0][2]) for x in cells], -1)
                tab, inv = torch.unique(cells.reshape(-1, 5), dim=0, return_inverse=True)
                tab = tab.cpu()
                ids_s = inv.reshape(cells.shape[:3]).to(torch.int32)
            b0, b1, b2, m1, m2 = (tab[:, k] for k in range(5))
            if bool(((b0 + b1 + b2).abs() > 1e-5 * (b0.abs() + b1.abs() + b2.abs())).any()):
                return False  # not the Drude ADE (b1 = -(b0 + b2))
            nid = tab.shape[0]
            if nid + 1 > 256:
                return False
            r = torch.stack([b0 * cbd, b2, m1, m2], 1)
            rows.append(torch.cat([r, torch.tensor([plain], dtype=torch.float64)]))
            # non-dispersive cells take the plain row too: the stepped chain runs the plain update
            # outside each row's material z range and leaves their D / D1 levels stale
            act = st["drude_active"][ssl].to(self.device)
            idc = torch.full(bshape, nid, dtype=torch.int32, device=self.device)
            idc[tuple(slice(Sl[0][d] - Bl[0][d], Sl[1][d] - Bl[0][d]) for d in range(3))] = torch.where(
                act, ids_s.to(self.device), torch.full_like(ids_s, nid, device=self.device))
            ids4 |= idc << (8 * q)
        nid = max(r.shape[0] for r in rows)
        lut = torch.zeros(3, nid, 4, dtype=torch.float64)
        for q, r in enumerate(rows):
            lut[q, :r.shape[0]] = r
        # gbox: this rank's box (the global box clipped to its allocation)
        return {"T": T, "box": Bl, "gbox": B, "store": store, "ids": ids4, "cbd": cbd,
                "lut": lut.to(device=self.device, dtype=self.dtype).contiguous()}

    def _finish_drude_blk(self) -> None:
        """Allocates the two state sets of the planned Drude pass (ids in
        .w of the first array, as float bits) and arms it."""
        dp = self._drude_plan
        bshape = tuple(dp["box"][1][d] - dp["box"][0][d] for d in range(3)) + (4,)
        state = []
        for _ in range(2):
            s0 = torch.zeros(bshape, dtype=self.dtype, device=self.device)
            s1 = torch.zeros(bshape, dtype=self.dtype, device=self.device)
            self._drude_ids_in(s0, dp["ids"])
            state.append((s0, s1))
        self.drude_blk = dict(dp, state=state, cur=0, loc="chain")
        self._chain_plan_cache = {}

    def _drude_ids_in(self, s0, ids) -> None:
        """The HIP kernels' material ids into .w of the first state array (as
        float bits; fp64: the low word of the double); the torch oracle reads
        them from the plan."""
        if self.ops.name != "hip":
            return
        if s0.dtype == torch.float32:
            s0[..., 3] = ids.view(torch.float32)
        else:
            s0[..., 3] = (ids.to(torch.int64) & 0xFFFFFFFF).view(torch.float64)

    def _drude_lv(self, t, S):
        """The local box ``S`` of an auxiliary level (region-local or full-grid)."""
        if hasattr(t, "view") and not isinstance(t, torch.Tensor):
            return t.view(S)
        return t[tuple(slice(S[0][d], S[1][d]) for d in range(3))]

    def _drude_blk_import(self) -> None:
        """Chain levels -> pass state: delta = D - Dp, Ep = D1p (E stands for D1)."""
        db = self.drude_blk
        if db is None or db["loc"] == "blk":
            return
        s0, s1 = db["state"][db["cur"]]
        Bl = db["box"]
        for q, c in enumerate(self.e_comps):
            s0[..., q] = 0
            s1[..., q] = 0
            S = db["store"][c]
            if S is None:
                continue
            Sl = self.domain.to_local(S)
            sl = tuple(slice(Sl[0][d] - Bl[0][d], Sl[1][d] - Bl[0][d]) for d in range(3))
            st = self.upml[c]
            D, D1 = st["D"][0], st["D1"][0]
            s0[sl + (q,)] = (self._drude_lv(D[0], Sl) - self._drude_lv(D[1], Sl)).to(s0.dtype)
            s1[sl + (q,)] = self._drude_lv(D1[1], Sl).to(s1.dtype)
        db["loc"] = "blk"

    def _drude_blk_export(self) -> None:
        """Pass state -> chain levels (checkpoints, stepped steps): the Drude
        chain reads D only through differences (b0 + b1 + b2 = 0), so D := 0,
        Dp := -delta; D1 := E, D1p := Ep."""
        db = self.drude_blk
        if db is None or db["loc"] != "blk":
            return
        s0, s1 = db["state"][db["cur"]]
        Bl = db["box"]
        for q, c in enumerate(self.e_comps):
            S = db["store"][c]
            if S is None:
                continue
            Sl = self.domain.to_local(S)
            sl = tuple(slice(Sl[0][d] - Bl[0][d], Sl[1][d] - Bl[0][d]) for d in range(3))
            st = self.upml[c]
            D, D1 = st["D"][0], st["D1"][0]
            self._drude_lv(D[0], Sl).zero_()
            self._drude_lv(D[1], Sl).copy_(-s0[sl + (q,)])
            self._drude_lv(D1[0], Sl).copy_(self._drude_lv(self.F[0][c], Sl))
            self._drude_lv(D1[1], Sl).copy_(s1[sl + (q,)])
        db["loc"] = "chain"

    def _drude_pass(self, T: int, srcs) -> None:
        """The Drude launch of a pass (after the core's plain launch, before
        the hybrid shell steps F in place): output = the box grown by T."""
        db = self.drude_blk
        if db is None:
            return  # decomposed: the box misses this rank
        self._drude_blk_import()
        Bl = db["box"]
        shape = self.domain.shape
        ob = (tuple(max(0, Bl[0][d] - T) for d in range(3)), tuple(min(shape[d], Bl[1][d] + T) for d in range(3)))
        upd = {c: self.local_box(c, self.domain.allocated_global()) for c in self.comps}
        sin, sout = db["state"][db["cur"]], db["state"][1 - db["cur"]]
        if self.halo is not None:
            # decomposed (after the exchange and every plain launch of the pass): this rank's owned
            # cells only; the ghost state came from the neighbours with THEIR material ids in .w
            # (fp32 state): this rank's ids back in
            ob = box_intersect(ob, self.domain.to_local(self.domain.owned_global()))
            self._drude_ids_in(sin[0], db["ids"])
            if box_empty(ob):
                db["cur"] ^= 1
                return
        with self.prof.phase("blocked-drude"):
            self.ops.tb_drude_step(self.F[0], self.F_alt[0], upd, ob, self.cb, T, srcs[0],
                                   {"box": Bl, "sin": sin, "sout": sout, "lut": db["lut"], "cbd": db["cbd"],
                                    "ids": db["ids"]})
        db["cur"] ^= 1

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
                if self.halo is not None:
                    H = self.domain.buffer_size  # decomposed: one pass per ghost exchange, every rank alike
        hmax = getattr(self.ops, "tb2d_max_steps" if two_d else "tb_max_steps", 8 if two_d else 6)
        dg = self._drude_glob
        if dg is not None and not self.fused and self.tb == 1 and dg[0] <= hmax:
            if not (cfg.use_pml or cfg.use_tfsf):
                # no absorbing layer: plain blocked passes over the whole grid + the Drude pass
                self.tb = dg[0]
                if not hasattr(self, "F_alt"):
                    self.F_alt = [{c: self._zeros() for c in self.comps} for _ in range(self.planes)]
                return
            H = dg[0]
        if (H <= 1 or self.fused or self.tb > 1 or cfg.scheme not in ("3d", "tmz", "tez")
                or not hasattr(self.ops, "tb_step") or cfg.use_amp_mode or self.graph_mode
                or not (cfg.use_pml or cfg.use_tfsf or cfg.use_metamaterials) or H > hmax):
            return
        if self.halo is not None and (cfg.scheme != "3d" or self.domain.buffer_size != H):
            # decomposed: one T-deep exchange per pass feeds both the core and
            # the deep-halo stepped shell, so the ghosts must be exactly T deep
            return
        # (2D UPML fp32 used to step everything: the hybrid shell's per-window
        # launches cost as much as the whole stepped grid -- 77.1k vs 88.7k at
        # 8192^2 TMz + TF/SF -- until the 2D passes replayed from HIP graphs:
        # 158k, profiles/graph2d_r4.md)
        # fp32 3D rows are float4 along z, 2D rows 16-byte lanes along y
        shape_ok = True  # (this rank's arrays: refused through the vote, which every rank reaches)
        if self.ops.name == "hip":
            if two_d and self.domain.shape[1] % (16 // self.dtype.itemsize) != 0:
                shape_ok = False
            if not two_d and self.dtype == torch.float32 and self.domain.shape[2] % 4 != 0:
                shape_ok = False
        plan = self._voted(self._hybrid_plan(H) if shape_ok else None)
        if plan is None and dg is not None:
            self._drude_plan = self._drude_glob = dg = None  # the stepped dispersive box after all
            plan = self._voted(self._hybrid_plan(H) if shape_ok else None)
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

    def _voted(self, plan):
        """Decomposed: a hybrid plan only when every rank found one (the
        checks near the TF/SF targets are local), so all ranks run the same
        pass structure and exchanges."""
        if self.halo is not None and self.halo.allreduce_max(1.0 if plan is None else 0.0) > 0:
            return None
        return plan

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

    def _hybrid_core_tfsf(self, T: int) -> bool:
        """True when the blocked core pass applies the TF/SF corrections
        itself (``TfsfSets``: incidence along x or y, 3D; csrc/tb3d_mr.h
        ``tf_fix``), so the TF/SF faces need not lie in the stepped shell."""
        cfg = self.cfg
        mode = getattr(cfg, "hybrid_tfsf", "auto")
        if (not cfg.use_tfsf or cfg.scheme != "3d" or getattr(self, "tfsf_sets", None) is None
                or mode == "shell" or T > TFSF_MAX_STEPS):
            return False
        if mode == "auto" and self.use_cpml and self.dtype == torch.float32:
            # measured (512^3 fp32, T = 5, profiles/tfsf_cost_r5.md): with UPML the
            # faces in the core win (87.0k vs 81.1k Mcells/s: the D/B-form chain
            # shell is dear per cell), with CPML the shell keeps them (93.1k vs
            # 91.2k: the folded CPML kernels step the vacuum windows cheaply
            # while the TF/SF face tiles still cost the core ~30%).  fp64: the
            # blocked kernel is HBM-bound, the corrections ride along
            # (profiles/physics_r6.md)
            return False
        return True

    def _hybrid_plan_m(self, T: int, m: int):
        """Hybrid plan with core margin ``m``.  With in-kernel TF/SF
        (:meth:`_hybrid_core_tfsf`) the core reaches ``m`` cells from the
        absorbing layers and carries the TF/SF faces; otherwise the faces lie
        in the stepped shell.  (Round 4's TF/SF variant cost twice the plain
        kernel per cell, so the faces stayed in the shell then:
        profiles/tfsf_core_r4.md; profiles/tfsf_cost_r5.md for the rewrite.)"""
        dom = self.domain
        cfg = self.cfg
        size = cfg.size
        alloc = dom.allocated_global()
        core_tf = self._hybrid_core_tfsf(T)
        # split: the x faces (every x-streaming tile of the core meets them) in
        # the stepped shell, the y / z faces in the core, whose tiles clear of
        # them run the plain kernel -- the TF/SF variant only on the core's
        # y / z border slabs (serial runs)
        split = (core_tf and getattr(cfg, "hybrid_tfsf", "auto") == "split" and self.halo is None
                 and cfg.scheme == "3d")
        lo, hi = [0, 0, 0], list(size)
        act = [self.layout.active(a) for a in range(3)]  # 2D: z is one cell, never cut
        for a in range(3):
            if not act[a]:
                continue
            edge = 0
            if cfg.use_pml:
                edge = max(edge, self.layout.pml_size[a])
            if cfg.use_tfsf and (not core_tf or (split and a == 0)):
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
        dblk = self._drude_glob is not None and self._drude_glob[0] == T
        if cfg.use_metamaterials and self.use_upml_chain and not dblk:
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
                    if dblk and kind == "E" and all(r[c] == self._disp_chain.get(c) for c in r):
                        continue  # the Drude box: inside the core, advanced by the Drude pass
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
            if cfg.use_tfsf and not core_tf and self._tfsf_targets_in(dom.to_local(g)):
                return None
        if dblk:
            # the Drude pass's output (the box grown by T) must lie inside the one core box
            gb = self._drude_glob[1]
            if len(couts) != 1 or any(gb[0][d] - T < couts[0][0][d] or gb[1][d] + T > couts[0][1][d]
                                      for d in range(3) if act[d]):
                return None
        if self.halo is not None:
            # decomposed: each rank's core is its owned part of the global core
            couts = [box_intersect(b, dom.owned_global()) for b in couts]
            couts = [b for b in couts if not box_empty(b)]
        # step s of the pass (0-based) advances the shell plus a band T - s
        # deep into the core: the stale core beyond the band corrupts one
        # more band cell per step, so after step s the band is exact to depth
        # T - 1 - s, and after the last step the shell itself (depth 0).  The
        # windows and the copy boxes come from the one geometry both drivers
        # use (csrc/host_native.cpp fdtd::hybrid_windows)
        from ..native import hybrid_windows
        got = hybrid_windows(alloc, K, Dm if Dm is not None and not box_empty(Dm) else None, size, act, T)
        if got is None:
            return None
        shells, copy_boxes = got
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
        core_tfs = None
        if split and D is None:
            # inner boxes: no TF/SF target within T + 1 of their output (the
            # plain kernel); the rest of the core (the y / z border slabs) takes
            # the TF/SF variant
            boxes, flags = [], []
            for ob in couts:
                ilo, ihi = list(ob[0]), list(ob[1])
                for a in (1, 2):
                    ilo[a] = max(ilo[a], cfg.tfsf_size[a] + T + 2)
                    ihi[a] = min(ihi[a], size[a] - cfg.tfsf_size[a] - T - 2)
                inner = (tuple(ilo), tuple(ihi))
                if box_empty(inner) or self._tfsf_targets_in(dom.to_local(grow(inner, T + 1))):
                    boxes, flags = None, None
                    break
                boxes.append(inner)
                flags.append(False)
                for b in box_subtract(ob, inner):
                    if not box_empty(b):
                        boxes.append(b)
                        flags.append(True)
            if boxes is not None:
                couts, core_tfs = boxes, flags
        # the Drude pass may run next to the shell steps when its cone (the box grown by 2T, one more
        # cell for the staggering) meets no shell window (stepped in place in F) and no copy box
        dside = False
        if dblk:
            cone = grow(self._drude_glob[1], 2 * T + 1)
            dside = not any(not box_empty(box_intersect(cone, w)) for ws in shells for w in ws + copy_boxes)
        return {"T": T, "core": [dom.to_local(b) for b in couts], "shell": shells[0], "shells": shells,
                "copy": [dom.to_local(b) for b in copy_boxes], "upd": upd, "core_cells": core_cells,
                "cut_cells": box_volume(Dm) if Dm is not None else 0, "core_tfsf": core_tf, "core_tfs": core_tfs,
                "drude": dblk,
                "drude_side": dside}

    def _tfsf_pass(self, p: int, T: int, level0: int = 0, dry: bool = False):
        """In-kernel TF/SF of a blocked pass starting at step ``self.t`` on
        plane ``p``: advances the plane's incident line ``T`` steps (``dry``:
        on scratch copies, the line stays -- hybrid passes, whose stepped
        shell advances it) and returns the ``tfsf`` argument of
        ``ops.tb_step`` (None without in-kernel TF/SF)."""
        sets = getattr(self, "tfsf_sets", None)
        if not self.cfg.use_tfsf or sets is None:
            return None
        vals = [self.source_value(self.t + l, p) for l in range(T)]
        g = self.ops.tfsf_pass(self.einc[p], self.hinc[p], self.inc_ce, self.inc_ch, vals, self.t + T + 2, sets,
                               slot=p, dry=dry)
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
        # in-kernel TF/SF of the core: the pass's g tables from scratch copies
        # of the incident line (the shell steps below advance the real one)
        tfs = ([self._tfsf_pass(p, T, dry=True) for p in range(self.planes)] if hp.get("core_tfsf")
               else [None] * self.planes)

        flags = hp.get("core_tfs") if self.halo is None else None  # split: the TF/SF variant per core box

        def core(boxes):
            for p in range(self.planes):
                for i, ob in enumerate(boxes):
                    if tfs[p] is not None and (flags is None or flags[i]):
                        self.ops.tb_step(self.F[p], self.F_alt[p], hp["upd"], ob, self.cb, T, srcs[p], tfsf=tfs[p])
                    else:
                        self.ops.tb_step(self.F[p], self.F_alt[p], hp["upd"], ob, self.cb, T, srcs[p])

        with self.prof.phase("blocked-core"):
            core(core_now)
        dside = None
        if hp.get("drude") and self.halo is None:
            if hp.get("drude_side") and self.device.type == "cuda" and self.drude_side:
                # its cone is clear of every shell window and copy box (_hybrid_plan_m): it runs next to
                # the shell steps on a stream of its own, after the core pass it overwrites
                dside = self.__dict__.get("_drude_stream")
                if dside is None:
                    dside = self._drude_stream = torch.cuda.Stream(device=self.device)
                dside.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(dside):
                    self._drude_pass(T, srcs)
            else:
                self._drude_pass(T, srcs)  # reads F: before the shell steps below advance it in place
        if self.halo is not None:
            self._mark("interior")
            self._join_side(side)
            self._mark("wait")
            with self.prof.phase("blocked-core"):
                core(core_later)
            if hp.get("drude"):
                self._drude_pass(T, srcs)  # after the exchange (its cone reads ghosts), before the shell steps
        for s in range(T):
            self.step(hp["shells"][s])
        if self.halo is not None:
            self._mark("end")
        with self.prof.phase("shell-copy"):
            fns = []
            for p in range(self.planes):
                src = [self.F[p][c] for c in self.comps]
                dst = [self.F_alt[p][c] for c in self.comps]
                fns += [(lambda b=b, src=src, dst=dst: self.ops.copy_box(src, dst, b)) for b in hp["copy"]]
            self._par_launches(fns)  # disjoint boxes: side by side on the shell streams
        if dside is not None:
            torch.cuda.current_stream(self.device).wait_stream(dside)
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
        tfs = [self._tfsf_pass(p, T) for p in range(self.planes)] if self.cfg.use_tfsf else [None] * self.planes
        # after the pass's g tables (the shells on the side stream read them), before the interior
        side = self._fork_side_stream() if self.halo is not None else None
        if self.halo is not None:
            self._mark("start")
        for p in range(self.planes):
            if not box_empty(outs[0]):
                with self.prof.phase("blocked-interior" if self.halo is not None else "blocked"):
                    if tfs[p] is not None:
                        self.ops.tb_step(self.F[p], self.F_alt[p], upd, outs[0], self.cb, T, srcs[p], tfsf=tfs[p])
                    else:
                        self.ops.tb_step(self.F[p], self.F_alt[p], upd, outs[0], self.cb, T, srcs[p])
        if self.drude_blk is not None and self.halo is None:
            self._drude_pass(T, srcs)  # overwrites the box grown by T (run plain above)
        if self.halo is not None:
            self._mark("interior")

            # disjoint output boxes that read F and write F_alt only
            def shell(ob, p):
                if tfs[p] is not None:
                    self.ops.tb_step(self.F[p], self.F_alt[p], upd, ob, self.cb, T, srcs[p], tfsf=tfs[p])
                else:
                    self.ops.tb_step(self.F[p], self.F_alt[p], upd, ob, self.cb, T, srcs[p])
            if side is not None and self.prof.enabled:
                with torch.cuda.stream(side):
                    with self.prof.phase("halo-overlapped"):
                        self.halo.exchange_all(self)
            else:
                with self.prof.phase("halo-overlapped"):
                    self.halo.exchange_all(self, stream=side)
            self._join_side(side)
            self._mark("wait")
            # in order on the main stream: side by side with the interior
            # (on the exchange stream after the unpack) the shells' small
            # workgroups fragment the CUs the interior's one-per-CU workgroups
            # need (4x2x1 0.646 vs 0.632 ms a step), and on three streams of
            # their own they gain nothing (profiles/decomp_r5.md)
            with self.prof.phase("blocked-shells"):
                for ob in outs[1:]:
                    for p in range(self.planes):
                        shell(ob, p)
            if self.drude_blk is not None:
                self._drude_pass(T, srcs)  # its cone reads the fresh ghosts: after the exchange
            self._mark("end")
        for p in range(self.planes):
            self.F[p], self.F_alt[p] = self.F_alt[p], self.F[p]
        self.t += T
        if self.cfg.check_finite and (self.t // max(1, self.cfg.finite_check_step)
                                      != (self.t - T) // max(1, self.cfg.finite_check_step)):
            self.check_finite()
