"""Ghost-cell (halo) exchange between sub-domains over ``torch.distributed``.

Replaces the reference's ``ParallelGrid::share`` (``Source/Grid/ParallelGrid.cpp:1600-1823``):
a serial loop over up to 26 directions, each packing all three time levels into
a ``std::vector`` and calling blocking ``MPI_Sendrecv`` followed by
``MPI_Barrier``, with no overlap.

Design here (one process per GPU, backend ``nccl`` == RCCL over xGMI on
MI355X, ``gloo`` on CPU):

* ``buffer_size == 1`` -- *face mode*.  The Yee curl is axis aligned, so E
  needs only H's low-face ghosts and H only E's high-face ghosts.  After each
  half step every rank packs (one HIP kernel per face) the 2 components the
  neighbour needs and posts all face sends/receives of that half step in ONE
  batched group (``batch_isend_irecv`` -> one RCCL group, every xGMI link busy
  at once).  The next half step updates the interior cells, which need no
  ghost, while the transfer is in flight; then waits, unpacks and updates the
  one-cell boundary slabs.  One message per neighbour per half step, no
  barriers.
* ``buffer_size == B > 1`` -- *deep halo*.  Every ``B`` steps all state arrays
  (fields and auxiliary UPML/Drude levels) exchange ``B``-deep ghosts; the
  scheme computes redundantly in the ghost zone in between
  (:meth:`fdtd3d_amd.parallel.domain.Domain.window`).  Default ``direct``
  mode: faces, edges and corners go straight to the face / edge / corner
  neighbour (up to 26 messages, the reference's ``BUFFER_COUNT`` directions,
  ``Source/Grid/BufferPosition.inc.h:8-61``) in ONE batched group -- a node's
  8 GPUs are fully connected by xGMI, so every peer has its own link and one
  round of concurrent transfers beats the ``sweep`` mode's three dependent
  rounds (axis after axis, edges and corners relayed through the faces).
"""

from __future__ import annotations

import itertools
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .comm import P2P, DistComm
from .domain import Domain, box_empty, box_intersect
from ..utils.assertions import fdtd_assert
from .topology import chunk_bounds, coords_rank

Box = Tuple[Tuple[int, int, int], Tuple[int, int, int]]


def _face_components(layout, kind_needed: str, axis: int) -> List[str]:
    """Components of kind ``kind_needed`` (H or E) read across a face normal to
    ``axis`` by the opposite kind's curl."""
    consumers = [c for c in layout.components if c[0] != kind_needed]
    out = []
    for c in consumers:
        for (s, ax, _) in layout.curl_terms(c):
            if ax == axis and s not in out:
                out.append(s)
    return sorted(out)


class HaloExchanger:
    def __init__(self, domain: Domain, group=None, comm=None, mode: str = "direct"):
        if mode not in ("direct", "sweep"):
            raise ValueError("halo exchange mode must be direct or sweep")
        self.mode = mode
        self.domain = domain
        self.group = group
        self.comm = comm if comm is not None else DistComm(group)
        self.backend = self.comm.backend
        self.pending: Dict[Tuple[str, int], list] = {}
        self.bufs: Dict[tuple, torch.Tensor] = {}
        self.bytes_sent = 0
        self.messages = 0
        # exchange timing (bench / --json): HIP events on the exchange's
        # stream around each deep exchange, wall clock on the CPU
        self.timing = False
        self._timed: List[tuple] = []
        self._wall_s = 0.0
        self.exchanges = 0

    # ------------------------------------------------------------ helpers
    def _buf(self, key, n, like: torch.Tensor) -> torch.Tensor:
        b = self.bufs.get(key)
        if b is None or b.numel() != n or b.dtype != like.dtype or b.device != like.device:
            b = torch.empty(n, dtype=like.dtype, device=like.device)
            self.bufs[key] = b
        return b

    def _post(self, ops_list):
        return self.comm.post(ops_list)

    def _face_box(self, axis: int, side: str, kind: str, send: bool) -> Box:
        """Global box of the one-cell face layer for face mode."""
        d = self.domain
        lo, hi = list(d.lo), list(d.hi)
        if kind == "H":      # H travels low -> high: sender's top layer -> receiver's low ghost
            if send:
                lo[axis], hi[axis] = d.hi[axis] - 1, d.hi[axis]
            else:
                lo[axis], hi[axis] = d.lo[axis] - 1, d.lo[axis]
        else:                # E travels high -> low: sender's bottom layer -> receiver's high ghost
            if send:
                lo[axis], hi[axis] = d.lo[axis], d.lo[axis] + 1
            else:
                lo[axis], hi[axis] = d.hi[axis], d.hi[axis] + 1
        return tuple(lo), tuple(hi)

    # ------------------------------------------------------------ face mode
    def start(self, scheme, kind: str, p: int) -> None:
        """Pack and post the faces produced by the ``kind`` half step."""
        d = self.domain
        ops = scheme.ops
        F = scheme.F[p]
        ops_list = []
        recvs = []
        for a in range(3):
            comps = _face_components(scheme.layout, kind, a)
            if not comps:
                continue
            if kind == "H":
                to, frm = d.neighbors[a][1], d.neighbors[a][0]
            else:
                to, frm = d.neighbors[a][0], d.neighbors[a][1]
            tensors = [F[c] for c in comps]
            if to >= 0:
                box = d.to_local(self._face_box(a, None, kind, True))
                n = _vol(box) * len(comps)
                sb = self._buf(("s", kind, p, a), n, tensors[0])
                ops.pack(tensors, box, sb)
                ops_list.append(P2P(True,sb, to,_tag(kind, a)))
                self.bytes_sent += sb.numel() * sb.element_size()
                self.messages += 1
            if frm >= 0:
                box = d.to_local(self._face_box(a, None, kind, False))
                n = _vol(box) * len(comps)
                rb = self._buf(("r", kind, p, a), n, tensors[0])
                ops_list.append(P2P(False,rb, frm,_tag(kind, a)))
                recvs.append((tensors, box, rb))
        works = self._post(ops_list)
        self.pending[(kind, p)] = (works, recvs)

    def _wait(self, kind: str, p: int, ops) -> None:
        pend = self.pending.pop((kind, p), None)
        if pend is None:
            return
        works, recvs = pend
        for w in works:
            w.wait()
        for tensors, box, rb in recvs:
            ops.unpack(tensors, box, rb)

    def regions(self, kind: str) -> Tuple[Box, List[Box]]:
        """(interior, boundary slabs) of the owned box for a half step: E
        slabs are the low layers next to a neighbour, H slabs the high ones."""
        d = self.domain
        lo, hi = list(d.lo), list(d.hi)
        slabs = []
        for a in range(3):
            if kind == "E" and d.has_low(a):
                s_lo, s_hi = list(lo), list(hi)
                s_hi[a] = lo[a] + 1
                slabs.append((tuple(s_lo), tuple(s_hi)))
                lo[a] += 1
            elif kind == "H" and d.has_high(a):
                s_lo, s_hi = list(lo), list(hi)
                s_lo[a] = hi[a] - 1
                slabs.append((tuple(s_lo), tuple(s_hi)))
                hi[a] -= 1
        return (tuple(lo), tuple(hi)), slabs

    def finish_and_update(self, scheme, kind: str, p: int) -> None:
        """Interior update overlapped with the pending exchange of the other
        kind, then boundary slabs."""
        other = "H" if kind == "E" else "E"
        interior, slabs = self.regions(kind)
        pend = self.pending.get((other, p))
        if pend is None or not slabs:
            self._wait(other, p, scheme.ops)
            scheme._update(kind, p, [interior] + slabs)
            return
        # interior first, overlapping the transfer; UPML level rotation must
        # happen once, so run all windows through one _update call after the wait
        if scheme.use_upml_chain:
            self._wait(other, p, scheme.ops)
            scheme._update(kind, p, [interior] + slabs)
            return
        scheme._update(kind, p, [interior])
        self._wait(other, p, scheme.ops)
        scheme._update(kind, p, slabs)

    def drain(self, scheme) -> None:
        for key in list(self.pending.keys()):
            self._wait(key[0], key[1], scheme.ops)

    # ------------------------------------------------------------ deep halo
    def exchange_all(self, scheme, stream=None) -> None:
        """B-deep exchange of every state array, edges and corners included
        (``direct``: one batched round to up to 26 neighbours; ``sweep``: axis
        by axis).  With ``stream`` the packing,
        RCCL transfers and unpacking are issued on that (side) stream so they
        overlap compute on the current stream."""
        if stream is not None:
            with torch.cuda.stream(stream):
                self._timed_exchange(scheme)
        else:
            self._timed_exchange(scheme)

    def _timed_exchange(self, scheme) -> None:
        self.exchanges += 1
        if not self.timing:
            self._exchange_all(scheme)
            return
        dev = scheme.device
        if getattr(dev, "type", str(dev)) == "cuda":
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            self._exchange_all(scheme)
            b.record()
            self._timed.append((a, b))
        else:
            import time
            t0 = time.perf_counter()
            self._exchange_all(scheme)
            self._wall_s += time.perf_counter() - t0

    def reset_timing(self) -> None:
        self._timed = []
        self._wall_s = 0.0
        self.exchanges = 0

    def exchange_ms(self) -> float:
        """Total milliseconds of the timed exchanges since :meth:`reset_timing`
        (pack + transfer + unpack, on the exchange's own stream: overlapped
        with the interior pass, so this is latency, not added step time).
        Synchronises the device."""
        ms = self._wall_s * 1e3
        for a, b in self._timed:
            b.synchronize()
            ms += a.elapsed_time(b)
        return ms

    def _exchange_all(self, scheme) -> None:
        if self.mode == "direct":
            self._exchange_direct(scheme)
        else:
            self._exchange_sweep(scheme)

    def deep_messages(self) -> List[Tuple[Tuple[int, int, int], int, Box, Box]]:
        """(offset, peer, send box, recv box) of every neighbour of a direct
        deep-halo exchange, global indices.  Along an axis the offset is
        -1 (low side: send the first B owned layers, receive the B ghost
        layers below), +1 (high side) or 0 (the owned range, which the peer
        shares since it sits in the same rank column)."""
        cached = getattr(self, "_deep_msgs", None)
        if cached is not None:
            return cached
        d = self.domain
        B = d.buffer_size
        out = []
        for off in itertools.product((-1, 0, 1), repeat=3):
            if off == (0, 0, 0):
                continue
            c = [d.coords[a] + off[a] for a in range(3)]
            if any(c[a] < 0 or c[a] >= d.topology[a] for a in range(3)):
                continue
            slo, shi, rlo, rhi = list(d.lo), list(d.hi), list(d.lo), list(d.hi)
            for a in range(3):
                if off[a] < 0:
                    shi[a] = d.lo[a] + B
                    rlo[a], rhi[a] = d.lo[a] - B, d.lo[a]
                elif off[a] > 0:
                    slo[a] = d.hi[a] - B
                    rlo[a], rhi[a] = d.hi[a], d.hi[a] + B
            if off[1] == 0 and off[2] == 0:
                # direct x faces send whole allocated planes: the peer's y / z extents (owned,
                # ghosts, padding) must be this rank's -- true of a Cartesian rank grid, whose
                # per-axis bounds depend on that axis' coordinate only
                for a in (1, 2):
                    fdtd_assert(chunk_bounds(d.global_size[a], d.topology[a], c[a]) == (d.lo[a], d.hi[a]),
                                "x-face peer with other y / z extents")
            out.append((off, coords_rank(c, d.topology), (tuple(slo), tuple(shi)), (tuple(rlo), tuple(rhi))))
        self._deep_msgs = out
        return out

    def _exchange_direct(self, scheme) -> None:
        ops = scheme.ops
        tensors, boxed = _split_state(scheme)
        if self.listed and hasattr(ops, "box_list") and tensors[0].is_cuda:
            self._exchange_direct_listed(ops, tensors, boxed)
            return
        d = self.domain
        ops_list, recvs = [], []
        for off, peer, sg, rg in self.deep_messages():
            sbox, rbox = d.to_local(sg), d.to_local(rg)
            key = (off[0] + 1) * 9 + (off[1] + 1) * 3 + (off[2] + 1)
            back = (-off[0] + 1) * 9 + (-off[1] + 1) * 3 + (-off[2] + 1)
            if (off[1] == 0 and off[2] == 0 and self.direct_x_faces
                    and not any(_boxed_part(g, cover, first, d) is not None
                                for g in (sg, rg) for _, cover, first, _ in boxed)
                    and all(t.is_contiguous() for t in tensors)):
                # x faces: x is the slowest axis, so B whole allocated planes
                # of an array are one contiguous slice -- sent from and received
                # into the arrays themselves, no pack / unpack kernels.  The
                # planes carry the sender's y / z ghost rows too; the edge and
                # corner messages, unpacked after every transfer has landed,
                # overwrite those parts of the receiver's ghost planes (peers of
                # one rank column share the allocated y / z extents).  Only when
                # no boxed array reaches either face (the same test on both
                # peers: a boxed array covers one global box clipped to each
                # rank's allocation).
                for i, t in enumerate(tensors):
                    ops_list.append(P2P(True, t[sbox[0][0]:sbox[1][0]], peer, 1000 + 32 * i + key))
                    ops_list.append(P2P(False, t[rbox[0][0]:rbox[1][0]], peer, 1000 + 32 * i + back))
                    self.bytes_sent += t[sbox[0][0]:sbox[1][0]].numel() * t.element_size()
                    self.messages += 1
                continue
            sb = self._buf(("xs", key), _msg_len(tensors, boxed, sg), tensors[0])
            _pack_state(ops, tensors, boxed, sbox, sg, d, sb)
            rb = self._buf(("xr", key), _msg_len(tensors, boxed, rg), tensors[0])
            # the peer sends its message for offset -off with tag(-off)
            ops_list.append(P2P(True, sb, peer, 300 + key))
            ops_list.append(P2P(False, rb, peer, 300 + back))
            recvs.append((rbox, rg, rb))
            self.bytes_sent += sb.numel() * sb.element_size()
            self.messages += 1
        for w in self._post(ops_list):
            w.wait()
        if self.debug_delay_cycles and tensors[0].is_cuda:
            # tests: hold the unpack back on the exchange's stream so that a
            # consumer not ordered after it deterministically reads old ghosts
            torch.cuda._sleep(int(self.debug_delay_cycles))
        for rbox, rg, rb in recvs:
            _unpack_state(ops, tensors, boxed, rbox, rg, d, rb)

    def _direct_plan(self, ops, tensors, boxed):
        """The direct exchange of this state set as a fixed plan: the P2P
        ops (x faces straight from the arrays, the other messages through
        plan-owned buffers) and ONE table of every pack and one of every
        unpack (``ops.box_list``), cached per set of state arrays (the field
        buffers alternate between passes, the UPML levels rotate).  The same
        message layout as :func:`_pack_state`: per array its box, fields first."""
        key = (tuple(t.data_ptr() for t in tensors),
               tuple((t.data_ptr(), cover, first, zmul) for t, cover, first, zmul in boxed))
        plans = self.__dict__.setdefault("_plans", {})
        plan = plans.get(key)
        if plan is not None:
            return plan
        d = self.domain
        ops_list, nbytes, nmsg = [], 0, 0
        pack, unpack = _BoxList(), _BoxList()
        bufs = []
        for off, peer, sg, rg in self.deep_messages():
            sbox, rbox = d.to_local(sg), d.to_local(rg)
            key_m = (off[0] + 1) * 9 + (off[1] + 1) * 3 + (off[2] + 1)
            back = (-off[0] + 1) * 9 + (-off[1] + 1) * 3 + (-off[2] + 1)
            if (off[1] == 0 and off[2] == 0 and self.direct_x_faces
                    and not any(_boxed_part(g, cover, first, d) is not None
                                for g in (sg, rg) for _, cover, first, _ in boxed)
                    and all(t.is_contiguous() for t in tensors)):
                # (see _exchange_direct: whole allocated planes, y / z ghosts overwritten by the edges)
                for i, t in enumerate(tensors):
                    ops_list.append(P2P(True, t[sbox[0][0]:sbox[1][0]], peer, 1000 + 32 * i + key_m))
                    ops_list.append(P2P(False, t[rbox[0][0]:rbox[1][0]], peer, 1000 + 32 * i + back))
                    nbytes += t[sbox[0][0]:sbox[1][0]].numel() * t.element_size()
                    nmsg += 1
                continue
            sb = torch.empty(_msg_len(tensors, boxed, sg), dtype=tensors[0].dtype, device=tensors[0].device)
            rb = torch.empty(_msg_len(tensors, boxed, rg), dtype=tensors[0].dtype, device=tensors[0].device)
            bufs += [sb, rb]
            for lst, lbox, g, buf in ((pack, sbox, sg, sb), (unpack, rbox, rg, rb)):
                n = 0
                for t in tensors:
                    lst.add(t, lbox, buf, n)
                    n += _vol(lbox)
                for t, cover, first, zmul in boxed:
                    b = _boxed_part(g, cover, first, d, zmul)
                    if b is not None:
                        lst.add(t, b, buf, n)
                        n += _vol(b)
            ops_list.append(P2P(True, sb, peer, 300 + key_m))
            ops_list.append(P2P(False, rb, peer, 300 + back))
            nbytes += sb.numel() * sb.element_size()
            nmsg += 1
        plan = {"ops": ops_list, "pack": pack.build(ops), "unpack": unpack.build(ops), "bytes": nbytes,
                "messages": nmsg, "bufs": bufs}
        if len(plans) >= 16:
            plans.pop(next(iter(plans)))
        plans[key] = plan
        return plan

    def _exchange_direct_listed(self, ops, tensors, boxed) -> None:
        """The direct exchange from a cached plan: one pack launch, the
        batched P2P ops, one unpack launch (a decomposed physics pass issued
        ~40 pack / unpack launches and their Python planning per exchange,
        profiles/decomp_r6.md)."""
        plan = self._direct_plan(ops, tensors, boxed)
        if plan["pack"] is not None:
            ops.box_list(*plan["pack"], True)
        for w in self._post(plan["ops"]):
            w.wait()
        if self.debug_delay_cycles and tensors[0].is_cuda:
            torch.cuda._sleep(int(self.debug_delay_cycles))
        if plan["unpack"] is not None:
            ops.box_list(*plan["unpack"], False)
        self.bytes_sent += plan["bytes"]
        self.messages += plan["messages"]

    debug_delay_cycles = 0
    direct_x_faces = True  # x-face messages straight from / into the arrays (no pack / unpack)
    # HIP: the direct exchange from a cached plan with one pack / unpack launch (FDTD3D_HALO_LISTED=0: per
    # message and array, A/B)
    listed = os.environ.get("FDTD3D_HALO_LISTED", "1") != "0"

    def _exchange_sweep(self, scheme) -> None:
        d = self.domain
        B = d.buffer_size
        ops = scheme.ops
        tensors, boxed = _split_state(scheme)
        alloc_lo, alloc_hi = d.allocated_global()
        for a in range(3):
            lo_n, hi_n = d.neighbors[a]
            if lo_n < 0 and hi_n < 0:
                continue
            ops_list, recvs = [], []

            def box_along(l, h):
                blo, bhi = list(alloc_lo), list(alloc_hi)
                blo[a], bhi[a] = l, h
                return d.to_local((tuple(blo), tuple(bhi)))

            if lo_n >= 0:
                sbox = box_along(d.lo[a], d.lo[a] + B)
                rbox = box_along(d.lo[a] - B, d.lo[a])
                sg, rg = d.to_global(sbox), d.to_global(rbox)
                sb = self._buf(("ds", a, 0), _msg_len(tensors, boxed, sg), tensors[0])
                _pack_state(ops, tensors, boxed, sbox, sg, d, sb)
                rb = self._buf(("dr", a, 0), _msg_len(tensors, boxed, rg), tensors[0])
                ops_list.append(P2P(True,sb, lo_n,100 + 2 * a))
                ops_list.append(P2P(False,rb, lo_n,101 + 2 * a))
                recvs.append((rbox, rg, rb))
                self.bytes_sent += sb.numel() * sb.element_size()
                self.messages += 1
            if hi_n >= 0:
                sbox = box_along(d.hi[a] - B, d.hi[a])
                rbox = box_along(d.hi[a], d.hi[a] + B)
                sg, rg = d.to_global(sbox), d.to_global(rbox)
                sb = self._buf(("ds", a, 1), _msg_len(tensors, boxed, sg), tensors[0])
                _pack_state(ops, tensors, boxed, sbox, sg, d, sb)
                rb = self._buf(("dr", a, 1), _msg_len(tensors, boxed, rg), tensors[0])
                ops_list.append(P2P(True,sb, hi_n,101 + 2 * a))
                ops_list.append(P2P(False,rb, hi_n,100 + 2 * a))
                recvs.append((rbox, rg, rb))
                self.bytes_sent += sb.numel() * sb.element_size()
                self.messages += 1
            for w in self._post(ops_list):
                w.wait()
            for rbox, rg, rb in recvs:
                _unpack_state(ops, tensors, boxed, rbox, rg, d, rb)

    # ------------------------------------------------------------ collectives
    def allreduce_sum(self, v: int) -> int:
        return int(self.comm.allreduce(v, "sum"))

    def allreduce_max(self, v: float) -> float:
        return float(self.comm.allreduce(v, "max"))


def _tag(kind: str, axis: int) -> int:
    return (0 if kind == "H" else 10) + axis


def _vol(box: Box) -> int:
    v = 1
    for d in range(3):
        v *= max(0, box[1][d] - box[0][d])
    return v


def _pack_many(ops, tensors, box, buf):
    """Pack many tensors (more than one kernel's pointer budget) into one buffer."""
    n = _vol(box)
    for i in range(0, len(tensors), 8):
        chunk = tensors[i:i + 8]
        ops.pack(chunk, box, buf[i * n:(i + len(chunk)) * n])


class _BoxList:
    """(array, local box, buffer, first buffer element) entries of one
    ``ops.box_list`` launch, as the device table of aux_kernels.hip
    ``BoxEnt`` (64 bytes: two pointers, ny, nz, box, first block, vector
    width)."""

    def __init__(self):
        self.rows = []

    def add(self, t: torch.Tensor, box: Box, buf: torch.Tensor, off: int) -> None:
        if t.dim() != 3 or not t.is_contiguous():
            raise ValueError("box list: contiguous 3D arrays")
        for a in range(3):
            if box[0][a] < 0 or box[1][a] > t.shape[a] or box[1][a] <= box[0][a]:
                raise ValueError("box list: box %s outside array %s" % (box, tuple(t.shape)))
        if off + _vol(box) > buf.numel() or buf.dtype != t.dtype:
            raise ValueError("box list: buffer part out of range")
        self.rows.append((t, box, buf, off))

    def build(self, ops):
        """(device table, entries, blocks) or None when empty."""
        import numpy as np
        if not self.rows:
            return None
        n = len(self.rows)
        if ops.box_ent_size() != 64:
            raise RuntimeError("BoxEnt layout mismatch")
        e64 = np.zeros((n, 8), dtype=np.int64)
        e32 = e64.view(np.int32)
        blk = 0
        for r, (t, box, buf, off) in enumerate(self.rows):
            e64[r, 0] = t.data_ptr()
            e64[r, 1] = buf.data_ptr() + off * buf.element_size()
            e32[r, 4], e32[r, 5] = t.shape[1], t.shape[2]
            e32[r, 6:9] = box[0]
            e32[r, 9:12] = box[1]
            e32[r, 12] = blk
            # 16-byte vectors when the array rows, the box's z range and the buffer part are aligned
            v = 16 // t.element_size()
            al = (t.shape[2] % v == 0 and box[0][2] % v == 0 and box[1][2] % v == 0 and off % v == 0
                  and t.data_ptr() % 16 == 0 and buf.data_ptr() % 16 == 0)
            e32[r, 13] = v if al else 1
            blk += -(-(_vol(box) // (v if al else 1)) // 256)
        tab = torch.from_numpy(e64).to(self.rows[0][0].device)
        return (tab, n, blk)


def _split_state(scheme):
    """(arrays of the local field shape, [(array, global box it covers, local
    index of its first element, values per cell along z)]) of the scheme's
    state."""
    ts = scheme.state_tensors()
    bx = scheme.state_boxes() if hasattr(scheme, "state_boxes") else [None] * len(ts)
    full = [t for t, b in zip(ts, bx) if b is None]
    boxed = [(t, b[0], b[1], b[2] if len(b) > 2 else 1) for t, b in zip(ts, bx) if b is not None]
    return full, boxed


def _boxed_part(g: Box, cover: Box, first, d, zmul: int = 1):
    """Local box inside a boxed array (first element at local ``first``) of
    the global message box ``g`` clipped to the array's global ``cover``
    (``zmul`` values per cell along z: a vector array seen as scalars)."""
    from .domain import box_intersect
    c = box_intersect(g, cover)
    if any(c[1][a] <= c[0][a] for a in range(3)):
        return None
    lc = d.to_local(c)
    lo = [lc[0][a] - first[a] for a in range(3)]
    hi = [lc[1][a] - first[a] for a in range(3)]
    lo[2], hi[2] = lo[2] * zmul, hi[2] * zmul
    return tuple(lo), tuple(hi)


def _msg_len(full, boxed, g) -> int:
    n = _vol(g) * len(full)
    for t, cover, first, zmul in boxed:
        from .domain import box_intersect
        n += _vol(box_intersect(g, cover)) * zmul
    return n


def _pack_state(ops, full, boxed, lbox, g, d, buf):
    n = _vol(lbox) * len(full)
    _pack_many(ops, full, lbox, buf[:n])
    for t, cover, first, zmul in boxed:
        b = _boxed_part(g, cover, first, d, zmul)
        if b is None:
            continue
        m = _vol(b)
        ops.pack([t], b, buf[n:n + m])
        n += m


def _unpack_state(ops, full, boxed, lbox, g, d, buf):
    n = _vol(lbox) * len(full)
    _unpack_many(ops, full, lbox, buf[:n])
    for t, cover, first, zmul in boxed:
        b = _boxed_part(g, cover, first, d, zmul)
        if b is None:
            continue
        m = _vol(b)
        ops.unpack([t], b, buf[n:n + m])
        n += m


def _unpack_many(ops, tensors, box, buf):
    n = _vol(box)
    for i in range(0, len(tensors), 8):
        chunk = tensors[i:i + 8]
        ops.unpack(chunk, box, buf[i * n:(i + len(chunk)) * n])


def gather_box(scheme, comp: str, box, plane: int = 0, dst: int = 0, group=None) -> Optional[torch.Tensor]:
    """The global index box ``box`` of ``comp`` assembled on rank ``dst``
    (None elsewhere): each rank sends only its owned part of the box (the
    NTFF face slabs of a decomposed run, instead of whole-grid gathers)."""
    from .topology import ParallelGridCore
    d = scheme.domain
    lo, hi = tuple(box[0]), tuple(box[1])
    shape = tuple(hi[a] - lo[a] for a in range(3))

    def part(dr):
        plo = tuple(max(lo[a], dr.lo[a]) for a in range(3))
        phi = tuple(min(hi[a], dr.hi[a]) for a in range(3))
        return None if any(phi[a] <= plo[a] for a in range(3)) else (plo, phi)

    own_full = scheme.owned_field(comp, plane)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return own_full[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]].clone()
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    core = ParallelGridCore(tuple(d.global_size), world, tuple(d.topology))
    mine = part(d)

    def local(pp):
        return own_full[tuple(slice(pp[0][a] - d.lo[a], pp[1][a] - d.lo[a]) for a in range(3))].contiguous()

    if rank == dst:
        out = torch.zeros(shape, dtype=own_full.dtype, device=own_full.device)
        for r in range(core.used_procs):
            pp = part(core.domain(r, d.buffer_size))
            if pp is None:
                continue
            if r == rank:
                blk = local(pp)
            else:
                blk = torch.empty(tuple(pp[1][a] - pp[0][a] for a in range(3)), dtype=own_full.dtype,
                                  device=own_full.device)
                dist.recv(blk, r, group=group, tag=201)
            out[tuple(slice(pp[0][a] - lo[a], pp[1][a] - lo[a]) for a in range(3))] = blk
        return out
    if rank < core.used_procs and mine is not None:
        dist.send(local(mine), dst, group=group, tag=201)
    return None


def gather_field(scheme, comp: str, plane: int = 0, dst: int = 0, group=None) -> Optional[torch.Tensor]:
    """Assemble the global array of ``comp`` on rank ``dst`` (None elsewhere).

    Replaces ``ParallelGrid::gatherFullGrid`` (ParallelGrid.cpp:2600-2845),
    which broadcast every rank's chunk to *all* ranks (O(P*N) traffic): here
    each rank sends only its owned block, once, to the destination."""
    return gather_owned(scheme, scheme.owned_field(comp, plane), dst, group)


def gather_owned(scheme, own: torch.Tensor, dst: int = 0, group=None) -> Optional[torch.Tensor]:
    """Global array assembled on rank ``dst`` from every rank's owned block
    ``own`` (any per-cell quantity laid out like the owned fields, e.g. the
    scattered field of a dump); None on the other ranks."""
    from .topology import ParallelGridCore
    d = scheme.domain
    own = own.contiguous()
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return own.clone()
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    core = ParallelGridCore(tuple(d.global_size), world, tuple(d.topology))
    if rank == dst:
        full = torch.zeros(tuple(d.global_size), dtype=own.dtype, device=own.device)
        for r in range(core.used_procs):
            dr = core.domain(r, d.buffer_size)
            if r == rank:
                blk = own
            else:
                blk = torch.empty(dr.owned_shape, dtype=own.dtype, device=own.device)
                dist.recv(blk, r, group=group, tag=200)
            full[dr.lo[0]:dr.hi[0], dr.lo[1]:dr.hi[1], dr.lo[2]:dr.hi[2]] = blk
        return full
    if rank < core.used_procs:
        dist.send(own, dst, group=group, tag=200)
    return None
