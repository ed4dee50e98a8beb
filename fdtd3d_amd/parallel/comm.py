"""Point-to-point transports for the halo exchange.

* :class:`DistComm` -- ``torch.distributed``.  With the ``nccl`` backend (RCCL
  on ROCm) every half step's sends/receives go out as ONE
  ``batch_isend_irecv`` group, so all xGMI links to the face neighbours work
  concurrently and the RCCL stream is ordered after the current HIP stream.
  With ``gloo`` CPU tensors are sent directly; GPU tensors are staged through
  host memory (used to run several ranks on one GPU, where RCCL refuses
  duplicate devices).
* :class:`LocalHub` / :class:`LocalComm` -- in-process transport between
  ranks that are Python threads of one process (GPU tests of the decomposed
  solver on a single device, no process spawning).
"""

from __future__ import annotations

import queue
import threading
from collections import namedtuple
from typing import Dict, List, Tuple

import torch
import torch.distributed as dist

# send=True: tensor is sent to peer; send=False: tensor receives from peer
P2P = namedtuple("P2P", "send tensor peer tag")


DEFAULT_TIMEOUT_S = 300


def nccl_init_kwargs(device=None, timeout_s: float = DEFAULT_TIMEOUT_S) -> dict:
    """Keyword arguments of ``init_process_group`` for the ``nccl`` (RCCL)
    backend: high-priority communication streams (halo transfers that overlap
    a long interior kernel get dispatched as soon as a CU has room), the
    device bound eagerly, and a collective timeout -- with the default
    asynchronous error handling a hung exchange aborts the process (non-zero
    exit) instead of hanging the job."""
    import datetime
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    kw = {"pg_options": opts, "timeout": datetime.timedelta(seconds=float(timeout_s))}
    if device is not None:
        kw["device_id"] = torch.device(device)
    return kw


def init_process_group(backend: str, device=None, timeout_s: float = DEFAULT_TIMEOUT_S) -> None:
    """``torch.distributed`` init for the solver (``nccl`` == RCCL over xGMI
    on MI355X, ``gloo`` on the CPU), with a timeout on every collective."""
    import datetime
    if backend == "nccl":
        dist.init_process_group("nccl", **nccl_init_kwargs(device, timeout_s))
    else:
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=float(timeout_s)))


def build_p2p_ops(ops: List[P2P], group=None) -> list:
    """``P2POp`` list of one batched RCCL group: every send and receive of
    one exchange, so ``batch_isend_irecv`` issues them between one
    ``ncclGroupStart`` / ``ncclGroupEnd`` pair (all xGMI links at once)."""
    return [dist.P2POp(dist.isend if o.send else dist.irecv, o.tensor, o.peer, group, o.tag) for o in ops]


class _Done:
    def wait(self):
        return True


class DistComm:
    def __init__(self, group=None):
        self.group = group
        self.backend = dist.get_backend(group) if dist.is_initialized() else "gloo"

    @property
    def rank(self) -> int:
        return dist.get_rank(self.group) if dist.is_initialized() else 0

    @property
    def world(self) -> int:
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def post(self, ops: List[P2P]):
        if not ops:
            return []
        if self.backend == "gloo" and ops[0].tensor.is_cuda:
            return self._post_staged(ops)
        if self.backend == "nccl":
            return dist.batch_isend_irecv(build_p2p_ops(ops, self.group))
        works = []
        for o in ops:
            f = dist.isend if o.send else dist.irecv
            works.append(f(o.tensor, o.peer, group=self.group, tag=o.tag))
        return works

    def _post_staged(self, ops: List[P2P]):
        works, recvs = [], []
        for o in ops:
            if o.send:
                works.append(dist.isend(o.tensor.cpu(), o.peer, group=self.group, tag=o.tag))
            else:
                host = torch.empty(o.tensor.shape, dtype=o.tensor.dtype)
                works.append(dist.irecv(host, o.peer, group=self.group, tag=o.tag))
                recvs.append((o.tensor, host))
        for w in works:
            w.wait()
        for dev, host in recvs:
            dev.copy_(host)
        return []

    def allreduce(self, v: float, op: str = "sum") -> float:
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX, group=self.group)
        return float(t.item())


class LocalHub:
    """Mailboxes shared by ``world`` in-process ranks.  ``tagless``: one FIFO
    per (sender, receiver) pair whatever the tag -- RCCL's matching rule (the
    k-th send to a peer lands in that peer's k-th receive from the sender), so
    an op list whose per-peer order differs between the two sides shows up as
    wrong ghosts on the CPU, where gloo's tag matching would hide it."""

    def __init__(self, world: int, tagless: bool = False):
        self.world = world
        self.tagless = tagless
        self._boxes: Dict[Tuple[int, ...], "queue.Queue"] = {}
        self._lock = threading.Lock()
        self._barrier = threading.Barrier(world)
        self._red: List[float] = [0.0] * world

    def box(self, src: int, dst: int, tag: int) -> "queue.Queue":
        key = (src, dst) if self.tagless else (src, dst, tag)
        with self._lock:
            q = self._boxes.get(key)
            if q is None:
                q = queue.Queue()
                self._boxes[key] = q
            return q

    def comm(self, rank: int) -> "LocalComm":
        return LocalComm(self, rank)


class _LocalRecv:
    def __init__(self, q, dst):
        self.q, self.dst = q, dst

    def wait(self):
        src, ev = self.q.get(timeout=120)
        if src.shape != self.dst.shape:
            raise RuntimeError("message size mismatch: sent %s, receive %s (send / receive order differs "
                               "between the peers)" % (tuple(src.shape), tuple(self.dst.shape)))
        if ev is not None:
            # stream-ordered like RCCL's work.wait(): the receiver's CURRENT
            # stream waits for the sender's snapshot, the host does not -- a
            # consumer that forgets to order its stream after this one reads
            # stale ghosts (tests/test_parallel_gpu.py negative control)
            cur = torch.cuda.current_stream(self.dst.device)
            cur.wait_event(ev)
            src.record_stream(cur)  # the snapshot's memory lives until the copy ran
        self.dst.copy_(src)
        return True


class LocalComm:
    """In-process transport with RCCL's ordering semantics: a send snapshots
    the buffer on the sender's current stream and publishes it with an event;
    a receive's ``wait()`` makes the receiver's current stream wait on that
    event.  Nothing synchronises the host, so a missing stream dependency on
    either side shows up as wrong fields instead of being hidden by a
    device-wide sync."""
    backend = "local"

    def __init__(self, hub: LocalHub, rank: int):
        self.hub = hub
        self.rank = rank
        self.world = hub.world

    def post(self, ops: List[P2P]):
        works = []
        for o in ops:
            if o.send:
                snap = o.tensor.clone()
                ev = None
                if snap.is_cuda:
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(snap.device))
                self.hub.box(self.rank, o.peer, o.tag).put((snap, ev))
                works.append(_Done())
            else:
                works.append(_LocalRecv(self.hub.box(o.peer, self.rank, o.tag), o.tensor))
        return works

    def allreduce(self, v: float, op: str = "sum") -> float:
        self.hub._red[self.rank] = float(v)
        self.hub._barrier.wait()
        r = sum(self.hub._red) if op == "sum" else max(self.hub._red)
        self.hub._barrier.wait()
        return r
