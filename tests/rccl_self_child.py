"""Child process of ``tests/test_rccl_gpu.py``: one direct deep-halo exchange
through REAL RCCL (backend ``nccl``) on one GPU, every peer mapped to self.

A 1-rank ``nccl`` group is initialised with the solver's own
``nccl_init_kwargs`` (high-priority streams, ``device_id`` bound eagerly),
then :class:`~fdtd3d_amd.parallel.halo.HaloExchanger` posts the exact op
list of one exchange of the middle rank of a 3 x 3 x 3 rank grid (26
neighbours: x-face array slices sent straight from the arrays, packed edge /
corner buffers, ``deep_messages()`` order) on a high-priority side stream via
``DistComm.post`` -> ``batch_isend_irecv``.  RCCL ignores tags: sends and
receives to one peer pair in posting order, so with every peer = self the
k-th send lands in the k-th receive, i.e. every ghost box ``rbox(off)``
receives this rank's own ``sbox(off)``.  The main stream then waits for the
side stream the way the blocked passes do (``BlockedStepping._join_side``)
and reads the arrays.  Checks: every ghost box, the owned cells untouched,
and (negative control) that a read NOT ordered after the side stream sees
stale ghosts while the unpack is held back.  Prints one JSON line.

Reference: ``Source/Grid/ParallelGrid.cpp:1535-1594`` (``SendReceiveRawBuffer``).
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from fdtd3d_amd.ops import make_ops  # noqa: E402
from fdtd3d_amd.parallel.comm import P2P, DistComm, init_process_group  # noqa: E402
from fdtd3d_amd.parallel.halo import HaloExchanger  # noqa: E402
from fdtd3d_amd.parallel.topology import ParallelGridCore  # noqa: E402


class SelfComm(DistComm):
    """``DistComm`` with every peer replaced by this rank (RCCL send-to-self)."""

    def post(self, ops):
        return super().post([P2P(o.send, o.tensor, self.rank, o.tag) for o in ops])


class FakeScheme:
    def __init__(self, ops, device, full, boxed):
        self.ops, self.device = ops, device
        self._full, self._boxed = full, boxed

    def state_tensors(self):
        return list(self._full) + [t for t, _, _ in self._boxed]

    def state_boxes(self):
        return [None] * len(self._full) + [(cover, first) for _, cover, first in self._boxed]


def _sl(b):
    return tuple(slice(b[0][a], b[1][a]) for a in range(3))


def expected(halo, dom, snap_full, snap_boxed, direct_x):
    """CPU model of one self-mapped exchange: x-face planes first (they land
    by the transfers), then the packed messages' unpacks."""
    full = [t.clone() for t in snap_full]
    boxed = [(t.clone(), cover, first) for t, cover, first in snap_boxed]
    msgs = halo.deep_messages()
    packed = []
    for off, _, sg, rg in msgs:
        sb, rb = dom.to_local(sg), dom.to_local(rg)
        if off[1] == 0 and off[2] == 0 and direct_x:
            for t, s in zip(full, snap_full):
                t[rb[0][0]:rb[1][0]] = s[sb[0][0]:sb[1][0]]
        else:
            packed.append((sg, rg, sb, rb))
    for sg, rg, sb, rb in packed:
        for t, s in zip(full, snap_full):
            t[_sl(rb)] = s[_sl(sb)]
        for (t, cover, first), (s, _, _) in zip(boxed, snap_boxed):
            # cover == the allocated box here: send / receive parts have equal sizes
            lo = tuple(first[a] for a in range(3))
            rbl = tuple(tuple(rb[i][a] - lo[a] for a in range(3)) for i in range(2))
            sbl = tuple(tuple(sb[i][a] - lo[a] for a in range(3)) for i in range(2))
            t[_sl(rbl)] = s[_sl(sbl)]
    return full, [t for t, _, _ in boxed]


def run_case(ops, dev, dom, with_boxed, delay):
    shape = dom.shape
    g = torch.Generator(device="cpu").manual_seed(7 + int(with_boxed))
    full = [torch.randn(shape, generator=g).to(dev) for _ in range(6)]
    boxed = []
    if with_boxed:
        alloc = dom.allocated_global()
        boxed.append((torch.randn(shape, generator=g).to(dev), alloc, dom.to_local(alloc)[0]))
    scheme = FakeScheme(ops, dev, full, boxed)
    halo = HaloExchanger(dom, comm=SelfComm())
    snap_full = [t.cpu() for t in full]
    snap_boxed = [(t.cpu(), c, f) for t, c, f in boxed]
    exp_full, exp_boxed = expected(halo, dom, snap_full, snap_boxed, direct_x=not with_boxed)
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev, priority=-1)
    torch.cuda.synchronize()

    # negative control: unpack held back, a main-stream read NOT ordered after the side stream
    halo.debug_delay_cycles = delay
    side.wait_stream(main)
    halo.exchange_all(scheme, stream=side)
    early = [t.clone() for t in full + [b[0] for b in boxed]]   # main stream, no wait
    main.wait_stream(side)                                        # BlockedStepping._join_side
    late = [t.clone() for t in full + [b[0] for b in boxed]]     # ordered after the exchange
    torch.cuda.synchronize()
    want = exp_full + exp_boxed
    worst = max(float((a.cpu() - b).abs().max()) for a, b in zip(late, want))
    stale = max(float((a.cpu() - b).abs().max()) for a, b in zip(early, want))
    owned = dom.to_local(dom.owned_global())
    owned_ok = all(torch.equal(a.cpu()[_sl(owned)], s[_sl(owned)])
                   for a, s in zip(late, snap_full + [s for s, _, _ in snap_boxed]))
    return {"messages": halo.messages, "bytes": halo.bytes_sent, "max_err": worst, "stale_err": stale,
            "owned_untouched": owned_ok, "n_msgs": len(halo.deep_messages())}


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    init_process_group("nccl", device=dev, timeout_s=120)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    ops = make_ops("hip", None, dev, torch.float32)
    B = 4
    core = ParallelGridCore((40, 36, 48), 27, (3, 3, 3))
    dom = core.domain(13, B, align_z=4)   # the middle rank: 26 neighbours
    out = {"backend": dist.get_backend(), "shape": list(dom.shape)}
    out["direct"] = run_case(ops, dev, dom, with_boxed=False, delay=40_000_000)
    out["packed"] = run_case(ops, dev, dom, with_boxed=True, delay=40_000_000)
    dist.destroy_process_group()
    print("RCCL_SELF " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
