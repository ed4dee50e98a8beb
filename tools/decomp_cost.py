#!/usr/bin/env python3
"""Per-GPU cost of a decomposed blocked run, measured on ONE GPU.

Runs one rank's sub-domain of an N-way decomposition through the scheme's
blocked step (interior pass + T-thick shells + halo pack / unpack kernels)
and compares the time per step with the serial blocked kernel on the same
number of cells.  Transports:

* ``null`` -- messages are not moved (the compute overhead of the
  decomposition: shell re-reads, pack / unpack);
* ``loopback`` -- every receive buffer is filled by a device-to-device copy
  of a send buffer of the same size on the exchange's side stream, plus
  (``--link-gbs``) a spin kernel for the wire time of the largest message
  over one xGMI link: real pack, copy and unpack kernels that must find CUs
  next to the interior pass.  The per-pass breakdown (``PassTimer``:
  interior, exchange wait, shell) says how much of the exchange the interior
  pass hides.  (Fields are not meaningful: timing only.)

    python tools/decomp_cost.py --size 1024 1024 1024 --world 8 --topology 4 2 1 --transport loopback
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class NullComm:
    """Transport that completes every send / receive immediately (timing only)."""
    backend = "null"

    def __init__(self, rank, world):
        self.rank, self.world = rank, world

    def post(self, ops):
        return []

    def allreduce(self, v, op="sum"):
        return v


class LoopbackComm:
    """Loopback transport (timing only): a receive is filled from a send
    buffer of the same size by a device copy on the current (side) stream;
    with ``link_gbs`` a spin kernel then stands in for the wire time of the
    largest message (every neighbour has its own xGMI link)."""
    backend = "loopback"

    def __init__(self, rank, world, link_gbs=0.0):
        self.rank, self.world = rank, world
        self.link_gbs = link_gbs
        self.bytes = 0
        self._cyc_per_us = None

    def _spin(self, us):
        import torch
        if self._cyc_per_us is None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            torch.cuda._sleep(1000000)
            b.record()
            b.synchronize()
            self._cyc_per_us = 1000000 / (a.elapsed_time(b) * 1e3)
        torch.cuda._sleep(max(1, int(us * self._cyc_per_us)))

    def post(self, ops):
        sends = {}
        for o in ops:
            if o.send:
                sends.setdefault(o.tensor.numel(), []).append(o.tensor)
        big = 0
        for o in ops:
            if o.send:
                continue
            pool = sends.get(o.tensor.numel())
            if pool:
                o.tensor.copy_(pool[-1])
            else:
                o.tensor.zero_()
            nb = o.tensor.numel() * o.tensor.element_size()
            self.bytes += nb
            big = max(big, nb)
        if self.link_gbs > 0 and big:
            self._spin(big / (self.link_gbs * 1e3))
        return []

    def allreduce(self, v, op="sum"):
        return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, nargs=3, default=[1024, 1024, 1024])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=-1, help="-1: the rank with the most neighbours")
    ap.add_argument("--axes", default="xy")
    ap.add_argument("--time-block", type=int, default=5)
    ap.add_argument("--topology", type=int, nargs=3, default=None, help="force a rank grid (e.g. 4 2 1)")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--thin", type=int, default=1, help="thin y shells on the single-row kernel (T <= 4)")
    ap.add_argument("--shell-streams", type=int, default=0,
                    help="streams the T-thick shell slabs run on (0 = automatic: 3, 1 = in order)")
    ap.add_argument("--skip-exchange", action="store_true",
                    help="no exchange at all (ghosts stale): the interior pass alone, no side-stream work")
    ap.add_argument("--transport", default="null", choices=("null", "loopback"))
    ap.add_argument("--link-gbs", type=float, default=0.0,
                    help="loopback: emulate the wire time of the largest message at this xGMI link rate (GB/s)")
    ap.add_argument("--physics", default="vacuum", choices=("vacuum", "cpml-tfsf", "upml-tfsf", "cpml"),
                    help="non-vacuum: hybrid passes (blocked owned core + deep-halo stepped shell), per-GPU "
                         "Mcells/s only")
    a = ap.parse_args()
    import torch
    from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
    from fdtd3d_amd.ops import make_ops
    from fdtd3d_amd.parallel.halo import HaloExchanger
    from fdtd3d_amd.parallel.topology import ParallelGridCore

    T = a.time_block
    size = tuple(a.size)
    if a.topology:
        core = ParallelGridCore.create(size, a.world, a.axes, requested=a.topology, optimal=False)
    else:
        core = ParallelGridCore.create(size, a.world, a.axes)
    rank = a.rank
    if rank < 0:
        def nn(r):
            d = core.domain(r, T)
            return sum((x >= 0) for pair in d.neighbors for x in pair)
        rank = max(range(core.used_procs), key=nn)
    dom = core.domain(rank, T, align_z=4)
    cfg = SchemeConfig(scheme="3d", size=size, scene="vacuum", dtype="f32", use_fused=True, time_block=T,
                       shell_streams=a.shell_streams)
    if a.physics != "vacuum":
        cfg = SchemeConfig(scheme="3d", size=size, scene="vacuum", dtype="f32", use_pml=True,
                           pml_type="upml" if a.physics.startswith("upml") else "cpml",
                           use_tfsf=a.physics.endswith("tfsf"), hybrid_block=T,
                           shell_streams=a.shell_streams)

    breakdown = {}

    def timed(domain, halo):
        s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32), domain, halo)
        s.ops.tb_thin_single_row = bool(a.thin)
        s.init_scheme()
        s.init_grids()
        if a.physics != "vacuum":
            print("hybrid pass: %s (ghost depth %d)" % (s.hybrid is not None, s.domain.buffer_size if s.domain else 0))
        s.advance(2 * T)
        torch.cuda.synchronize()
        if halo is not None:
            from fdtd3d_amd.models.blocking import PassTimer
            s.pass_timer = PassTimer(s.device)
            halo.reset_timing()
            halo.timing = True
            if hasattr(halo.comm, "bytes"):
                halo.comm.bytes = 0
        t0 = time.perf_counter()
        s.advance(a.steps)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        if halo is not None:
            bd = s.pass_timer.summary()
            n = max(1, bd["passes"])
            breakdown.update({k: bd[k] / n for k in ("interior_ms", "exchange_wait_ms", "shell_ms")})
            breakdown["exchange_ms"] = halo.exchange_ms() / max(1, halo.exchanges)
            breakdown["passes"] = bd["passes"]
            s.pass_timer = None
            halo.timing = False
        del s
        torch.cuda.empty_cache()
        return dt

    comm = (LoopbackComm(rank, a.world, a.link_gbs) if a.transport == "loopback" else NullComm(rank, a.world))
    halo = HaloExchanger(dom, comm=comm)
    if a.skip_exchange:
        halo.exchange_all = lambda scheme, stream=None: None
    t_dec = timed(dom, halo)
    if breakdown:
        wait_frac = breakdown["exchange_wait_ms"] / max(1e-9, breakdown["interior_ms"])
        print("per pass (%s transport%s): interior %.3f ms, exchange (side stream) %.3f ms, exchange wait %.3f ms "
              "(%.1f%% of the interior), shell %.3f ms; %d passes, %.1f MB moved per pass"
              % (a.transport, ", %.0f GB/s links" % a.link_gbs if a.link_gbs else "", breakdown["interior_ms"],
                 breakdown["exchange_ms"], breakdown["exchange_wait_ms"], 100 * wait_frac, breakdown["shell_ms"],
                 breakdown["passes"], getattr(comm, "bytes", 0) / 1e6 / max(1, breakdown["passes"])))
    own = dom.owned_shape
    cells = own[0] * own[1] * own[2]
    if a.physics != "vacuum":
        glob = size[0] * size[1] * size[2]
        print("%s %s: topology %s rank %d owned %s neighbours %s: decomposed step %.3f ms, %.0f Mcells/s per "
              "GPU (x %d GPUs = %.0f if the exchange hides under the interior pass)"
              % (a.physics, "x".join(map(str, size)), "x".join(map(str, core.topology)), rank, own, dom.neighbors,
                 t_dec * 1e3, cells / t_dec / 1e6, a.world, glob / t_dec / 1e6))
        return
    # serial reference on the rank's owned extent
    from fdtd3d_amd.parallel.domain import Domain
    cfg_serial = SchemeConfig(scheme="3d", size=tuple(own), scene="vacuum", dtype="f32", use_fused=True,
                              time_block=T)
    cfg, cfg_dec = cfg_serial, cfg
    t_ser = timed(None, None)
    print("topology %s rank %d owned %s neighbours %s" % ("x".join(map(str, core.topology)), rank, own,
                                                        dom.neighbors))
    print("decomposed step %.3f ms (%.0f Mcells/s per GPU), serial same cells %.3f ms (%.0f Mcells/s): "
          "overhead %.1f%%" % (t_dec * 1e3, cells / t_dec / 1e6, t_ser * 1e3, cells / t_ser / 1e6,
                               100 * (t_dec / t_ser - 1)))


if __name__ == "__main__":
    main()
