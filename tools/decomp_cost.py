#!/usr/bin/env python3
"""Per-GPU compute cost of a decomposed blocked run, measured on ONE GPU.

Runs one rank's sub-domain of an N-way decomposition through the scheme's
blocked step (interior pass + T-thick shells + halo pack / unpack kernels)
with a null transport (messages are not moved), and compares the time per
step with the serial blocked kernel on the same number of cells.  The
difference is the compute overhead of the decomposition (shell re-reads,
pack / unpack) that RCCL transfers must hide under.

    python tools/decomp_cost.py --size 1024 1024 1024 --world 8 --rank 3 --time-block 4
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
    cfg = SchemeConfig(scheme="3d", size=size, scene="vacuum", dtype="f32", use_fused=True, time_block=T)
    if a.physics != "vacuum":
        cfg = SchemeConfig(scheme="3d", size=size, scene="vacuum", dtype="f32", use_pml=True,
                           pml_type="upml" if a.physics.startswith("upml") else "cpml",
                           use_tfsf=a.physics.endswith("tfsf"), hybrid_block=T)

    def timed(domain, halo):
        s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32), domain, halo)
        s.ops.tb_thin_single_row = bool(a.thin)
        s.init_scheme()
        s.init_grids()
        if a.physics != "vacuum":
            print("hybrid pass: %s (ghost depth %d)" % (s.hybrid is not None, s.domain.buffer_size if s.domain else 0))
        s.advance(2 * T)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.advance(a.steps)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        del s
        torch.cuda.empty_cache()
        return dt

    halo = HaloExchanger(dom, comm=NullComm(rank, a.world))
    t_dec = timed(dom, halo)
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
