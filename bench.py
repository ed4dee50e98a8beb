#!/usr/bin/env python3
"""Headline benchmark: Mcells/s (whole node) of the 3D vacuum Yee leapfrog on a
1024^3 grid, fp32, point-dipole source, on 1/2/4/8 MI355X (BASELINE.json).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
launched under ``torch.distributed.run`` (one rank per GPU, RCCL).  W untimed
steps, then exactly K timed steps bracketed by barrier + device sync on both
sides; the slowest rank's time is used; rank 0 prints one JSON line.

Scaling is *strong*: the global grid stays 1024^3 and is decomposed over the
GPUs on x and y (2 -> 2x1x1, 4 -> 2x2x1, 8 -> 4x2x1 by the halo-surface
optimiser).  Every timed step is the full leapfrog: E and H updates of all
cells, the hard source and (N>1) the RCCL halo exchange.  Several leapfrog
steps run per HBM pass through the temporally blocked kernel
(``csrc/yee3d_tb.hip``; automatic: 5 steps per pass on one and two GPUs, 4
on more); decomposed runs exchange T-deep ghosts with all face,
edge and corner neighbours once per pass, overlapped with the interior pass.
A step count that is not a multiple of T ends with one shorter pass, so
exactly K steps are timed.  ``--time-block 1`` selects the single-pass fused
kernel.  Fields start from zero plus the source -- the data dependence of the
kernels is nil (pure streaming).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", type=int, nargs=3, default=[1024, 1024, 1024])
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--split", action="store_true", help="use the split E / H kernels instead of the fused one")
    ap.add_argument("--xchunk", type=int, default=0)
    ap.add_argument("--buffer-size", type=int, default=1, help="halo depth (deep halo when > 1)")
    ap.add_argument("--time-block", type=int, default=0,
                    help="leapfrog steps per HBM pass (temporally blocked kernel; 0 automatic: 5 on one or two "
                         "GPUs, 4 on more); decomposed runs use a halo of the same depth")
    ap.add_argument("--tb-xchunk", type=int, default=0, help="x planes per workgroup of the blocked kernel")
    ap.add_argument("--tb-vec", type=int, default=0, help="lane width of the blocked kernel (0 auto, 2, 4)")
    ap.add_argument("--tb-rows", type=int, default=0, help="grid rows per wave of the blocked kernel (0 auto, 1, 2)")
    ap.add_argument("--tb-mrows", type=int, default=0,
                    help="adjacent y rows per wave of the blocked kernel (0 auto, 1 single-row kernel, 2)")
    ap.add_argument("--tb-variant", type=int, default=-1,
                    help="multi-row blocked kernel: bit 0 deferred stores, bit 1 two planes prefetched (-1 default)")
    ap.add_argument("--tb-xcd", type=int, default=0, help="XCD-aware tile order of the blocked kernel (1 on, 0 off)")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
    from fdtd3d_amd.ops import make_ops, resolve_backend
    from fdtd3d_amd.parallel.halo import HaloExchanger
    from fdtd3d_amd.parallel.topology import ParallelGridCore

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if rank == 0:
            print("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (a.gpus, world), file=sys.stderr)
    backend, device = resolve_backend(a.backend, "auto")
    # FDTD_BENCH_COMM=gloo rehearses the multi-rank path with several ranks on
    # one GPU (RCCL refuses duplicate devices; gloo stages halos through host)
    comm = os.environ.get("FDTD_BENCH_COMM", "nccl")
    if device == "cuda":
        dev_index = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_index)
        device = "cuda:%d" % dev_index
    if world > 1:
        from fdtd3d_amd.parallel.comm import init_process_group
        use_nccl = device.startswith("cuda") and comm == "nccl"
        init_process_group("nccl" if use_nccl else "gloo", device if use_nccl else None)
        # establish the communicator with a collective before the first
        # batched point-to-point exchange
        dist.barrier()

    size = tuple(a.size)
    core = None
    if world > 1:
        # the blocked kernel tiles z in 54..60-cell rows, so a T-thick z shell
        # would cost a whole tile row: decompose x and y only when blocking
        core = ParallelGridCore.create(size, world, "xy" if a.time_block != 1 else "xyz")
    if a.time_block <= 0:
        # automatic: 5 steps per pass on one and two GPUs, 4 on more -- there
        # the 5-deep ghosts and shells cost more than the saved HBM traffic
        # (tools/decomp_cost.py, per-GPU Mcells/s with a null transport on
        # 1024^3, three runs each: 2 ranks T=5 269-281k vs T=4 238-274k; 4
        # ranks T=4 224-252k vs T=5 239-245k; 8 ranks T=4 229k vs T=5 221k;
        # one GPU T=5 281-289k vs T=4 260-263k)
        a.time_block = 5 if world <= 2 else 4
        if a.dtype == "f64":
            from fdtd3d_amd.models.scheme import F64_AUTO_STEPS
            a.time_block = F64_AUTO_STEPS
    cfg = SchemeConfig(scheme="3d", size=size, time_steps=a.steps, scene="vacuum", dtype=a.dtype,
                       use_pml=False, use_tfsf=False, use_fused=not a.split, time_block=a.time_block)
    if a.time_block > 1 and world > 1:
        a.buffer_size = a.time_block
    dtype = torch.float32 if a.dtype == "f32" else torch.float64
    if world > 1:
        domain = core.domain(rank, a.buffer_size, align_z=4 if a.time_block > 1 else 1)
        halo = HaloExchanger(domain)
        topo = core.topology
    else:
        domain, halo, topo = None, None, (1, 1, 1)
    kw = {"xchunk": a.xchunk} if backend == "hip" else {}
    ops = make_ops(backend, None, device, dtype, **kw)
    if a.tb_xchunk:
        ops.tb_xchunk = a.tb_xchunk
    if backend == "hip":
        ops.tb_vec, ops.tb_rows, ops.tb_xcd, ops.tb_mrows = a.tb_vec, a.tb_rows, a.tb_xcd, a.tb_mrows
        if a.tb_variant >= 0:
            ops.tb_variant = a.tb_variant
    scheme = YeeScheme(cfg, ops, domain, halo)
    scheme.init_scheme()
    scheme.init_grids()

    def sync():
        if device.startswith("cuda"):
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    scheme.advance(a.warmup)
    if halo is not None:
        halo.drain(scheme)
        # one ghost refresh outside the timed region (idempotent: the ghosts
        # get the values they already hold) so that RCCL's lazily created
        # peer connections exist even with --warmup 0
        if scheme.tb > 1 or a.buffer_size > 1:
            halo.exchange_all(scheme)
    sync()
    t0 = time.perf_counter()
    scheme.advance(a.steps)
    if halo is not None:
        halo.drain(scheme)
    if device.startswith("cuda"):
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device if device.startswith("cuda") else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    cells = size[0] * size[1] * size[2]
    mcells = cells * a.steps / dt / 1e6
    if rank == 0:
        par = "x".join(str(v) for v in topo)
        out = {
            "metric": "Mcells/sec (whole node), 3D vacuum 1024^3 grid at 1/2/4/8 MI355X",
            "value": round(mcells, 1),
            "unit": "Mcells/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32" if a.dtype == "f32" else "fp64",
            "data": "synthetic (zero fields + hard point-dipole Ez source, vacuum)",
            "config": {
                "model": "fdtd3d 3D Yee leapfrog, vacuum, point dipole (BASELINE.json headline)",
                "grid": "%dx%dx%d" % size,
                "global_batch": 1,
                "seq_len": cells,
                "parallelism": "domain-decomposition %s (dp%d-equivalent ranks)" % (par, world),
                "backend": backend,
                "time_block": scheme.tb,
                "halo_bytes_per_step": (halo.bytes_sent // max(1, a.steps + a.warmup)) if halo else 0,
            },
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
