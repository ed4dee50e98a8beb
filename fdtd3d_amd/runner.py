"""The ``fdtd3d`` driver: command line -> distributed setup -> scheme -> timed
time loop -> report.  Python counterpart of the reference ``Source/main.cpp``
(the standalone native driver is ``csrc/main.cpp``).

Launch:
    python -m fdtd3d_amd --3d --sizex 128 --same-size --time-steps 200
    torchrun --nproc-per-node 8 -m fdtd3d_amd --3d --parallel-grid ...

Differences from the reference driver (``main.cpp:36-241``), all fixes:
``--num-cuda-gpus`` selects ``rank % N`` also in serial runs (bug #11); 2D
honours ``--2d-mode tez`` (bug #20); the point source is injected at the
*global* centre by whichever rank holds it (bug #17); every option listed
by ``--help`` is honoured.
"""

from __future__ import annotations

import json
import math
import os
import sys
import time
from typing import List, Optional

from .utils import logging as log
from .utils.settings import (EXIT_BREAK_ARG_PARSING, EXIT_OK, Settings, setup_from_cmd)


def select_device_index(settings: Settings, local_rank: int, world: int, avail: int) -> int:
    """GPU of this rank: ``local_rank % n`` with ``n`` = ``--num-cuda-gpus``
    clipped to the visible devices (reference bug #11 fixed); under torchrun
    with the default ``--num-cuda-gpus 1`` on a multi-GPU node one rank per GPU
    (RCCL refuses two ranks on one device)."""
    avail = max(1, avail)
    n = max(1, min(settings.numCudaGPUs, avail))
    if world > 1 and settings.numCudaGPUs <= 1 and avail > 1:
        n = avail
    return local_rank % n


def _init_distributed(settings: Settings):
    """Process group of a torchrun launch.  The rank's GPU is bound BEFORE
    ``init_process_group`` (``device_id`` = eager RCCL communicator on the
    right device), and a barrier establishes the communicator before the
    first batched point-to-point exchange -- the order ``bench.py`` uses."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None, 0, 1
    if not dist.is_initialized():
        use_gpu = (torch.cuda.device_count() > 0 and settings.backend != "torch" and settings.device != "cpu")
        backend = "nccl" if use_gpu else "gloo"
        device = None
        if use_gpu:
            local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
            idx = select_device_index(settings, local, world, torch.cuda.device_count())
            torch.cuda.set_device(idx)
            device = "cuda:%d" % idx
        from .parallel.comm import init_process_group
        init_process_group(backend, device)
        dist.barrier()
    return dist, dist.get_rank(), dist.get_world_size()


def build(settings: Settings, rank: int = 0, world: int = 1):
    """Create (scheme, halo, core) for the settings on this rank."""
    import torch
    from .models.scheme import SchemeConfig, YeeScheme
    from .ops import make_ops, resolve_backend
    from .parallel.halo import HaloExchanger
    from .parallel.topology import ParallelGridCore, read_available_topologies

    cfg = SchemeConfig.from_settings(settings)
    backend, device = resolve_backend(settings.backend, settings.device)
    if device.startswith("cuda"):
        local = int(os.environ.get("LOCAL_RANK", rank))
        dev_index = select_device_index(settings, local, world, torch.cuda.device_count())
        torch.cuda.set_device(dev_index)
        device = "cuda:%d" % dev_index
    dtype = torch.float32 if cfg.dtype == "f32" else torch.float64
    ops = make_ops(backend, None, device, dtype)
    domain, halo, core = None, None, None
    if world > 1:
        active = {"3d": (0, 1, 2), "tmz": (0, 1), "tez": (0, 1), "1d": (0,)}[cfg.scheme]
        avail = None
        if settings.fileWithAvailableTopologies not in ("", "nofile"):
            avail = read_available_topologies(settings.fileWithAvailableTopologies)
        requested = (settings.topologySizeX, settings.topologySizeY, settings.topologySizeZ)
        user = requested[0] * requested[1] * requested[2] == world and not settings.doUseOptimalVirtualTopology
        core = ParallelGridCore.create(cfg.size, world, settings.parallelBufferDimension,
                                       requested if user else None, optimal=not user, available=avail,
                                       active_axes=active)
        if rank >= core.used_procs:
            raise SystemExit("rank %d is unused by topology %s" % (rank, core.topology))
        buf = settings.bufferSize
        tb = settings.timeBlock
        plain = (backend == "hip" and cfg.use_fused
                 and not (cfg.use_pml or cfg.use_tfsf or cfg.use_metamaterials or cfg.use_amp_mode))
        if tb <= 0:  # automatic: the scheme's own rule (models/blocking.py auto_time_block)
            from .layout.materials import Scene
            from .models.blocking import auto_time_block
            percell = Scene(cfg.scene, cfg.scheme).percell_kinds(cfg.use_metamaterials)
            tb = auto_time_block(cfg.scheme, cfg.dtype, backend, percell, world) if plain else 1
        if tb > 1 and cfg.scheme in ("3d", "tmz", "tez"):
            buf = tb  # blocked passes exchange tb-deep ghosts every tb steps
        hyb = (backend == "hip" and cfg.use_fused and cfg.scheme == "3d" and not cfg.use_amp_mode
               and (cfg.use_pml or cfg.use_tfsf or cfg.use_metamaterials) and settings.hybridBlock != 1)
        if hyb:
            # hybrid passes (models/blocking.py): blocked core + stepped shell,
            # one hybridBlock-deep exchange per pass
            from .models.blocking import F64_AUTO_STEPS, HYBRID_AUTO_STEPS
            buf = settings.hybridBlock if settings.hybridBlock > 1 else (HYBRID_AUTO_STEPS if cfg.dtype == "f32"
                                                                          else F64_AUTO_STEPS)
        # float4 rows: z extent (3D) / y extent (2D) padded to a multiple of 4
        domain = core.domain(rank, buf, align_z=4 if (tb > 1 or hyb) else 1,
                             align_axis=2 if cfg.scheme == "3d" else 1)
        halo = HaloExchanger(domain)
    scheme = YeeScheme(cfg, ops, domain, halo)
    return scheme, halo, core


def _report(settings: Settings, scheme, seconds: float, world: int, core, steps: int, out=sys.stdout):
    """The reference's end-of-run report (main.cpp:173-238) plus throughput."""
    cfg = scheme.cfg
    dim = {"3d": 3, "tmz": 2, "tez": 2, "1d": 1}[cfg.scheme]
    out.write("Total time = %f seconds\n" % seconds)
    out.write("Dimension: %d\n" % dim)
    if dim == 3:
        out.write("Grid size: %dx%dx%d\n" % tuple(cfg.size))
    elif dim == 2:
        out.write("Grid size: %dx%d\n" % tuple(cfg.size[:2]))
    else:
        out.write("Grid size: %d\n" % cfg.size[0])
    out.write("Number of time steps: %d\n\n" % steps)
    out.write("Value type: %s%s\n" % ("float" if cfg.dtype == "f32" else "double",
                                     " (complex)" if scheme.planes == 2 else ""))
    out.write("\n-------- Details --------\n")
    out.write("Parallel grid: %d\n" % (1 if world > 1 else 0))
    if world > 1:
        out.write("Number of processes: %d\n" % world)
        out.write("Parallel grid scheme: %s (topology %dx%dx%d)\n" % (
            settings.parallelBufferDimension.upper(), *core.topology))
        # effective ghost depth: blocked passes exchange T-deep ghosts whatever --buffer-size says
        out.write("Buffer size: %d\n" % scheme.domain.buffer_size)
    cells = cfg.size[0] * cfg.size[1] * cfg.size[2]
    mc = cells * steps / max(seconds, 1e-12) / 1e6
    kern = "fused E+H" if getattr(scheme, "fused", False) else "split"
    if getattr(scheme, "tb", 1) > 1:
        kern = "temporally blocked (%d steps per pass)" % scheme.tb
    if getattr(scheme, "graph_mode", False):
        kern += ", HIP graphs"
    out.write("Backend: %s on %s, %s kernels\n" % (scheme.ops.name, scheme.device, kern))
    out.write("Throughput: %.1f Mcells/s\n" % mc)
    return mc


def run(argv: Optional[List[str]] = None, out=sys.stdout) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    status, settings = setup_from_cmd(argv, out=out)
    if status == EXIT_BREAK_ARG_PARSING:
        return EXIT_OK
    if status != EXIT_OK:
        return status
    log.set_level(settings.logLevel)
    dist, rank, world = _init_distributed(settings)
    log.set_rank(rank)
    import torch
    from .io.checkpoint import load_checkpoint, save_checkpoint
    from .io.dump import dump_fields, dump_materials
    from .models.ntff import ntff_report

    scheme, halo, core = build(settings, rank, world)
    scheme.init_scheme()
    scheme.init_grids()
    log.info("scheme %s size %s backend %s dtype %s" % (scheme.cfg.scheme, scheme.cfg.size, scheme.ops.name,
                                                         scheme.cfg.dtype))
    if settings.doSaveMaterials:
        dump_materials(scheme, settings)
    start_step = 0
    if settings.loadFromFile:
        start_step = load_checkpoint(scheme, settings.loadFromFile)
        log.info("resumed from %s at step %d" % (settings.loadFromFile, start_step))

    # periodic work (reference: NTFF every 100 steps, dumps every N steps),
    # run between blocked passes (YeeScheme.add_periodic)
    def ntff_hook(s, t):
        # the reference evaluates after finishing step t-1 of its loop
        if halo is not None:
            halo.drain(s)
        ntff_report(s, t - 1, out=out if rank == 0 else open(os.devnull, "w"))

    def interm_hook(s, t):
        if halo is not None:
            halo.drain(s)
        dump_fields(s, settings, t, "interm-")
        if settings.doSaveScatteredFieldIntermediate:
            dump_fields(s, settings, t, "interm-scattered-", scattered=True)

    def checkpoint_hook(s, t):
        if halo is not None:
            halo.drain(s)
        save_checkpoint(s, settings.checkpointDir)

    if scheme.cfg.use_ntff and scheme.cfg.scheme == "3d":
        scheme.add_periodic(scheme.cfg.ntff_step, 1, ntff_hook)
    if settings.doSaveIntermediateRes:
        scheme.add_periodic(settings.intermediateSaveStep, 0, interm_hook)
    if settings.checkpointDir and settings.checkpointStep > 0:
        scheme.add_periodic(settings.checkpointStep, 0, checkpoint_hook)
    steps = max(0, settings.numTimeSteps - start_step)

    def sync():
        if scheme.device.type == "cuda":
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    warm = min(max(0, settings.warmupSteps), steps)
    if warm:
        scheme.advance(warm)  # regular steps only: amplitude mode follows the timed ones
        steps -= warm
    sync()
    scheme.prof.reset()  # phase timings cover the timed steps only
    if halo is not None:
        halo.bytes_sent = 0
        if settings.doPrintJson:
            from .models.blocking import PassTimer
            scheme.pass_timer = PassTimer(scheme.device)
    t0 = time.perf_counter()
    t_start = scheme.t
    scheme.perform_steps(steps)
    steps = scheme.t - t_start  # amplitude mode: its steps count as timed steps too
    if halo is not None:
        halo.drain(scheme)
    sync()
    seconds = time.perf_counter() - t0
    if settings.doSaveRes:
        dump_fields(scheme, settings, scheme.t)
    if settings.doSaveScatteredFieldRes:
        dump_fields(scheme, settings, scheme.t, "scattered-", scattered=True)
    if settings.checkpointDir:
        save_checkpoint(scheme, settings.checkpointDir)
    phases = scheme.prof.summary() if scheme.prof.enabled else None
    breakdown = None
    if scheme.pass_timer is not None:
        breakdown = scheme.pass_timer.summary()
        scheme.pass_timer = None
    if rank == 0:
        mc = _report(settings, scheme, seconds, world, core, steps, out)
        if scheme.cfg.use_amp_mode:
            taken = getattr(scheme, "amplitude_taken", 0)
            if getattr(scheme, "amplitude_converged", False):
                out.write("Amplitude mode: stable after %d steps (%d amplitude steps taken)\n"
                          % (scheme.amplitude_stable_step, taken))
            else:
                out.write("Amplitude mode: stable state not reached after %d steps\n" % taken)
        if phases:
            out.write(scheme.prof.report() + "\n")
        if settings.doPrintJson:
            rec = {"seconds": seconds, "steps": steps, "mcells_per_s": mc, "size": list(scheme.cfg.size),
                   "ranks": world, "backend": scheme.ops.name}
            if phases:
                rec["phases"] = phases
            if breakdown is not None:
                rec["rank0_passes"] = breakdown  # decomposed passes: interior / exchange wait / shell ms
            if scheme.device.type == "cuda":
                rec["max_mem_gb"] = torch.cuda.max_memory_allocated(scheme.device) / 1e9
                rec["mem_plan_gb"] = round(sum(getattr(scheme, "mem_plan", {}).values()) / 1e9, 2)
            if halo is not None:
                # rank 0's halo traffic over the timed steps (sent bytes; every
                # rank receives as much as its neighbours send it)
                rec["halo_gb_sent"] = halo.bytes_sent / 1e9
                rec["halo_gb_per_s"] = halo.bytes_sent / 1e9 / seconds if seconds > 0 else 0.0
            out.write(json.dumps(rec) + "\n")
    if dist is not None:
        dist.destroy_process_group()
    return EXIT_OK


def main() -> None:
    sys.exit(run())
