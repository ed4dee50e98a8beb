#!/usr/bin/env python3
"""Headline benchmark: Mcells/s (whole node) of the 3D vacuum Yee leapfrog on a
1024^3 grid, fp32, point-dipole source, random-init fields, on 1/2/4/8 MI355X
(BASELINE.json).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
launched under ``torch.distributed.run`` (one rank per GPU, RCCL).  W untimed
steps, then exactly K timed steps bracketed by barrier + device sync on both
sides; the slowest rank's time is used; rank 0 prints one JSON line.

Scaling is *strong*: the global grid (``--size``, default 1024^3) stays fixed
and is decomposed over the GPUs (``--topology``: ``auto``, an axis set such as
``xy`` / ``xyz`` for the halo-surface optimiser, or an explicit ``2x2x2``).
Every timed step is the full leapfrog: E and H updates of all cells, the hard
source and (N>1) the RCCL halo exchange.  Several leapfrog steps run per HBM
pass through the temporally blocked kernel (``csrc/yee3d_tb.hip``;
automatic: 5 steps per pass on one GPU, 4 on more); decomposed runs
exchange T-deep ghosts with all face, edge and corner neighbours once per
pass, overlapped with the interior pass.  A step count that is not a multiple
of T ends with one shorter pass, so exactly K steps are timed.

Self-check: fields start from a deterministic hash of the *global* cell index
(``utils/synthetic.py``), so every decomposition starts from the same state and
must end in the same state; the JSON carries the all-reduced field energy
(sum of E^2 + eta0^2 H^2 over owned cells, fp64) before and after, which
``tests/test_bench_cpu.py`` checks against the serial run.  With
``--fp64-companion`` (default on one GPU) the same measurement is repeated in
fp64 -- the reference's default value type (``CMakeLists.txt:11``) -- and
reported under ``"fp64"`` without changing the headline fields.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
T_START = time.perf_counter()

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

HEADLINE_SIZE = (1024, 1024, 1024)
# rank grids of the headline grid measured fastest per GPU (profiles/decomp_r6.md)
MEASURED_GRIDS = {2: (2, 1, 1), 4: (2, 2, 1), 8: (4, 2, 1)}


def metric_name(size) -> str:
    s = tuple(size)
    if s[0] == s[1] == s[2]:
        g = "%d^3" % s[0]
    else:
        g = "%dx%dx%d" % s
    return "Mcells/sec (whole node), 3D vacuum %s grid at 1/2/4/8 MI355X" % g


def parse_topology(spec: str, size, world: int, blocked: bool):
    """Rank grid for ``--topology``: ``auto``, an axis set for the optimiser,
    or an explicit ``AxBxC``."""
    from fdtd3d_amd.parallel.topology import ParallelGridCore
    spec = spec.lower()
    if "x" in spec and spec.replace("x", "").isdigit():
        t = tuple(int(v) for v in spec.split("x"))
        if len(t) != 3 or t[0] * t[1] * t[2] != world:
            raise SystemExit("--topology %s does not match %d ranks" % (spec, world))
        return ParallelGridCore.create(size, world, "xyz", requested=t, optimal=False)
    if spec == "auto":
        # blocked passes: the measured best rank grid at 1024^3 (per-GPU cost
        # with a loopback transport, tools/decomp_cost.py, profiles/decomp_r6.md:
        # 8 ranks T = 4 -- 4x2x1 240.5k, 2x4x1 237.4k, 8x1x1 226.6k, 2x2x2
        # 219.0k Mcells/s per GPU; a T-thick z shell costs a whole 56-lane tile
        # row), else x and y split by the reference's halo-surface optimiser
        if blocked and world in MEASURED_GRIDS and tuple(size) == HEADLINE_SIZE:
            return ParallelGridCore.create(size, world, "xyz", requested=MEASURED_GRIDS[world], optimal=False)
        spec = "xy" if blocked else "xyz"
    return ParallelGridCore.create(size, world, spec)


def run_one(a, dtype_name: str, world: int, rank: int, device: str, backend: str, core):
    """Build, warm up, time ``a.steps`` steps; returns a result dict (only
    rank 0's is used)."""
    import torch
    import torch.distributed as dist

    from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
    from fdtd3d_amd.models.blocking import auto_time_block
    from fdtd3d_amd.ops import make_ops
    from fdtd3d_amd.parallel.halo import HaloExchanger

    size = tuple(a.size)
    if device.startswith("cuda"):
        torch.cuda.reset_peak_memory_stats()
    T = a.time_block
    if T <= 0:
        # automatic (models/blocking.py auto_time_block; the torch backend
        # rehearses the HIP rule): 5 steps per pass on one GPU, 4 on more --
        # there the 5-deep ghosts and shells cost more than the saved HBM
        # traffic (profiles/decomp_r6.md)
        T = auto_time_block("3d", dtype_name, "hip", False, world)
    cfg = SchemeConfig(scheme="3d", size=size, time_steps=a.steps, scene="vacuum", dtype=dtype_name,
                       use_pml=False, use_tfsf=False, use_fused=not a.split, time_block=T)
    buf = T if (T > 1 and world > 1) else a.buffer_size
    dtype = torch.float32 if dtype_name == "f32" else torch.float64
    if world > 1:
        domain = core.domain(rank, buf, align_z=4 if T > 1 else 1)
        halo = HaloExchanger(domain)
    else:
        domain, halo = None, None
    kw = {"xchunk": a.xchunk} if backend == "hip" else {}
    ops = make_ops(backend, None, device, dtype, **kw)
    if a.tb_xchunk:
        ops.tb_xchunk = a.tb_xchunk
    if backend == "hip":
        ops.tb_vec, ops.tb_rows, ops.tb_xcd, ops.tb_mrows = a.tb_vec, a.tb_rows, a.tb_xcd, a.tb_mrows
        if a.tb_variant >= 0:
            ops.tb_variant = a.tb_variant
    trace = os.environ.get("FDTD3D_BENCH_TRACE") == "1"  # phase lines on stderr (profiler runs)

    def phase(msg):
        if trace:
            print("[bench %.1fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)

    phase("ops ready")
    scheme = YeeScheme(cfg, ops, domain, halo)
    scheme.init_scheme()
    scheme.init_grids()
    phase("grids ready")
    if a.init == "random":
        scheme.randomize_fields(seed=a.seed)
    phase("fields initialised")

    def allsum(v: float) -> float:
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=device if device.startswith("cuda") else "cpu")
        dist.all_reduce(t)
        return float(t.item())

    def sync():
        if device.startswith("cuda"):
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    energy0 = allsum(scheme.field_energy())
    phase("warmup")
    scheme.advance(a.warmup)
    if halo is not None:
        halo.drain(scheme)
        # one ghost refresh outside the timed region (idempotent: the ghosts
        # get the values they already hold) so that RCCL's lazily created
        # peer connections exist even with --warmup 0
        if scheme.tb > 1 or buf > 1:
            halo.exchange_all(scheme)
        halo.reset_timing()
        halo.timing = True
        halo.bytes_sent = 0
        # per-pass main-stream breakdown (interior / exchange wait / shell)
        from fdtd3d_amd.models.blocking import PassTimer
        scheme.pass_timer = PassTimer(scheme.device)
    sync()
    phase("timed steps")
    t0 = time.perf_counter()
    scheme.advance(a.steps)
    if halo is not None:
        halo.drain(scheme)
    if device.startswith("cuda"):
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    halo_ms, nex = 0.0, 0
    if halo is not None:
        halo_ms, nex = halo.exchange_ms(), halo.exchanges
        halo.timing = False
    per_rank = []
    if world > 1:
        tdev = device if device.startswith("cuda") else "cpu"
        t = torch.tensor([dt, halo_ms / max(1, nex), halo_ms / max(1, nex)], dtype=torch.float64, device=tdev)
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t)
        dt = float(tmax[0].item())
        halo_max, halo_mean = float(tmax[1].item()), float(t[2].item()) / world
        # every rank's pass breakdown, so an 8-GPU record says which rank
        # waited on its exchange and for how long
        bd = scheme.pass_timer.summary() if scheme.pass_timer is not None else {}
        scheme.pass_timer = None
        mine = torch.tensor([bd.get("passes", 0), bd.get("interior_ms", 0.0), bd.get("exchange_wait_ms", 0.0),
                             bd.get("shell_ms", 0.0), halo_ms / max(1, nex)], dtype=torch.float64, device=tdev)
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        for r, v in enumerate(allv):
            v = v.cpu().tolist()
            n = max(1.0, v[0])
            per_rank.append({"rank": r, "passes": int(v[0]), "interior_ms": round(v[1] / n, 4),
                             "exchange_wait_ms": round(v[2] / n, 4), "shell_ms": round(v[3] / n, 4),
                             "exchange_ms": round(v[4], 4)})
    else:
        halo_max = halo_mean = 0.0
    energy = allsum(scheme.field_energy())
    cells = size[0] * size[1] * size[2]
    res = {
        "mcells": cells * a.steps / dt / 1e6,
        "dt": dt,
        "tb": scheme.tb,
        "energy0": energy0,
        "energy": energy,
        "halo_bytes": halo.bytes_sent if halo else 0,
        "halo_ms_per_pass_max": halo_max,
        "halo_ms_per_pass_mean": halo_mean,
        "exchanges": nex,
        "per_rank": per_rank,
        "max_mem_gb": (torch.cuda.max_memory_allocated() / 1e9) if device.startswith("cuda") else 0.0,
    }
    del scheme, halo, ops
    if device.startswith("cuda"):
        torch.cuda.empty_cache()
    return res


# BASELINE.json physics configs timed next to the headline on one GPU
# (``--physics-companion``): the driver's own record then carries them.  The
# command lines are the ones tools/bench_configs.py uses (reference scenes:
# zero fields, plane wave / dipole sources, default 10-cell layers and
# TF/SF distance 20).
PHYSICS_CONFIGS = (
    ("cpml_tfsf_512", "3D 512^3 CPML (10 cells) + TF/SF plane wave, fp32 (BASELINE config 3)",
     ["--3d", "--sizex", "512", "--same-size", "--dtype", "f32", "--scene", "vacuum", "--use-pml",
      "--pml-type", "cpml", "--use-tfsf"]),
    ("drude_512", "3D 512^3 Drude sphere r=128 in vacuum, no absorbing layer, fp32 (BASELINE config 4 as named)",
     ["--3d", "--sizex", "512", "--same-size", "--dtype", "f32", "--scene", "drude-sphere", "--use-metamaterials",
      "--sphere-center-x", "256", "--sphere-center-y", "256", "--sphere-center-z", "256", "--sphere-radius", "128"]),
    ("drude_upml_512", "3D 512^3 Drude sphere r=128 + UPML, fp32 (BASELINE config 4 with absorbing layers)",
     ["--3d", "--sizex", "512", "--same-size", "--dtype", "f32", "--scene", "drude-sphere", "--use-metamaterials",
      "--use-pml", "--sphere-center-x", "256", "--sphere-center-y", "256", "--sphere-center-z", "256",
      "--sphere-radius", "128"]),
)
# the same configs in fp64, the reference's default value type (CMakeLists.txt VALUE_TYPE "d")
PHYSICS_CONFIGS += tuple(
    (name + "_f64", desc.replace("fp32", "fp64 (the reference's default value type)"),
     [("f64" if v == "f32" else v) for v in args])
    for name, desc, args in PHYSICS_CONFIGS)


def physics_args(args, n: int):
    """A physics config's command line on an n^3 grid (sphere scaled along)."""
    out = list(args)
    for i, v in enumerate(out):
        if i and out[i - 1] == "--sizex":
            out[i] = str(n)
        elif i and out[i - 1].startswith("--sphere-"):
            out[i] = str(int(v) * n // 512)
    return out


def run_physics(args, steps: int, warmup: int) -> dict:
    """One physics config through the regular driver path (runner.build):
    ``warmup`` untimed steps, then ``steps`` timed steps between device syncs."""
    import torch
    from fdtd3d_amd.runner import build
    from fdtd3d_amd.utils.settings import setup_from_cmd

    # (the steps are rounded up to whole passes below: T <= 8, so 8 x 8 more at most)
    status, settings = setup_from_cmd(list(args) + ["--time-steps", str(warmup + steps + 64)],
                                      out=open(os.devnull, "w"))
    if torch.cuda.is_available():
        torch.cuda.reset_peak_memory_stats()
    if status != 0:
        raise RuntimeError("bad physics config %s" % " ".join(args))
    scheme, _, _ = build(settings)
    scheme.init_scheme()
    scheme.init_grids()
    # whole blocked / hybrid passes in both phases: a pass cut short costs about a whole
    # pass (Drude + UPML at T = 4 timed over 30 steps: 75.5k vs 81k Mcells/s over whole passes)
    hyb = getattr(scheme, "hybrid", None)
    per = int(hyb["T"]) if hyb else max(1, int(getattr(scheme, "tb", 1)))
    warmup = -(-warmup // per) * per
    steps = -(-steps // per) * per
    scheme.perform_steps(warmup)
    cuda = scheme.device.type == "cuda"
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    scheme.perform_steps(steps)
    if cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    size = scheme.cfg.size
    res = {"value": round(size[0] * size[1] * size[2] * steps / dt / 1e6, 1),
           "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps, "warmup": warmup,
           "hybrid": scheme.hybrid.get("kind", "stepped-shell") if getattr(scheme, "hybrid", None) else "none",
           "energy": scheme.field_energy(),
           "max_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2) if cuda else 0.0}
    del scheme
    if cuda:
        torch.cuda.empty_cache()
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", type=int, nargs=3, default=list(HEADLINE_SIZE))
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--topology", default="auto",
                    help="rank grid: auto, an axis set for the optimiser (x, xy, xyz, ...) or explicit AxBxC")
    ap.add_argument("--init", default="random", choices=("random", "zero"),
                    help="initial fields: hash of the global cell index (random) or zero")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--fp64-companion", default="auto", choices=("auto", "on", "off"),
                    help="repeat the measurement in fp64 and report it under 'fp64' (auto: one GPU, fp32 runs)")
    ap.add_argument("--physics-companion", default="auto", choices=("auto", "on", "off"),
                    help="also time the 512^3 CPML + TF/SF, Drude and Drude + UPML configs and report them "
                         "under 'physics' (auto: one GPU, fp32 runs)")
    ap.add_argument("--physics-steps", type=int, default=30, help="timed steps (rounded up to whole passes)")
    ap.add_argument("--physics-warmup", type=int, default=45,
                    help="untimed steps before the physics configs' timed ones (hybrid passes capture their HIP "
                         "graph there)")
    ap.add_argument("--physics-size", type=int, default=512, help="edge of the physics configs' cubic grid")
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
    ap.add_argument("--timeout", type=float, default=300.0, help="collective timeout (s): a hung exchange aborts")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    from fdtd3d_amd.ops import resolve_backend

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
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
        init_process_group("nccl" if use_nccl else "gloo", device if use_nccl else None, timeout_s=a.timeout)
        # establish the communicator with a collective before the first
        # batched point-to-point exchange
        dist.barrier()

    size = tuple(a.size)
    core = parse_topology(a.topology, size, world, a.time_block != 1) if world > 1 else None
    topo = core.topology if core is not None else (1, 1, 1)
    res = run_one(a, a.dtype, world, rank, device, backend, core)
    fp64 = None
    companion = a.fp64_companion == "on" or (a.fp64_companion == "auto" and world == 1 and a.dtype == "f32"
                                              and backend == "hip")
    if companion:
        try:
            fp64 = run_one(a, "f64", world, rank, device, backend, core)
        except Exception as e:  # the headline line must still be printed
            fp64 = {"error": "%s: %s" % (type(e).__name__, e)}
    physics = None
    if a.physics_companion == "on" or (a.physics_companion == "auto" and world == 1 and a.dtype == "f32"
                                       and backend == "hip"):
        physics = {}
        for name, desc, args in PHYSICS_CONFIGS:
            try:
                physics[name] = dict(run_physics(physics_args(args, a.physics_size), a.physics_steps, a.physics_warmup),
                                     desc=desc)
            except Exception as e:  # the headline line must still be printed
                physics[name] = {"error": "%s: %s" % (type(e).__name__, e), "desc": desc}
    if rank == 0:
        par = "x".join(str(v) for v in topo)
        cells = size[0] * size[1] * size[2]
        out = {
            "metric": metric_name(size),
            "value": round(res["mcells"], 1),
            "unit": "Mcells/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(res["dt"] / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32" if a.dtype == "f32" else "fp64",
            "data": ("synthetic (random-init fields: hash of the global cell index, + hard point-dipole Ez source, "
                     "vacuum)" if a.init == "random" else "synthetic (zero fields + hard point-dipole Ez source, "
                                                           "vacuum)"),
            "config": {
                "model": "fdtd3d 3D Yee leapfrog, vacuum, point dipole (BASELINE.json headline)",
                "grid": "%dx%dx%d" % size,
                "global_batch": 1,
                "seq_len": cells,
                "parallelism": "domain-decomposition %s (dp%d-equivalent ranks)" % (par, world),
                "backend": backend,
                "time_block": res["tb"],
                "halo_bytes_per_step": res["halo_bytes"] // max(1, a.steps),
                "halo_ms_per_pass_max": round(res["halo_ms_per_pass_max"], 4),
                "halo_ms_per_pass_mean": round(res["halo_ms_per_pass_mean"], 4),
            },
            "checksum": {"energy0": res["energy0"], "energy": res["energy"],
                         "steps_total": a.warmup + a.steps},
            "max_mem_gb_rank0": round(res["max_mem_gb"], 2),
        }
        if res["per_rank"]:
            # ms per pass on each rank's main stream: interior (overlapped with
            # the exchange on the side stream), exchange_wait (the part of the
            # exchange the interior did not hide), shell; exchange_ms = the
            # exchange's own duration on the side stream
            out["per_rank"] = res["per_rank"]
        if fp64 is not None:
            if "error" in fp64:
                out["fp64"] = fp64
            else:
                out["fp64"] = {"value": round(fp64["mcells"], 1), "ms_per_step": round(fp64["dt"] / a.steps * 1e3, 4),
                               "time_block": fp64["tb"], "energy": fp64["energy"]}
        if physics is not None:
            out["physics"] = physics
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
