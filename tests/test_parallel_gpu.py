"""Decomposed runs through the HIP kernels on ONE GPU (GPU only).

The ranks are threads of the test process talking through the in-process
:class:`~fdtd3d_amd.parallel.comm.LocalHub` transport (RCCL refuses several
ranks on one device, and spawning processes from a GPU-initialised test
process is not allowed on the GPU pool).  This exercises the GPU pack/unpack
kernels, the split face-mode overlap, the interior/shell split of the
overlapped fused step and its side stream, and compares the assembled global
fields with a serial HIP run.
"""

import threading

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops
from fdtd3d_amd.parallel.comm import LocalHub
from fdtd3d_amd.parallel.halo import HaloExchanger
from fdtd3d_amd.parallel.topology import ParallelGridCore

pytestmark = pytest.mark.gpu


def run_threads(cfg, world, axes, buf, device, delay_cycles=0, skip_side_wait=False, split=None,
                random_init=False, check=None):
    """Decomposed run with one thread per rank, each on its OWN main stream
    (like one process per GPU): the in-process transport orders streams with
    events only, so every cross-stream dependency must be explicit.
    ``delay_cycles`` holds every ghost unpack back on the exchange stream;
    ``skip_side_wait`` drops the main stream's wait on it (negative control);
    ``split`` = (steps, ...) runs perform_steps in pieces (passes cut short);
    ``check(scheme)`` runs on every rank before the steps."""
    core = ParallelGridCore.create(cfg.size, world, axes, active_axes=(0, 1, 2) if cfg.scheme == "3d" else (0, 1))
    hub = LocalHub(world)
    dt = torch.float32 if cfg.dtype == "f32" else torch.float64
    schemes = [None] * world
    errors = []

    def body(rank):
        try:
            stream = torch.cuda.Stream(device=device)
            with torch.cuda.stream(stream):
                dom = core.domain(rank, buf, align_z=4 if (cfg.time_block > 1 or cfg.hybrid_block > 1) else 1,
                                  align_axis=2 if cfg.scheme == "3d" else 1)
                halo = HaloExchanger(dom, comm=hub.comm(rank))
                halo.debug_delay_cycles = delay_cycles
                s = YeeScheme(cfg, make_ops("hip", None, device, dt), dom, halo)
                s._skip_side_wait = skip_side_wait
                s.init_scheme()
                s.init_grids()
                # time_block 0: the automatic rule must pick the ghost depth the
                # driver sized the domain for (models/blocking.py auto_time_block)
                if cfg.hybrid_block > 1:
                    assert s.hybrid is not None, "hybrid pass not selected"
                else:
                    assert s.tb == (buf if cfg.time_block == 0 else max(1, cfg.time_block))
                if random_init:
                    s.randomize_fields()
                if check is not None:
                    check(s)
                if split:
                    for n in split:
                        s.perform_steps(n)
                else:
                    s.perform_steps()
                halo.drain(s)
            torch.cuda.synchronize()
            schemes[rank] = s
        except BaseException as e:  # surface thread failures in the test
            errors.append(e)

    ths = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    if errors:
        raise errors[0]
    full = {}
    for c in schemes[0].comps:
        f = torch.zeros(cfg.size, dtype=torch.float64)
        for s in schemes:
            d = s.domain
            f[d.lo[0]:d.hi[0], d.lo[1]:d.hi[1], d.lo[2]:d.hi[2]] = s.owned_field(c).double().cpu()
        full[c] = f
    return full


CASES = [
    ("split-face-x2", SchemeConfig(scheme="3d", size=(32, 24, 40), time_steps=12, scene="vacuum", dtype="f32"),
     2, "x", 1),
    ("split-pml-tfsf-xy4", SchemeConfig(scheme="3d", size=(32, 32, 32), time_steps=10, use_pml=True, use_tfsf=True,
                                        pml_size=(4, 4, 4), tfsf_size=(8, 8, 8), dtype="f64"), 4, "xy", 1),
    ("fused-overlap-xyz8", SchemeConfig(scheme="3d", size=(40, 36, 64), time_steps=11, scene="sphere",
                                        sphere_radius=8, sphere_center=(20.5, 17.5, 30.5), dtype="f32",
                                        use_fused=True), 8, "xyz", 1),
    ("fused-deep-b2-yz2", SchemeConfig(scheme="3d", size=(24, 40, 48), time_steps=9, scene="vacuum", dtype="f32",
                                       use_fused=True), 2, "yz", 2),
    # temporally blocked kernel, 2-deep ghosts every 2 steps; z split needs the
    # alignment padding (local nz = 34 + 2)
    ("tb2-xyz8", SchemeConfig(scheme="3d", size=(40, 36, 64), time_steps=11, scene="vacuum", dtype="f32",
                              use_fused=True, time_block=2), 8, "xyz", 2),
    ("tb4-xy4", SchemeConfig(scheme="3d", size=(44, 40, 256), time_steps=13, scene="vacuum", dtype="f32",
                             use_fused=True, time_block=4), 4, "xy", 4),
    ("tb2-z2-sphere", SchemeConfig(scheme="3d", size=(24, 30, 520), time_steps=8, scene="sphere", sphere_radius=9,
                                   sphere_center=(12.0, 15.0, 260.0), dtype="f32", use_fused=True, time_block=2),
     2, "z", 2),
    # multi-row kernel (5 steps per pass, 5-deep ghosts, direct 26-neighbour exchange)
    ("tb5-xy4", SchemeConfig(scheme="3d", size=(60, 56, 128), time_steps=13, scene="vacuum", dtype="f32",
                             use_fused=True, time_block=5), 4, "xy", 5),
    # automatic steps per pass on a dielectric (sparse per-cell) scene, 4 ranks -> T = 4
    ("auto-sphere-xy4", SchemeConfig(scheme="3d", size=(48, 44, 128), time_steps=13, scene="sphere", sphere_radius=10,
                                     sphere_center=(24.0, 20.0, 64.0), dtype="f32", use_fused=True, time_block=0),
     4, "xy", 4),
    # hybrid passes on decomposed ranks (blocked core + deep-halo stepped shell)
    ("hybrid-cpml-tfsf-xy4", SchemeConfig(scheme="3d", size=(96, 96, 96), time_steps=10, scene="vacuum", dtype="f32",
                                          use_pml=True, pml_type="cpml", use_tfsf=True, pml_size=(5, 5, 5),
                                          tfsf_size=(10, 10, 10), use_fused=True, hybrid_block=4), 4, "xy", 4),
    # UPML + TF/SF: automatic mode puts the TF/SF faces inside the blocked core
    # (models/blocking.py _hybrid_core_tfsf), split over an x / y rank grid
    ("hybrid-upml-tfsf-xy4", SchemeConfig(scheme="3d", size=(96, 88, 96), time_steps=10, scene="vacuum", dtype="f32",
                                          use_pml=True, pml_type="upml", use_tfsf=True, pml_size=(5, 5, 5),
                                          tfsf_size=(8, 8, 8), use_fused=True, hybrid_block=4), 4, "xy", 4),
    ("hybrid-upml-drude-z2", SchemeConfig(scheme="3d", size=(80, 80, 96), time_steps=9, dtype="f32", use_pml=True,
                                          use_metamaterials=True, scene="drude-sphere", sphere_radius=6,
                                          sphere_center=(40.0, 40.0, 48.0), pml_size=(5, 5, 5), use_fused=True,
                                          hybrid_block=3, blocked_drude="off"), 2, "z", 3),
    # (the serial run keeps the stepped dispersive box too: random initial fields break the E = D1
    # invariant the blocked Drude pass relies on, and decomposed runs step the box)
    # fp64 blocked kernel
    ("tb4-f64-xyz8", SchemeConfig(scheme="3d", size=(40, 36, 44), time_steps=10, scene="vacuum", dtype="f64",
                                  use_fused=True, time_block=4), 8, "xyz", 4),
    # 2D blocked kernel (yee2d_tb.hip), local y extents padded to float4 rows
    ("tmz-tb7-xy4", SchemeConfig(scheme="tmz", size=(300, 290, 1), time_steps=17, scene="vacuum", dtype="f32",
                                 use_fused=True, time_block=7), 4, "xy", 7),
    ("tez-tb6-y2", SchemeConfig(scheme="tez", size=(100, 522, 1), time_steps=15, scene="vacuum", dtype="f32",
                                use_fused=True, time_block=6), 2, "y", 6),
]


def _serial(cfg, gpu, random_init=False):
    dt = torch.float32 if cfg.dtype == "f32" else torch.float64
    s = YeeScheme(cfg, make_ops("hip", None, gpu, dt))
    s.init_scheme()
    s.init_grids()
    if random_init:
        s.randomize_fields()
    s.perform_steps()
    return s


def _max_rel_err(par, s):
    worst = 0.0
    for c in s.comps:
        b = s.F[0][c].double().cpu()
        scale = max(float(s.F[0][o].abs().max()) for o in s.comps if o[0] == c[0]) + 1e-30
        worst = max(worst, float((par[c] - b).abs().max()) / scale)
    return worst


@pytest.mark.parametrize("name,cfg,world,axes,buf", CASES, ids=[c[0] for c in CASES])
def test_gpu_decomposed_equals_serial(gpu, name, cfg, world, axes, buf):
    par = run_threads(cfg, world, axes, buf, gpu)
    s = _serial(cfg, gpu)
    for c in s.comps:
        a = par[c]
        b = s.F[0][c].double().cpu()
        scale = max(float(s.F[0][o].abs().max()) for o in s.comps if o[0] == c[0]) + 1e-30
        err = float((a - b).abs().max())
        # the serial hybrid may run the single-pass shell kernel while the
        # decomposed ranks run the stepped shell: fp32 rounding of two kernels
        assert err <= (5e-6 if name.startswith("hybrid") else 1e-6) * scale, (name, c, err, scale)


# the exchange overlapped with the interior / core pass on the side stream
STREAM_CASES = [c for c in CASES if c[0] in ("tb5-xy4", "hybrid-cpml-tfsf-xy4", "hybrid-upml-drude-z2")]
DELAY = 40_000_000  # GPU clock cycles of torch.cuda._sleep before every ghost unpack (~20 ms)


@pytest.mark.parametrize("name,cfg,world,axes,buf", STREAM_CASES, ids=[c[0] for c in STREAM_CASES])
def test_gpu_side_stream_order(gpu, name, cfg, world, axes, buf):
    """Every unpack is held back ~20 ms on the side stream: the decomposed
    result still equals the serial one (the main stream waits for the
    exchange) -- and with that wait removed it does NOT (negative control:
    proves the test sees a missing stream dependency)."""
    s = _serial(cfg, gpu, random_init=True)
    ok = run_threads(cfg, world, axes, buf, gpu, delay_cycles=DELAY, random_init=True)
    assert _max_rel_err(ok, s) <= 1e-5, name
    bad = run_threads(cfg, world, axes, buf, gpu, delay_cycles=DELAY, skip_side_wait=True, random_init=True)
    assert _max_rel_err(bad, s) > 1e-3, "%s: a missing side-stream wait went unnoticed" % name


def test_gpu_hybrid_split_passes(gpu):
    """Decomposed hybrid run advanced in pieces that are not multiples of T
    (passes cut short, as periodic work does): equals one serial run
    (the deep-halo sub-step must restart with every exchange)."""
    name, cfg, world, axes, buf = [c for c in CASES if c[0] == "hybrid-cpml-tfsf-xy4"][0]
    s = _serial(cfg, gpu, random_init=True)
    par = run_threads(cfg, world, axes, buf, gpu, split=(2, 4, 3, 1), random_init=True)
    assert _max_rel_err(par, s) <= 1e-5


DRUDE = dict(scheme="3d", dtype="f32", scene="drude-sphere", use_metamaterials=True, use_fused=True,
             blocked_drude="on")
DRUDE_CASES = [
    # plain blocked passes + the Drude pass, the sphere across the x / y rank borders
    ("drude-tb4-xy4", SchemeConfig(size=(80, 72, 96), time_steps=23, sphere_center=(40.0, 36.0, 48.0),
                                   sphere_radius=9.0, time_block=4, **DRUDE), 4, "xy", 4),
    # the reference's scattering scene (Drude sphere + UPML + TF/SF, incidence along x: the faces in the
    # blocked core) on hybrid passes; the sphere across the y border, inside the x = 0..48 ranks
    ("drude-upml-tfsf-xy4", SchemeConfig(size=(96, 96, 100), time_steps=48, sphere_center=(30.0, 48.0, 50.0),
                                         sphere_radius=6.0, use_pml=True, pml_size=(5, 5, 5), use_tfsf=True,
                                         tfsf_size=(9, 9, 9), hybrid_block=4, time_block=4, **DRUDE), 4, "xy", 4),
]


@pytest.mark.parametrize("name,cfg,world,axes,buf", DRUDE_CASES, ids=[c[0] for c in DRUDE_CASES])
def test_gpu_decomposed_drude_blocked(gpu, name, cfg, world, axes, buf):
    """The Drude box inside decomposed blocked / hybrid passes (its state in
    the deep exchange, the pass after the exchange join) on the HIP kernels:
    equals the serial blocked run and the serial stepped chain."""
    seen = []

    def check(s):
        seen.append((s.drude_blk is not None, s._drude_glob is not None))

    par = run_threads(cfg, world, axes, buf, gpu, check=check)
    assert all(g for _, g in seen) and any(d for d, _ in seen), seen
    import dataclasses
    blk = _serial(cfg, gpu)
    assert blk.drude_blk is not None
    st = _serial(dataclasses.replace(cfg, blocked_drude="off", hybrid_block=1, time_block=1, use_fused=False), gpu)
    assert st.drude_blk is None
    assert _max_rel_err(par, blk) <= 5e-6, name
    assert _max_rel_err(par, st) <= 2e-5, name


@pytest.mark.parametrize("name", ["hybrid-cpml-tfsf-xy4", "tb4-xy4"])
def test_gpu_listed_exchange_bitwise(gpu, name, monkeypatch):
    """The direct exchange from a cached plan (one box-list pack and unpack
    launch, parallel/halo.py _exchange_direct_listed) moves exactly the
    bytes of the per-message, per-array form: the decomposed runs agree bit
    for bit."""
    _, cfg, world, axes, buf = [c for c in CASES if c[0] == name][0]
    a = run_threads(cfg, world, axes, buf, gpu, random_init=True)
    monkeypatch.setattr(HaloExchanger, "listed", False)
    b = run_threads(cfg, world, axes, buf, gpu, random_init=True)
    for c in a:
        assert torch.equal(a[c], b[c]), (name, c)
