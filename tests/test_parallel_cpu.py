"""Domain decomposition on CPU (gloo): a decomposed run must reproduce the
serial run on the same global grid.

The reference's only test (``Tests/unit-test-parallel-grid.cpp``) checks that
after ``share()`` + ``gatherFullGrid()`` every cell is owned by the right
rank; it never checks halo *contents* or physics.  Here the whole solver runs
decomposed (face mode ``--buffer-size 1`` and deep halo ``--buffer-size 2/3``)
and the gathered fields are compared with a serial run, plus a halo-content
check that ghost cells equal the neighbour's interior.
"""

import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops
from fdtd3d_amd.parallel.halo import HaloExchanger, gather_field
from fdtd3d_amd.parallel.topology import ParallelGridCore


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, topo_axes, buf, outdir, mode="direct", split=None, random_init=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        core = ParallelGridCore.create(cfg.size, world, topo_axes,
                                       active_axes=(0, 1, 2) if cfg.scheme == "3d" else ((0, 1) if cfg.scheme in ("tmz", "tez") else (0,)))
        dom = core.domain(rank, buf, align_z=4 if cfg.time_block > 1 else 1,
                          align_axis=2 if cfg.scheme == "3d" else 1)
        halo = HaloExchanger(dom, mode=mode)
        s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64), dom, halo)
        s.init_scheme()
        s.init_grids()
        assert s.tb == max(1, cfg.time_block)
        if cfg.hybrid_block > 1:
            assert s.hybrid is not None, "hybrid pass not selected on rank %d" % rank
        if random_init:
            s.randomize_fields()
        for n in (split or (cfg.time_steps,)):
            s.perform_steps(n)
        halo.drain(s)
        res = {}
        for p in range(s.planes):
            for c in s.comps:
                full = gather_field(s, c, p)
                if rank == 0:
                    res["%s%d" % (c, p)] = full
        if rank == 0:
            res["topology"] = torch.tensor(core.topology)
            torch.save(res, os.path.join(outdir, "par.pt"))
    finally:
        dist.destroy_process_group()


def run_parallel(cfg, world, axes="xyz", buf=1, mode="direct", split=None, random_init=False):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), cfg, axes, buf, d, mode, split, random_init), nprocs=world,
                 join=True)
        return torch.load(os.path.join(d, "par.pt"), weights_only=True)


def run_serial(cfg, random_init=False):
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    if random_init:
        s.randomize_fields()
    s.perform_steps()
    return s


CASES = [
    ("vacuum-x2", SchemeConfig(scheme="3d", size=(20, 14, 12), time_steps=12, scene="vacuum"), 2, "x", 1),
    ("vacuum-xyz4", SchemeConfig(scheme="3d", size=(16, 18, 14), time_steps=12, scene="vacuum"), 4, "xyz", 1),
    ("pml-tfsf-yz4", SchemeConfig(scheme="3d", size=(24, 24, 24), time_steps=10, use_pml=True, use_tfsf=True,
                                  pml_size=(4, 4, 4), tfsf_size=(8, 8, 8), theta=50, phi=20, psi=30), 4, "yz", 1),
    ("drude-z2", SchemeConfig(scheme="3d", size=(64, 64, 30), time_steps=6, use_pml=True, use_metamaterials=True,
                              pml_size=(4, 4, 4)), 2, "z", 1),
    ("deep-halo-x2-b3", SchemeConfig(scheme="3d", size=(24, 12, 12), time_steps=10, scene="vacuum"), 2, "x", 3),
    ("deep-halo-xyz8-b2", SchemeConfig(scheme="3d", size=(16, 16, 16), time_steps=7, use_pml=True,
                                       pml_size=(3, 3, 3)), 8, "xyz", 2),
    ("tmz-xy4", SchemeConfig(scheme="tmz", size=(40, 36, 1), time_steps=20, use_pml=True, pml_size=(5, 5, 1)), 4,
     "xy", 1),
    ("tez-x2-complex", SchemeConfig(scheme="tez", size=(30, 30, 1), time_steps=15, scene="vacuum",
                                    complex_values=True), 2, "x", 1),
    ("1d-x4", SchemeConfig(scheme="1d", size=(200, 1, 1), time_steps=80, scene="vacuum", source="gaussian"), 4,
     "x", 1),
    ("fused-xyz8-b1", SchemeConfig(scheme="3d", size=(18, 16, 20), time_steps=9, scene="sphere", sphere_radius=5,
                                   sphere_center=(9.5, 8.5, 10.5), use_fused=True), 8, "xyz", 1),
    ("fused-xy4-b2", SchemeConfig(scheme="3d", size=(20, 20, 12), time_steps=9, scene="vacuum", use_fused=True,
                                  complex_values=True), 4, "xy", 2),
    # hybrid passes in decomposed runs: blocked core (owned part of the global
    # core) + deep-halo stepped shell, one T-deep exchange (aux state included)
    ("hybrid-upml-tfsf-xy4-b3", SchemeConfig(scheme="3d", size=(80, 80, 80), time_steps=8, use_pml=True,
                                             use_tfsf=True, pml_size=(4, 4, 4), tfsf_size=(8, 8, 8), theta=50,
                                             phi=20, psi=30, hybrid_block=3), 4, "xy", 3),
    ("hybrid-cpml-point-xyz8-b2", SchemeConfig(scheme="3d", size=(64, 64, 64), time_steps=7, use_pml=True,
                                               pml_type="cpml", pml_size=(4, 4, 4), scene="vacuum",
                                               hybrid_block=2), 8, "xyz", 2),
    ("deep-drude-z2-b3", SchemeConfig(scheme="3d", size=(64, 64, 72), time_steps=7, use_pml=True,
                                      use_metamaterials=True, scene="drude-sphere", sphere_radius=4,
                                      sphere_center=(32.0, 32.0, 36.0), pml_size=(4, 4, 4), hybrid_block=1),
     2, "z", 3),
    ("hybrid-drude-off-z2-b3", SchemeConfig(scheme="3d", size=(64, 64, 72), time_steps=7, use_pml=True,
                                            use_metamaterials=True, scene="drude-sphere", sphere_radius=4,
                                            sphere_center=(32.0, 32.0, 20.0), pml_size=(4, 4, 4), hybrid_block=3),
     2, "z", 3),
    ("hybrid-drude-z2-b3", SchemeConfig(scheme="3d", size=(64, 64, 72), time_steps=7, use_pml=True,
                                        use_metamaterials=True, scene="drude-sphere", sphere_radius=4,
                                        sphere_center=(32.0, 32.0, 36.0), pml_size=(4, 4, 4), hybrid_block=3),
     2, "z", 3),
    # no PML: the core reaches the domain faces; the dispersive box straddles
    # the rank boundary (per-row material ranges on both ranks)
    ("hybrid-drude-nopml-xy4-b3", SchemeConfig(scheme="3d", size=(48, 44, 40), time_steps=8,
                                               use_metamaterials=True, scene="drude-sphere", sphere_radius=5,
                                               sphere_center=(24.0, 22.0, 20.0), hybrid_block=3),
     4, "xy", 3),
    # temporal blocking: T steps per pass, T-deep ghosts exchanged every T steps
    ("tb2-xyz8", SchemeConfig(scheme="3d", size=(16, 18, 20), time_steps=9, scene="vacuum", use_fused=True,
                              time_block=2), 8, "xyz", 2),
    ("tb2-z2-pad", SchemeConfig(scheme="3d", size=(10, 12, 26), time_steps=6, scene="vacuum", use_fused=True,
                                time_block=2), 2, "z", 2),
    ("tb4-xy4", SchemeConfig(scheme="3d", size=(20, 22, 16), time_steps=11, scene="vacuum", use_fused=True,
                             time_block=4), 4, "xy", 4),
    ("tb3-x2-sphere", SchemeConfig(scheme="3d", size=(22, 12, 16), time_steps=10, scene="sphere", sphere_radius=4,
                                   sphere_center=(11.0, 6.0, 8.0), use_fused=True, time_block=3), 2, "x", 3),
    ("tb5-xy4", SchemeConfig(scheme="3d", size=(24, 26, 16), time_steps=12, scene="vacuum", use_fused=True,
                             time_block=5), 4, "xy", 5),
    # 2D blocked passes (yee2d_tb.hip path): y extent padded to whole float4 rows
    ("tmz-tb4-xy4", SchemeConfig(scheme="tmz", size=(40, 34, 1), time_steps=13, scene="vacuum", use_fused=True,
                                 time_block=4), 4, "xy", 4),
    ("tez-tb7-y2-complex", SchemeConfig(scheme="tez", size=(30, 50, 1), time_steps=16, scene="vacuum",
                                        use_fused=True, complex_values=True, time_block=7), 2, "y", 7),
    # the axis-sweep deep-halo exchange (edges / corners relayed through faces)
    ("sweep-deep-halo-xyz8-b2", SchemeConfig(scheme="3d", size=(16, 16, 16), time_steps=7, use_pml=True,
                                             pml_size=(3, 3, 3)), 8, "xyz", 2, "sweep"),
    ("sweep-tb4-xy4", SchemeConfig(scheme="3d", size=(20, 22, 16), time_steps=11, scene="vacuum", use_fused=True,
                                   time_block=4), 4, "xy", 4, "sweep"),
]


@pytest.mark.parametrize("name,cfg,world,axes,buf,mode", [c if len(c) == 6 else c + ("direct",) for c in CASES],
                         ids=[c[0] for c in CASES])
def test_decomposed_equals_serial(name, cfg, world, axes, buf, mode):
    par = run_parallel(cfg, world, axes, buf, mode)
    ser = run_serial(cfg)
    for p in range(ser.planes):
        for c in ser.comps:
            a = par["%s%d" % (c, p)]
            b = ser.F[p][c]
            # per kind: a near-silent component is compared on its kind's scale
            scale = max(float(ser.F[p][o].abs().max()) for o in ser.comps if o[0] == c[0]) + 1e-300
            err = float((a - b).abs().max())
            if err > 1e-12 * scale:
                d = (a - b).abs()
                zs = [(z, float(d[:, :, z].max())) for z in range(d.shape[2]) if float(d[:, :, z].max()) > 1e-12 * scale]
                xs = [(x, float(d[x].max())) for x in range(d.shape[0]) if float(d[x].max()) > 1e-12 * scale]
                print("ERRMAP", name, c, "z", zs[:12], "x", xs[:12])
            assert err <= 1e-12 * scale, (name, c, err, scale, par["topology"].tolist())


@pytest.mark.parametrize("name,split", [("hybrid-upml-tfsf-xy4-b3", (2, 3, 3)),
                                        ("hybrid-cpml-point-xyz8-b2", (1, 3, 3))])
def test_decomposed_hybrid_split_passes(name, split):
    """A decomposed hybrid run advanced in pieces that are not multiples of T
    (passes cut short, as periodic work does), from random fields (every
    rank-boundary cell of the stepped shell carries signal), equals one serial
    run: every pass's exchange restarts the deep-halo sub-step."""
    _, cfg, world, axes, buf = [c for c in CASES if c[0] == name][0]
    assert sum(split) == cfg.time_steps
    par = run_parallel(cfg, world, axes, buf, split=split, random_init=True)
    ser = run_serial(cfg, random_init=True)
    for c in ser.comps:
        b = ser.F[0][c]
        err = float((par["%s0" % c] - b).abs().max())
        assert err <= 1e-12 * (float(b.abs().max()) + 1e-300), (name, c, err)


def _ntff_worker(rank, world, port, cfg, axes, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import io
        from fdtd3d_amd.models.ntff import ntff_report
        core = ParallelGridCore.create(cfg.size, world, axes)
        dom = core.domain(rank, 1)
        s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64), dom, HaloExchanger(dom))
        s.init_scheme()
        s.init_grids()
        s.perform_steps()
        p = ntff_report(s, s.t, out=io.StringIO())
        if rank == 0:
            torch.save({"p": p}, os.path.join(outdir, "ntff.pt"))
        else:
            assert p is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,axes", [(4, "xyz"), (8, "xyz")])
def test_decomposed_ntff_equals_serial(world, axes):
    """The decomposed NTFF diagram gathers only the face slabs (gather_box)
    and must equal the serial diagram."""
    import io
    from fdtd3d_amd.models.ntff import ntff_report
    cfg = SchemeConfig(scheme="3d", size=(22, 20, 24), time_steps=14, scene="vacuum", use_pml=True,
                       pml_size=(3, 3, 3), use_tfsf=True, tfsf_size=(5, 5, 5), ntff_size=(4, 4, 4),
                       complex_values=True, theta=60, phi=30, psi=10)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ntff_worker, args=(world, _free_port(), cfg, axes, d), nprocs=world, join=True)
        par = torch.load(os.path.join(d, "ntff.pt"), weights_only=True)["p"]
    ser = ntff_report(run_serial(cfg), cfg.time_steps, out=io.StringIO())
    assert float(ser.abs().max()) > 0
    assert torch.allclose(par, ser, rtol=1e-10, atol=0), float((par - ser).abs().max())
