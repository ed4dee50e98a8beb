"""Decomposed runs over a transport that ignores tags (CPU).

RCCL matches point-to-point operations per peer pair in posting order; it
ignores tags.  The gloo tests (``test_parallel_cpu.py``) match by tag, so an
op list whose per-peer order differs between the two sides of a message would
pass there and deliver wrong ghosts over RCCL.  Here the ranks are threads
talking through :class:`~fdtd3d_amd.parallel.comm.LocalHub` with
``tagless=True`` (one FIFO per sender / receiver pair, receives checked for
equal sizes): the decomposed run must still equal the serial one, over face
mode, the direct 26-neighbour deep exchange (x faces straight from the
arrays), the sweep exchange and hybrid passes with region-local auxiliary
arrays.  Also: the direct exchange with and without the unpacked x faces is
bit-for-bit the same, and the Drude box inside decomposed blocked
/ hybrid passes (its float4-per-cell state in the deep exchange, ranks the box
misses, a box across rank borders) equals the serial stepped chain.
"""

import threading

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops
from fdtd3d_amd.parallel.comm import LocalHub
from fdtd3d_amd.parallel.halo import HaloExchanger
from fdtd3d_amd.parallel.topology import ParallelGridCore


def run_threads(cfg, world, axes, buf, mode="direct", direct_x=True, tagless=True, randomize=True,
                check=None):
    core = ParallelGridCore.create(cfg.size, world, axes)
    hub = LocalHub(world, tagless=tagless)
    out, errors = [None] * world, []

    def body(rank):
        try:
            dom = core.domain(rank, buf, align_z=4 if cfg.time_block > 1 else 1)
            halo = HaloExchanger(dom, comm=hub.comm(rank), mode=mode)
            halo.direct_x_faces = direct_x
            s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64), dom, halo)
            s.init_scheme()
            s.init_grids()
            if randomize:
                s.randomize_fields()
            if check is not None:
                check(s)
            s.perform_steps()
            halo.drain(s)
            out[rank] = s
        except BaseException as e:  # surface thread failures in the test
            errors.append(e)

    torch.set_num_threads(1)
    ths = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    if errors:
        raise errors[0]
    full = {}
    for c in out[0].comps:
        f = torch.zeros(cfg.size, dtype=torch.float64)
        for s in out:
            d = s.domain
            f[d.lo[0]:d.hi[0], d.lo[1]:d.hi[1], d.lo[2]:d.hi[2]] = s.owned_field(c)
        full[c] = f
    return full


def serial(cfg, randomize=True):
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    if randomize:
        s.randomize_fields()
    s.perform_steps()
    return {c: s.F[0][c] for c in s.comps}


CASES = [
    ("face-xyz8", SchemeConfig(scheme="3d", size=(16, 18, 14), time_steps=7, scene="vacuum"), 8, "xyz", 1, "direct"),
    ("tb4-xyz8", SchemeConfig(scheme="3d", size=(20, 22, 24), time_steps=9, scene="vacuum", use_fused=True,
                              time_block=4), 8, "xyz", 4, "direct"),
    ("deep-upml-xyz8-b2", SchemeConfig(scheme="3d", size=(16, 16, 16), time_steps=6, use_pml=True,
                                       pml_size=(3, 3, 3)), 8, "xyz", 2, "direct"),
    ("hybrid-upml-tfsf-xy4-b3", SchemeConfig(scheme="3d", size=(48, 48, 40), time_steps=7, use_pml=True,
                                             use_tfsf=True, pml_size=(4, 4, 4), tfsf_size=(8, 8, 8), theta=50,
                                             phi=20, psi=30, hybrid_block=3), 4, "xy", 3, "direct"),
    ("sweep-tb3-xy4", SchemeConfig(scheme="3d", size=(20, 22, 16), time_steps=7, scene="vacuum", use_fused=True,
                                   time_block=3), 4, "xy", 3, "sweep"),
]


@pytest.mark.parametrize("name,cfg,world,axes,buf,mode", CASES, ids=[c[0] for c in CASES])
def test_tagless_decomposed_equals_serial(name, cfg, world, axes, buf, mode):
    par = run_threads(cfg, world, axes, buf, mode)
    ser = serial(cfg)
    for c, b in ser.items():
        scale = max(float(v.abs().max()) for o, v in ser.items() if o[0] == c[0]) + 1e-300
        err = float((par[c] - b).abs().max())
        assert err <= 1e-12 * scale, (name, c, err, scale)


def test_direct_x_faces_bitwise():
    """x faces sent from / into the arrays (whole planes, ghost rows included,
    then overwritten by the edge / corner unpacks) == x faces packed."""
    _, cfg, world, axes, buf, _ = [c for c in CASES if c[0] == "tb4-xyz8"][0]
    a = run_threads(cfg, world, axes, buf, direct_x=True)
    b = run_threads(cfg, world, axes, buf, direct_x=False)
    for c in a:
        assert torch.equal(a[c], b[c]), c


DRUDE = dict(scheme="3d", dtype="f64", scene="drude-sphere", use_metamaterials=True, blocked_drude="on")
DRUDE_CASES = [
    # plain blocked passes + the Drude pass; the box across the x / y rank borders
    ("nopml-xy4-b3", SchemeConfig(size=(32, 30, 36), time_steps=10, sphere_center=(16.0, 15.0, 18.0),
                                  sphere_radius=6.0, time_block=3, **DRUDE), 4, "xy", 3),
    # x slabs 8 cells thick: the box misses the last rank's allocation
    ("nopml-x4-b3-miss", SchemeConfig(size=(32, 30, 36), time_steps=10, sphere_center=(12.0, 15.0, 18.0),
                                      sphere_radius=4.0, time_block=3, **DRUDE), 4, "x", 3),
    # hybrid passes with UPML: the Drude pass after the exchange join, before the shell steps
    ("upml-xy4-b3", SchemeConfig(size=(48, 48, 40), time_steps=10, sphere_center=(24.0, 24.0, 20.0),
                                 sphere_radius=5.0, use_pml=True, pml_size=(4, 4, 4), hybrid_block=3,
                                 time_block=3, **DRUDE), 4, "xy", 3),
]


@pytest.mark.parametrize("name,cfg,world,axes,buf", DRUDE_CASES, ids=[c[0] for c in DRUDE_CASES])
def test_tagless_drude_blocked_equals_serial(name, cfg, world, axes, buf):
    seen = []

    def check(s):
        seen.append((s.drude_blk is not None, s.hybrid is not None and bool(s.hybrid.get("drude")), s.tb,
                     s._drude_glob is not None))

    par = run_threads(cfg, world, axes, buf, randomize=False, check=check)
    # every rank runs the pass form (the ranks the box misses without a Drude launch)
    assert all(g for _, _, _, g in seen), seen
    if cfg.use_pml:
        assert all(h for _, h, _, _ in seen), seen
    else:
        assert all(tb == buf for _, _, tb, _ in seen), seen
    if name.endswith("-miss"):
        assert not all(d for d, _, _, _ in seen) and any(d for d, _, _, _ in seen), seen
    else:
        assert all(d for d, _, _, _ in seen), seen
    import dataclasses
    ser = serial(dataclasses.replace(cfg, blocked_drude="off", time_block=1, hybrid_block=1), randomize=False)
    for c, b in ser.items():
        scale = max(float(v.abs().max()) for o, v in ser.items() if o[0] == c[0]) + 1e-300
        err = float((par[c] - b).abs().max())
        assert err <= 1e-12 * scale, (name, c, err, scale)
