"""Hybrid blocking on the GPU: blocked core (yee3d_tb.hip) + stepped shell
(UPML chain / CPML / TF/SF kernels) vs the plain stepped HIP run, and vs the
fp64 torch oracle."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

pytestmark = pytest.mark.gpu

BASE = dict(scheme="3d", size=(80, 72, 96), dtype="f32", pml_size=(5, 5, 5), tfsf_size=(8, 8, 8))

CASES = [
    ("upml-tfsf", dict(scene="vacuum", use_pml=True, use_tfsf=True, theta=40, phi=25, psi=15), 4, 13),
    ("cpml-tfsf", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, theta=60, phi=10, psi=5), 4, 12),
    ("upml-point", dict(scene="vacuum", use_pml=True), 3, 10),
    ("drude-upml", dict(scene="drude-sphere", use_pml=True, use_metamaterials=True, blocked_drude="off", sphere_center=(40.0, 36.0, 48.0),
                        sphere_radius=7.0), 4, 12),
    ("sphere-cpml", dict(scene="sphere", use_pml=True, pml_type="cpml", sphere_center=(40.0, 36.0, 48.0),
                         sphere_radius=10.0), 4, 9),
    ("upml-tfsf-f64", dict(scene="vacuum", use_pml=True, use_tfsf=True, theta=30, phi=40, psi=20, dtype="f64"), 4, 10),
    # fp64 CPML shell on the double4 fused CPML kernels (yee3d_cpml.hip)
    ("cpml-tfsf-f64", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, theta=60, phi=10, psi=5,
                           dtype="f64"), 4, 10),
    # (the Drude cases keep the stepped dispersive box: blocked_drude="off"; the blocked Drude pass is
    # tests/test_drude_blk_gpu.py)
    # no PML: the blocked core reaches the domain faces around the dispersive box
    ("drude-nopml", dict(scene="drude-sphere", use_metamaterials=True, blocked_drude="off", sphere_center=(40.0, 36.0, 48.0),
                         sphere_radius=7.0), 5, 12),
    ("drude-nopml-face", dict(scene="drude-sphere", use_metamaterials=True, blocked_drude="off", sphere_center=(9.0, 30.0, 60.0),
                              sphere_radius=6.0), 4, 11),
    # 2D: blocked core through yee2d_tb.hip
    ("tmz-upml-tfsf", dict(scheme="tmz", size=(120, 104, 1), pml_size=(6, 6, 1), tfsf_size=(10, 10, 1),
                           scene="vacuum", use_pml=True, use_tfsf=True, phi=30), 7, 23),
    ("tez-cpml-tfsf", dict(scheme="tez", size=(96, 128, 1), pml_size=(6, 6, 1), tfsf_size=(10, 10, 1),
                           scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=60), 5, 17),
    # TF/SF along x / y, T = 5 passes, complex fields
    ("cpml-tfsf-x", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True), 4, 13),
    # TF/SF faces in the blocked core (automatic with UPML; forced here), x and y incidence, T = 5
    ("cpml-tfsf-x-core", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, hybrid_tfsf="core"), 5,
     13),
    ("cpml-tfsf-y-core", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=90.0, psi=30.0,
                              hybrid_tfsf="core"), 4, 11),
    ("cpml-tfsf-y", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=90.0, psi=30.0), 3, 11),
    # split: the x faces in the shell, the y / z faces in the core (the TF/SF variant on its border slabs only)
    ("cpml-tfsf-x-split", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, hybrid_tfsf="split"), 5,
     13),
    ("cpml-tfsf-y-split", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=90.0, psi=30.0,
                               hybrid_tfsf="split"), 4, 11),
    ("upml-tfsf-x-split", dict(scene="vacuum", use_pml=True, use_tfsf=True, hybrid_tfsf="split"), 4, 12),
    # fp64: the TF/SF faces in the fp64 blocked core (yee3d_tb64.hip tf_fix; automatic in fp64), x and y
    # incidence, CPML and UPML shells
    ("cpml-tfsf-x-f64-core", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, dtype="f64"), 4,
     13),
    ("cpml-tfsf-y-f64-core", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=90.0, psi=30.0,
                                  dtype="f64"), 3, 11),
    ("upml-tfsf-x-f64-core", dict(scene="vacuum", use_pml=True, use_tfsf=True, dtype="f64"), 4, 12),
    ("cpml-tfsf-sphere", dict(scene="sphere", use_pml=True, pml_type="cpml", use_tfsf=True,
                              sphere_center=(40.0, 36.0, 48.0), sphere_radius=10.0), 4, 10),
    ("cpml-point-T5", dict(scene="vacuum", use_pml=True, pml_type="cpml"), 5, 12),
    ("upml-tfsf-x-T5", dict(scene="vacuum", use_pml=True, use_tfsf=True), 5, 12),
    ("cpml-tfsf-complex", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, complex_values=True),
     2, 7),
    ("tmz-upml-point-f64", dict(scheme="tmz", size=(150, 90, 1), pml_size=(8, 8, 1), scene="vacuum", use_pml=True,
                                dtype="f64"), 6, 19),
    # 2D passes long enough to replay from a HIP graph (one warm pass, graphs of two passes, a tail)
    ("tmz-cpml-tfsf-graph", dict(scheme="tmz", size=(120, 104, 1), pml_size=(6, 6, 1), tfsf_size=(10, 10, 1),
                                 scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=30), 5, 37),
    ("tez-upml-tfsf-graph", dict(scheme="tez", size=(96, 128, 1), pml_size=(6, 6, 1), tfsf_size=(10, 10, 1),
                                 scene="vacuum", use_pml=True, use_tfsf=True, phi=60), 4, 30),
    # the same passes replayed from HIP graphs (--hybrid-graph graph) instead of launch records
    ("tmz-cpml-tfsf-hipgraph", dict(scheme="tmz", size=(120, 104, 1), pml_size=(6, 6, 1), tfsf_size=(10, 10, 1),
                                    scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=30,
                                    hybrid_graph="graph"), 5, 37),
    # the shell's window launches run on several streams (--shell-streams auto = 3); the in-order single-stream
    # form stays covered
    ("cpml-tfsf-inorder", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, theta=60, phi=10, psi=5,
                               shell_streams=1), 4, 12),
    ("cpml-tfsf-3streams", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, theta=60, phi=10,
                                psi=5, shell_streams=3), 4, 12),
    ("drude-upml-3streams", dict(scene="drude-sphere", use_pml=True, use_metamaterials=True, sphere_center=(40.0, 36.0,
                                 48.0), sphere_radius=7.0, shell_streams=3), 4, 12),
    ("drude-upml-inorder", dict(scene="drude-sphere", use_pml=True, use_metamaterials=True, blocked_drude="off",
                                sphere_center=(40.0, 36.0, 48.0), sphere_radius=7.0, shell_streams=1), 4, 12),
]


def _run(cfg, backend, device, dtype):
    s = YeeScheme(cfg, make_ops(backend, None, device, dtype))
    s.init_scheme()
    s.init_grids()
    s.perform_steps()
    if device != "cpu":
        torch.cuda.synchronize()
    return s


@pytest.mark.parametrize("name,extra,T,steps", CASES, ids=[c[0] for c in CASES])
def test_hybrid_gpu(gpu, name, extra, T, steps):
    keys = ("dtype", "scheme", "size", "pml_size", "tfsf_size")
    base = dict(BASE, **{k: v for k, v in extra.items() if k in keys})
    extra = {k: v for k, v in extra.items() if k not in keys}
    cfg = SchemeConfig(time_steps=steps, **base, **extra)
    dt = torch.float32 if cfg.dtype == "f32" else torch.float64
    tol = 2e-5 if cfg.dtype == "f32" else 1e-12
    hy = _run(dataclasses.replace(cfg, hybrid_block=T), "hip", gpu, dt)
    assert hy.hybrid is not None, "hybrid plan rejected"
    if name.endswith("-graph"):
        assert getattr(hy, "_hrec", None) is not None, "no launch-record replay"
    if name.endswith("-hipgraph"):
        assert getattr(hy, "_hgraph", None) is not None, "no graph replay"
    if name.endswith("-core"):
        assert hy.hybrid["core_tfsf"], "TF/SF faces not in the blocked core"
    if name.endswith("-split"):
        assert hy.hybrid["core_tfsf"] and hy.hybrid["core_tfs"], "no split core"
        assert False in hy.hybrid["core_tfs"] and True in hy.hybrid["core_tfs"], hy.hybrid["core_tfs"]
    st = _run(dataclasses.replace(cfg, hybrid_block=1), "hip", gpu, dt)
    assert st.hybrid is None
    ref = _run(dataclasses.replace(cfg, hybrid_block=1, dtype="f64"), "torch", "cpu", torch.float64)
    for p in range(ref.planes):
        for c in ref.comps:
            r = ref.F[p][c]
            # scale by the kind's largest component (a point Ez source leaves Hz ~ 0)
            scale = max(float(ref.F[p][o].abs().max()) for o in ref.comps if o[0] == c[0]) + 1e-30
            e_hy = float((hy.F[p][c].double().cpu() - st.F[p][c].double().cpu()).abs().max())
            e_ref = float((hy.F[p][c].double().cpu() - r).abs().max())
            assert e_hy <= tol * scale, (name, p, c, "hybrid vs stepped", e_hy, scale)
            assert e_ref <= 10 * tol * scale, (name, p, c, "hybrid vs fp64 oracle", e_ref, scale)
    if hy.use_cpml:
        # the CPML auxiliaries advanced identically
        # (psi is a convolution of field differences of the source kind: its
        # absolute error is bounded like that kind's fields')
        for c in hy.comps:
            src_scale = max(float(ref.F[0][o].abs().max()) for o in ref.comps if o[0] != c[0]) + 1e-30
            for a, b in zip(hy.cpml.slabs[c], st.cpml.slabs[c]):
                x, y = a.psi[0].double().cpu(), b.psi[0].double().cpu()
                err = float((x - y).abs().max())
                assert err <= 1e-4 * float(y.abs().max()) + tol * src_scale, (name, c, "psi", err, src_scale)


@pytest.mark.parametrize("T,tfsf,point,size,phi", [(4, True, False, (96, 88, 96), 0.0),
                                                   (5, True, True, (112, 104, 112), 0.0),
                                                   (4, False, True, (72, 80, 64), 0.0),
                                                   (3, True, False, (80, 80, 128), 90.0),
                                                   (5, False, True, (112, 96, 100), 0.0)])
def test_hybrid_random_fields(gpu, T, tfsf, point, size, phi):
    """Hybrid passes from random fields (every face and slab carries field
    from step 1, so the band's CPML psi terms are live) against the stepped
    run; 2T + 1 steps = two passes and a one-step tail."""
    cfg = SchemeConfig(time_steps=2 * T + 1, scheme="3d", size=size, dtype="f32", pml_size=(5, 6, 7),
                       tfsf_size=(9, 10, 11), scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=tfsf, phi=phi)
    if point:
        cfg = dataclasses.replace(cfg, use_point_source=True)
    runs = {}
    for hb in (T, 1):
        s = YeeScheme(dataclasses.replace(cfg, hybrid_block=hb), make_ops("hip", None, gpu, torch.float32))
        s.init_scheme()
        s.init_grids()
        s.randomize_fields(seed=11)
        s.perform_steps()
        torch.cuda.synchronize()
        runs[hb] = s
    hy, st = runs[T], runs[1]
    assert hy.hybrid is not None, "hybrid plan rejected"
    assert st.hybrid is None
    for c in hy.comps:
        x, y = hy.F[0][c].double().cpu(), st.F[0][c].double().cpu()
        scale = max(float(st.F[0][o].abs().max()) for o in st.comps if o[0] == c[0])
        assert float((x - y).abs().max()) <= 2e-5 * scale, (c, float((x - y).abs().max()), scale)
        src_scale = max(float(st.F[0][o].abs().max()) for o in st.comps if o[0] != c[0])
        for a, b in zip(hy.cpml.slabs[c], st.cpml.slabs[c]):
            err = float((a.psi[0].double() - b.psi[0].double()).abs().max())
            assert err <= 2e-5 * src_scale, (c, "psi", err, src_scale)


SCALE_CASES = [
    ("cpml-tfsf-256", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True)),
    ("upml-tfsf-256", dict(scene="vacuum", use_pml=True, use_tfsf=True)),
    ("drude-256", dict(scene="drude-sphere", use_pml=True, use_metamaterials=True, sphere_center=(128.0, 128.0, 128.0),
                       sphere_radius=64)),
    ("drude-256-nopml", dict(scene="drude-sphere", use_metamaterials=True, sphere_center=(128.0, 128.0, 128.0),
                             sphere_radius=64)),
]


@pytest.mark.parametrize("name,extra", SCALE_CASES, ids=[c[0] for c in SCALE_CASES])
def test_hybrid_at_scale(gpu, name, extra):
    """Bench-like configs at 256^3 (reference PML / TF-SF sizes, automatic
    hybrid plan and T, random-init fields): two hybrid passes + one step
    equal the stepped run of the same kernels.  (The fp64 torch oracle is
    checked on the small cases above; at this size it would take minutes on
    the CPU.)"""
    cfg = SchemeConfig(scheme="3d", size=(256, 256, 256), time_steps=9, dtype="f32", **extra)
    runs = []
    for hb in (0, 1):
        s = YeeScheme(dataclasses.replace(cfg, hybrid_block=hb), make_ops("hip", None, gpu, torch.float32))
        s.init_scheme()
        s.init_grids()
        s.randomize_fields(seed=7)
        if hb == 0:
            assert s.hybrid is not None, "automatic hybrid plan rejected"
        else:
            assert s.hybrid is None
        s.perform_steps()
        torch.cuda.synchronize()
        runs.append(s)
    hy, st = runs
    for c in hy.comps:
        scale = max(float(st.F[0][o].abs().max()) for o in st.comps if o[0] == c[0]) + 1e-30
        err = float((hy.F[0][c] - st.F[0][c]).abs().max())
        assert err <= 2e-5 * scale, (name, c, err, scale)
        del scale
    del runs, hy, st
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mode,attr", [("auto", "_hrec"), ("graph", "_hgraph")])
def test_hybrid_graph_reuse_across_advance(gpu, mode, attr):
    """2D UPML hybrid passes replayed from a launch record (auto) / a HIP
    graph over TWO ``advance`` calls: T = 4, 25 steps end on a
    tail of one 4-step and one 1-step pass, so the field buffers are back in
    the recorded parity while the UPML D level lists are rotated by an odd
    number of steps.  The second call (30 steps) must re-record rather than
    replay launches that read the stale level -- the result equals the
    stepped run."""
    cfg = SchemeConfig(scheme="tez", size=(96, 128, 1), pml_size=(6, 6, 1), tfsf_size=(10, 10, 1), dtype="f32",
                       scene="vacuum", use_pml=True, use_tfsf=True, phi=60, time_steps=55, hybrid_block=4,
                       hybrid_graph=mode)
    hy = YeeScheme(cfg, make_ops("hip", None, gpu, torch.float32))
    hy.init_scheme()
    hy.init_grids()
    assert hy.hybrid is not None and hy.hybrid["T"] == 4
    hy.advance(25)
    k1 = getattr(hy, attr)["key"] if getattr(hy, attr, None) else None
    hy.advance(30)
    torch.cuda.synchronize()
    assert k1 is not None and getattr(hy, attr)["key"] != k1, "not re-recorded after the level lists rotated"
    st = _run(dataclasses.replace(cfg, hybrid_block=1), "hip", gpu, torch.float32)
    for c in st.comps:
        b = st.F[0][c].double().cpu()
        scale = max(float(st.F[0][o].abs().max()) for o in st.comps if o[0] == c[0]) + 1e-30
        err = float((hy.F[0][c].double().cpu() - b).abs().max())
        assert err <= 2e-5 * scale, (c, err, scale)
