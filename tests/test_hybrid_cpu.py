"""Hybrid blocking (blocked core + stepped shell) on the torch CPU oracle:
a run with ``hybrid_block=T`` must reproduce the plain stepped run to
round-off for absorbing layers, TF/SF injection and dispersive media
(models/scheme.py ``_init_hybrid``)."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

BASE = dict(scheme="3d", size=(72, 72, 72), dtype="f64", pml_size=(4, 4, 4), tfsf_size=(6, 6, 6))

CASES = [
    ("upml-tfsf", dict(scene="vacuum", use_pml=True, use_tfsf=True, theta=40, phi=25, psi=15), 3, 9),
    ("cpml-tfsf", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, theta=60, phi=10, psi=5), 4, 10),
    ("upml-point", dict(scene="vacuum", use_pml=True), 3, 7),
    ("drude-upml", dict(scene="drude-sphere", use_pml=True, use_metamaterials=True, sphere_center=(36.0, 36.0, 36.0),
                        sphere_radius=6.0), 3, 8),
    ("sphere-cpml", dict(scene="sphere", use_pml=True, pml_type="cpml", sphere_center=(36.0, 36.0, 36.0),
                         sphere_radius=9.0), 2, 6),
    ("upml-tfsf-complex", dict(scene="vacuum", use_pml=True, use_tfsf=True, complex_values=True), 3, 7),
    # no PML / TF-SF: the core reaches the domain faces (only the dispersive box is stepped)
    ("drude-nopml", dict(scene="drude-sphere", use_metamaterials=True, sphere_center=(36.0, 36.0, 36.0),
                         sphere_radius=6.0), 3, 8),
    ("drude-nopml-face", dict(scene="drude-sphere", use_metamaterials=True, sphere_center=(9.0, 30.0, 40.0),
                              sphere_radius=6.0), 4, 9),
]


BASE2 = dict(size=(80, 76, 1), dtype="f64", pml_size=(5, 5, 1), tfsf_size=(9, 9, 1))
CASES_2D = [
    ("tmz-upml-tfsf", dict(scheme="tmz", scene="vacuum", use_pml=True, use_tfsf=True, phi=30), 4, 11),
    ("tez-upml-point", dict(scheme="tez", scene="vacuum", use_pml=True), 5, 12),
    ("tmz-cpml-tfsf", dict(scheme="tmz", scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=70), 7, 16),
    ("tez-cpml-tfsf-complex", dict(scheme="tez", scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True,
                                   complex_values=True), 3, 8),
]


def _run(cfg):
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    s.perform_steps()
    return s


@pytest.mark.parametrize("name,extra,T,steps", CASES, ids=[c[0] for c in CASES])
def test_hybrid_matches_stepped(name, extra, T, steps):
    cfg = SchemeConfig(time_steps=steps, hybrid_block=1, **BASE, **extra)
    ref = _run(cfg)
    assert ref.hybrid is None
    hy = _run(dataclasses.replace(cfg, hybrid_block=T))
    assert hy.hybrid is not None, "hybrid plan rejected"
    assert hy.hybrid["core_cells"] > 0
    for p in range(ref.planes):
        for c in ref.comps:
            a, b = hy.F[p][c], ref.F[p][c]
            # the kind's largest component: a component the wave does not
            # excite holds round-off noise only (1e-20 here)
            scale = max(float(ref.F[p][o].abs().max()) for o in ref.comps if o[0] == c[0]) + 1e-300
            err = float((a - b).abs().max())
            assert err <= 1e-12 * scale, (name, c, err, scale)


@pytest.mark.parametrize("name,extra,T,steps", CASES_2D, ids=[c[0] for c in CASES_2D])
def test_hybrid_2d_matches_stepped(name, extra, T, steps):
    """2D (TMz / TEz): blocked core (2D blocked kernel semantics) + stepped
    shell == stepping everything."""
    cfg = SchemeConfig(time_steps=steps, hybrid_block=1, **BASE2, **extra)
    ref = _run(cfg)
    assert ref.hybrid is None
    hy = _run(dataclasses.replace(cfg, hybrid_block=T))
    assert hy.hybrid is not None, "hybrid plan rejected"
    for p in range(ref.planes):
        for c in ref.comps:
            a, b = hy.F[p][c], ref.F[p][c]
            scale = float(b.abs().max()) + 1e-300
            err = float((a - b).abs().max())
            assert err <= 1e-12 * scale, (name, c, err, scale)
    assert max(float(ref.F[0][c].abs().max()) for c in ref.comps) > 0


def test_hybrid_checkpoint_resume(tmp_path):
    """Checkpoint after 7 hybrid steps (a pass boundary mid-way through the
    next pass count), resume, finish: bitwise equal to the uninterrupted
    hybrid run."""
    from fdtd3d_amd.io.checkpoint import load_checkpoint, save_checkpoint
    cfg = SchemeConfig(time_steps=15, hybrid_block=3, scene="vacuum", use_pml=True, pml_type="cpml",
                       use_tfsf=True, **BASE)

    def mk():
        s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
        s.init_scheme()
        s.init_grids()
        assert s.hybrid is not None
        return s

    full = mk()
    full.perform_steps(15)
    half = mk()
    half.perform_steps(7)
    save_checkpoint(half, str(tmp_path))
    resumed = mk()
    assert load_checkpoint(resumed, str(tmp_path)) == 7
    resumed.perform_steps(8)
    for c in full.comps:
        assert torch.equal(full.F[0][c], resumed.F[0][c]), c


RANDOM_CASES = [
    # TF/SF along +x (the reference default) and +y
    ("cpml-tfsf-x", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True), 4, 11),
    # the TF/SF faces inside the blocked core (in-kernel TfsfSets; automatic with UPML, asked for here)
    ("cpml-tfsf-x-core", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, hybrid_tfsf="core"), 5,
     12),
    ("cpml-tfsf-y-core", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=90, psi=30,
                              hybrid_tfsf="core"), 3, 10),
    ("cpml-tfsf-y", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, phi=90), 3, 10),
    ("upml-tfsf-x", dict(scene="vacuum", use_pml=True, use_tfsf=True), 5, 12),
    ("cpml-point", dict(scene="vacuum", use_pml=True, pml_type="cpml"), 5, 11),
    ("drude-upml", dict(scene="drude-sphere", use_pml=True, use_metamaterials=True, sphere_center=(36.0, 36.0, 36.0),
                        sphere_radius=6.0), 3, 8),
    ("drude-nopml-face", dict(scene="drude-sphere", use_metamaterials=True, sphere_center=(9.0, 30.0, 40.0),
                              sphere_radius=6.0), 4, 9),
    ("sphere-cpml-tfsf", dict(scene="sphere", use_pml=True, pml_type="cpml", use_tfsf=True,
                              sphere_center=(36.0, 36.0, 36.0), sphere_radius=9.0), 3, 7),
    ("cpml-tfsf-complex", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, complex_values=True),
     3, 7),
    # TF/SF faces inside the stepped shell (distance 2 < PML 4 + margin)
    ("cpml-tfsf-near", dict(scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, tfsf_size=(2, 2, 2)), 3, 8),
    # non-cubic grid, unequal layers: every face layer a different shape
    ("cpml-tfsf-box", dict(size=(64, 80, 56), pml_size=(4, 6, 5), scene="vacuum", use_pml=True, pml_type="cpml",
                           use_tfsf=True, tfsf_size=(5, 6, 5)), 4, 9),
    ("upml-point-box", dict(size=(60, 52, 76), pml_size=(5, 4, 6), scene="vacuum", use_pml=True), 3, 8),
]


@pytest.mark.parametrize("name,extra,T,steps", RANDOM_CASES, ids=[c[0] for c in RANDOM_CASES])
def test_hybrid_random_fields_match_stepped(name, extra, T, steps):
    """Hybrid passes (blocked core + stepped shell with its shrinking band,
    models/blocking.py ``_hybrid_plan``) from random fields -- every slab
    and face carries field from step 1 -- through full passes and a short
    tail equal stepping everything, on cubic and non-cubic grids."""
    kw = dict(BASE)
    kw.update(extra)
    cfg = SchemeConfig(time_steps=steps, hybrid_block=1, **kw)
    runs = []
    for hb in (T, 1):
        s = YeeScheme(dataclasses.replace(cfg, hybrid_block=hb), make_ops("torch", None, "cpu", torch.float64))
        s.init_scheme()
        s.init_grids()
        if hb > 1:
            assert s.hybrid is not None, "hybrid plan rejected"
            if name.endswith("-core"):
                assert s.hybrid["core_tfsf"], "TF/SF faces not in the blocked core"
        s.randomize_fields(seed=5)
        s.perform_steps()
        runs.append(s)
    hy, st = runs
    for p in range(st.planes):
        for c in st.comps:
            b = st.F[p][c]
            scale = max(float(st.F[p][o].abs().max()) for o in st.comps if o[0] == c[0]) + 1e-300
            err = float((hy.F[p][c] - b).abs().max())
            assert err <= 1e-12 * scale, (name, c, err, scale)
    if st.cfg.use_tfsf:
        assert torch.equal(hy.einc[0], st.einc[0]) and torch.equal(hy.hinc[0], st.hinc[0])
