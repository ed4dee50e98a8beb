"""TF/SF corrections folded into the blocked kernels (models/tfsf.py
TfsfSets, yee3d_tb.hip k_tfsf_pass / tf_fix, fp64: yee3d_tb64.hip tf_fix):
blocked runs vs the stepped table path on the GPU and vs the fp64 torch
oracle."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

pytestmark = pytest.mark.gpu

BASE = dict(scheme="3d", size=(40, 44, 72), dtype="f32", tfsf_size=(6, 7, 9), use_tfsf=True, use_fused=True)

CASES = [
    # name, extra, T, steps
    ("x-vacuum", dict(scene="vacuum"), 4, 13),
    ("x-vacuum-T5", dict(scene="vacuum"), 5, 11),
    ("x-vacuum-T1", dict(scene="vacuum"), 1, 7),
    ("y-vacuum", dict(scene="vacuum", phi=90.0, psi=30.0), 3, 10),
    ("x-sphere", dict(scene="sphere", sphere_center=(20.0, 22.0, 36.0), sphere_radius=9.0, sphere_eps=3.0), 4, 12),
    ("x-complex", dict(scene="vacuum", complex_values=True), 2, 9),
]


def _run(cfg, backend, device, dtype):
    s = YeeScheme(cfg, make_ops(backend, None, device, dtype))
    s.init_scheme()
    s.init_grids()
    s.perform_steps()
    if device != "cpu":
        torch.cuda.synchronize()
    return s


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("name,extra,T,steps", CASES, ids=[c[0] for c in CASES])
def test_tfsf_blocked(gpu, name, extra, T, steps, dtype):
    if dtype == "f64" and T > 5:
        pytest.skip("fp64 blocked kernel: 1..5 steps")
    cfg = SchemeConfig(time_steps=steps, **dict(BASE, dtype=dtype), **extra)
    dt = torch.float32 if dtype == "f32" else torch.float64
    tol = 2e-5 if dtype == "f32" else 1e-11
    bl = _run(dataclasses.replace(cfg, time_block=T), "hip", gpu, dt)
    assert bl.tfsf_sets is not None and bl.tfsf_blocked
    if T > 1:
        assert bl.tb == T
    st = _run(dataclasses.replace(cfg, time_block=1, use_fused=False), "hip", gpu, dt)
    ref = _run(dataclasses.replace(cfg, time_block=1, use_fused=False, dtype="f64"), "torch", "cpu", torch.float64)
    for p in range(bl.planes):
        for c in ref.comps:
            r = ref.F[p][c]
            scale = max(float(ref.F[p][o].abs().max()) for o in ref.comps if o[0] == c[0]) + 1e-30
            for s in (bl, st):
                err = float((s.F[p][c].double().cpu() - r).abs().max())
                assert err <= tol * scale, (name, dtype, p, c, err, scale)
    # the incident line advanced the same number of steps in both paths
    for p in range(bl.planes):
        assert float((bl.einc[p] - st.einc[p]).abs().max()) <= tol * (float(st.einc[p].abs().max()) + 1e-30)


def test_tfsf_oblique_takes_hybrid_passes(gpu):
    """Oblique incidence (theta 60, phi 20): the incident index of a target is
    not a function of one axis, so there are no in-kernel TF/SF sets -- the
    run takes hybrid passes instead (blocked core, stepped shell carrying the
    TF/SF tables of any angle, reference YeeGridLayout.cpp:327-845) and
    matches the fp64 oracle through two passes and a tail."""
    cfg = SchemeConfig(scheme="3d", size=(96, 88, 96), dtype="f32", tfsf_size=(8, 8, 8), use_tfsf=True,
                       use_fused=True, scene="vacuum", theta=60.0, phi=20.0, psi=30.0, time_steps=13)
    s = _run(cfg, "hip", gpu, torch.float32)
    assert s.tfsf_sets is None and not s.tfsf_blocked
    assert s.hybrid is not None and s.hybrid["T"] > 1 and s.hybrid["core_cells"] > 0.25 * s.cells()
    ref = _run(dataclasses.replace(cfg, use_fused=False, dtype="f64"), "torch", "cpu", torch.float64)
    for c in ref.comps:
        scale = max(float(ref.F[0][o].abs().max()) for o in ref.comps if o[0] == c[0]) + 1e-30
        err = float((s.F[0][c].double().cpu() - ref.F[0][c]).abs().max())
        assert err <= 2e-5 * scale, (c, err, scale)
