"""The Drude box inside the blocked passes on the GPU (csrc/tb3d_mr.h DrDev,
fdtd_tb3d_drude_f32; fp64: csrc/yee3d_tb64.hip DrDev64, fdtd_tb3d_drude_f64):
blocked vs the stepped HIP chain vs the fp64 torch oracle, without and with
UPML, a sphere on the domain face, TF/SF, tails."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

pytestmark = pytest.mark.gpu

BASE = dict(scheme="3d", size=(80, 72, 96), dtype="f32", scene="drude-sphere", use_metamaterials=True,
            sphere_center=(40.0, 36.0, 48.0), sphere_radius=9.0)

CASES = [
    ("nopml-T5", {}, 5, 23),
    ("nopml-T4-tail", {}, 4, 19),
    ("upml-T5", dict(use_pml=True, pml_size=(6, 6, 6)), 5, 22),
    ("upml-T3", dict(use_pml=True, pml_size=(6, 6, 6)), 3, 17),
    # the box on the x = 0 face (grown by T it is clipped to the grid), off-centre in y / z
    ("face", dict(sphere_center=(8.5, 29.0, 61.0), sphere_radius=6.0), 5, 21),
    # the reference's scattering scene: Drude sphere + UPML + TF/SF plane wave; the sphere near the face the
    # wave enters by, its Drude launch's cone clear of the TF/SF faces.  Incidence along x: the faces in the
    # blocked core (in-kernel TF/SF); oblique: in the stepped shell
    ("upml-tfsf", dict(use_pml=True, pml_size=(5, 5, 5), use_tfsf=True, tfsf_size=(9, 9, 9), size=(96, 96, 100),
                       sphere_center=(30.0, 48.0, 50.0), sphere_radius=6.0), 4, 48),
    ("upml-tfsf-oblique", dict(use_pml=True, pml_size=(5, 5, 5), use_tfsf=True, tfsf_size=(9, 9, 9), theta=60.0,
                               phi=20.0, psi=30.0, size=(96, 96, 100), sphere_center=(30.0, 30.0, 30.0),
                               sphere_radius=6.0), 4, 60),
    ("tfsf-nopml", dict(use_tfsf=True, tfsf_size=(10, 10, 10), sphere_center=(28.0, 36.0, 48.0), sphere_radius=6.0),
     4, 37),
]


def _run(cfg, backend, device, dtype, steps=None):
    s = YeeScheme(cfg, make_ops(backend, None, device, dtype))
    s.init_scheme()
    s.init_grids()
    if steps is None:
        s.perform_steps()
    else:
        s.advance(steps)
    if device != "cpu":
        torch.cuda.synchronize()
    return s


# fp64 (the reference's default value type): the fp64 blocked kernel's Drude variant
F64 = ("nopml-T4-tail", "upml-T3", "face", "upml-tfsf", "upml-tfsf-oblique")


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("name,extra,T,steps", CASES, ids=[c[0] for c in CASES])
def test_drude_blocked_gpu(gpu, name, extra, T, steps, dtype):
    if dtype == "f64" and name not in F64:
        pytest.skip("fp64: a subset of the cases")
    cfg = SchemeConfig(time_steps=steps, **dict(BASE, dtype=dtype, **extra))
    dt = torch.float32 if dtype == "f32" else torch.float64
    blk = _run(dataclasses.replace(cfg, hybrid_block=T, time_block=T), "hip", gpu, dt)
    assert blk.drude_blk is not None, "blocked Drude plan rejected"
    assert blk.ops.launches > 0
    if cfg.use_tfsf:
        assert blk.hybrid is not None and blk.hybrid["drude"]
        assert blk.hybrid["core_tfsf"] == (not name.endswith("oblique")), blk.hybrid["core_tfsf"]
    st = _run(dataclasses.replace(cfg, blocked_drude="off", hybrid_block=1, time_block=1), "hip", gpu, dt)
    assert st.drude_blk is None
    ref = _run(dataclasses.replace(cfg, blocked_drude="off", hybrid_block=1, time_block=1, dtype="f64"), "torch",
               "cpu", torch.float64)
    tol = 2e-5 if dtype == "f32" else 1e-11
    for c in ref.comps:
        scale = max(float(ref.F[0][o].abs().max()) for o in ref.comps if o[0] == c[0]) + 1e-30
        e_st = float((blk.F[0][c].double().cpu() - st.F[0][c].double().cpu()).abs().max())
        e_ref = float((blk.F[0][c].double().cpu() - ref.F[0][c]).abs().max())
        assert e_st <= tol * scale, (name, dtype, c, "blocked vs stepped", e_st, scale)
        assert e_ref <= 10 * tol * scale, (name, dtype, c, "blocked vs fp64 oracle", e_ref, scale)


def test_drude_blocked_state_round_trip_gpu(gpu):
    """named_state() (checkpoint form) between passes and a stepped step in
    between leave the run on the stepped one."""
    cfg = SchemeConfig(time_steps=21, time_block=4, **BASE)
    ref = _run(dataclasses.replace(cfg, blocked_drude="off", hybrid_block=1, time_block=1), "hip", gpu, torch.float32)
    s = _run(cfg, "hip", gpu, torch.float32, steps=10)
    assert s.drude_blk is not None
    s.named_state()
    s.step()
    s.advance(10)
    torch.cuda.synchronize()
    for c in ref.comps:
        scale = max(float(ref.F[0][o].abs().max()) for o in ref.comps if o[0] == c[0]) + 1e-30
        err = float((s.F[0][c] - ref.F[0][c]).abs().max())
        assert err <= 2e-5 * scale, (c, err, scale)
