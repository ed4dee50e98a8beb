"""The torch/CPU backend's 1D runs take the host library's native loop
(csrc/host_yee1d.cpp, BASELINE config 1): it must equal the torch oracle
(the per-step fused ops) to rounding (the native loop may contract to FMA) --
vacuum with a Gaussian point source, and a dielectric scene with per-cell
coefficients."""
import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops


def _run(cfg, native, dtype):
    ops = make_ops("torch", None, "cpu", dtype)
    ops.native_1d = native
    s = YeeScheme(cfg, ops)
    s.init_scheme()
    s.init_grids()
    s.perform_steps()
    return s


@pytest.mark.parametrize("scene,dt", [("vacuum", "f64"), ("vacuum", "f32"), ("sphere", "f64")])
def test_native_1d_equals_oracle(scene, dt):
    extra = dict(sphere_center=(300.0, 0.0, 0.0), sphere_radius=40.0) if scene == "sphere" else {}
    cfg = SchemeConfig(scheme="1d", size=(1000, 1, 1), time_steps=700, dtype=dt, scene=scene, source="gaussian",
                       use_fused=True, **extra)
    dtype = torch.float64 if dt == "f64" else torch.float32
    a, b = _run(cfg, True, dtype), _run(cfg, False, dtype)
    assert a.res1d and b.res1d
    tol = 1e-12 if dt == "f64" else 2e-5
    for c in a.comps:
        scale = max(float(b.F[0][o].abs().max()) for o in b.comps if o[0] == c[0])
        err = float((a.F[0][c].double() - b.F[0][c].double()).abs().max())
        assert err <= tol * scale, (c, err, scale)
    assert float(a.F[0]["Ez"].abs().max()) > 0.1  # the pulse is on the grid
