"""Scattered-field kernel (generic_kernels.hip k_scattered, used for the
--save-scattered-field dumps) against the torch expression of io/dump.py on
the same fields: 3D (oblique incidence, fp32 / fp64) and TMz."""
import pytest
import torch

from fdtd3d_amd.io.dump import scattered_field, scattered_field_torch
from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scheme,size,dtype", [("3d", (30, 26, 36), "f32"), ("3d", (30, 26, 36), "f64"),
                                               ("tmz", (60, 52, 1), "f32")])
def test_scattered_kernel_vs_torch(gpu, scheme, size, dtype):
    dt = torch.float32 if dtype == "f32" else torch.float64
    tf = (6, 5, 7) if scheme == "3d" else (8, 7, 0)
    cfg = SchemeConfig(scheme=scheme, size=size, time_steps=25, use_tfsf=True, tfsf_size=tf, theta=50, phi=35,
                       psi=20, scene="sphere", sphere_radius=4, sphere_center=tuple(v / 2.0 for v in size),
                       dtype=dtype)
    s = YeeScheme(cfg, make_ops("hip", None, gpu, dt))
    s.init_scheme()
    s.init_grids()
    s.perform_steps()
    for c in s.comps:
        a = scattered_field(s, c)
        b = scattered_field_torch(s, c)
        torch.cuda.synchronize()
        scale = float(b.abs().max()) + 1e-30
        assert float((a - b).abs().max()) <= (1e-6 if dtype == "f32" else 1e-14) * scale, c
        # inside the TF box something was subtracted
        assert not torch.equal(a, s.F[0][c]) or float(s.F[0][c].abs().max()) == 0.0, c
