"""Region-local UPML/Drude chain (plain Yee outside the PML slabs and the
dispersive box, fused chain inside) against the full reference chain on every
cell (three sweeps per component, Scheme3D.cpp:266-416), on the CPU oracle."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops


def _run(cfg, regional: bool):
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    if not regional:
        s.chain_regions = None
    else:
        assert s.chain_regions is not None
    s.perform_steps()
    return s


CASES = {
    "upml-tfsf": SchemeConfig(scheme="3d", size=(30, 28, 26), time_steps=25, use_pml=True, use_tfsf=True,
                              pml_size=(5, 4, 6), tfsf_size=(9, 9, 9), theta=60, phi=30, psi=45, dtype="f64"),
    "upml-sphere-point": SchemeConfig(scheme="3d", size=(28, 28, 28), time_steps=20, use_pml=True, pml_size=(5, 5, 5),
                                      scene="sphere", sphere_radius=6, sphere_center=(14.5, 14.5, 14.5),
                                      dtype="f64"),
    "drude-upml": SchemeConfig(scheme="3d", size=(40, 40, 32), time_steps=16, use_pml=True, use_metamaterials=True,
                               pml_size=(5, 5, 5), scene="drude-sphere", sphere_radius=7,
                               sphere_center=(20.0, 20.0, 16.0), dtype="f64"),
    "drude-reference-tfsf": SchemeConfig(scheme="3d", size=(64, 64, 36), time_steps=12, use_pml=True,
                                         use_metamaterials=True, use_tfsf=True, pml_size=(5, 5, 5),
                                         tfsf_size=(10, 10, 8), dtype="f64"),
}


@pytest.mark.parametrize("name", list(CASES))
def test_regional_chain_equals_full_chain(name):
    cfg = CASES[name]
    a = _run(cfg, True)
    b = _run(cfg, False)
    for c in a.comps:
        x, y = a.F[0][c], b.F[0][c]
        scale = max(float(b.F[0][o].abs().max()) for o in b.comps if o[0] == c[0]) + 1e-300
        err = float((x - y).abs().max())
        assert err <= 1e-9 * scale, (name, c, err, scale)
