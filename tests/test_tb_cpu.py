"""Temporal blocking semantics on the CPU oracle: ``tb_step`` (T fused steps
per pass, update boxes vs output box) equals T single fused steps."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops


def _run(cfg, steps):
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    g = torch.Generator().manual_seed(5)
    for c in s.comps:
        s.F[0][c].copy_(torch.randn(s.F[0][c].shape, generator=g, dtype=torch.float64))
        s.F_alt[0][c].copy_(s.F[0][c])  # cells outside the boxes are never written
    s.advance(steps)
    return s


@pytest.mark.parametrize("T", [2, 3])
@pytest.mark.parametrize("scene", ["vacuum", "sphere"])
def test_tb_equals_fused_steps(T, scene):
    cfg = SchemeConfig(scheme="3d", size=(14, 12, 16), scene=scene, sphere_radius=4,
                       sphere_center=(7.0, 6.0, 8.0), dtype="f64", use_fused=True)
    a = _run(dataclasses.replace(cfg, time_block=T), 2 * T + 1)
    b = _run(cfg, 2 * T + 1)
    assert a.tb == T and b.tb == 1
    for c in a.comps:
        torch.testing.assert_close(a.F[0][c], b.F[0][c], rtol=1e-12, atol=1e-12)


def test_tb_output_box_only():
    """Cells outside the output box are left untouched in ``fout``."""
    cfg = SchemeConfig(scheme="3d", size=(10, 10, 12), scene="vacuum", dtype="f64", use_fused=True)
    s = _run(cfg, 0)
    fout = {c: torch.full_like(s.F[0][c], 7.0) for c in s.comps}
    ob = ((2, 3, 4), (8, 7, 9))
    upd = {c: s.local_box(c) for c in s.comps}
    s.ops.tb_step(s.F[0], fout, upd, ob, s.cb, 2, None)
    for c in s.comps:
        m = torch.ones_like(fout[c], dtype=torch.bool)
        m[2:8, 3:7, 4:9] = False
        assert bool((fout[c][m] == 7.0).all())
