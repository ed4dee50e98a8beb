"""2D blocked stepping on the torch oracle: a time_block=T run (the generic
tb_step: T fused steps on padded copies) equals the stepped run exactly."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops


def _run(cfg):
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    s.perform_steps()
    return s


@pytest.mark.parametrize("mode", ["tmz", "tez"])
@pytest.mark.parametrize("T", [3, 8])
def test_tb2d_oracle_matches_stepped(mode, T):
    cfg = SchemeConfig(scheme=mode, size=(64, 48, 1), dtype="f64", use_fused=True, time_steps=21)
    a = _run(dataclasses.replace(cfg, time_block=T))
    b = _run(cfg)
    assert a.tb == T and b.tb == 1
    for c in a.comps:
        assert torch.equal(a.F[0][c], b.F[0][c]), c
    assert float(b.F[0][a.comps[0]].abs().max()) > 0


def test_tb2d_off_with_pml():
    cfg = SchemeConfig(scheme="tmz", size=(64, 48, 1), dtype="f64", use_fused=True, time_block=4, use_pml=True)
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    assert s.tb == 1


def test_res1d_oracle_matches_stepped():
    """The torch twin of the resident 1D kernel equals per-step stepping."""
    cfg = SchemeConfig(scheme="1d", size=(300, 1, 1), dtype="f64", source="gaussian", time_steps=60)
    a = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    a.init_scheme()
    a.init_grids()
    a.res1d = True  # the scheme enables it for HIP runs; force the oracle path
    a.perform_steps()
    b = _run(cfg)
    for c in a.comps:
        assert torch.allclose(a.F[0][c], b.F[0][c], rtol=0, atol=1e-14), c
    assert float(b.F[0]["Ez"].abs().max()) > 0
