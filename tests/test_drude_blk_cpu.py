"""The Drude box inside the blocked passes (csrc/tb3d_mr.h DrDev,
models/blocking.py _plan_drude_blk) on the torch oracle: its pass form --
E' = (b0 cbd) curl - b2 (D - Dp) + m1 E + m2 Ep with (D - Dp, Ep) as the
carried state -- against the stepped UPML / Drude chain (fp64), without and
with absorbing layers, through a tail pass, a checkpoint-style state round
trip and a whole-grid stepped step in between."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

BASE = dict(scheme="3d", size=(64, 60, 68), dtype="f64", scene="drude-sphere", use_metamaterials=True,
            sphere_center=(32.0, 30.0, 34.0), sphere_radius=6.0)


def _scheme(cfg):
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    return s


def _close(a, b, tol=1e-12):
    for c in b.comps:
        scale = max(float(b.F[0][o].abs().max()) for o in b.comps if o[0] == c[0]) + 1e-300
        err = float((a.F[0][c] - b.F[0][c]).abs().max())
        assert err <= tol * scale, (c, err, scale)


@pytest.mark.parametrize("extra,T,steps", [({}, 4, 13), ({"use_pml": True, "pml_size": (5, 5, 5)}, 4, 14),
                                           ({}, 5, 12),
                                           # the reference's scattering scene: Drude sphere + UPML + TF/SF
                                           # (the faces lie in the stepped shell here: a grid big enough for
                                           # a core of a quarter of the cells; the sphere near the corner the
                                           # wave enters by, its cone clear of the faces)
                                           ({"use_pml": True, "pml_size": (5, 5, 5), "use_tfsf": True,
                                             "tfsf_size": (9, 9, 9), "theta": 60.0, "phi": 20.0, "psi": 30.0,
                                             "size": (80, 80, 84), "sphere_center": (27.0, 27.0, 27.0)}, 4, 56),
                                           ({"use_tfsf": True, "tfsf_size": (10, 10, 10),
                                             "sphere_center": (26.0, 30.0, 34.0)}, 3, 36)],
                         ids=["nopml", "upml", "nopml-T5", "upml-tfsf", "tfsf-nopml"])
def test_drude_blocked_vs_chain(extra, T, steps):
    cfg = SchemeConfig(time_steps=steps, **dict(BASE, **extra))
    blk = _scheme(dataclasses.replace(cfg, blocked_drude="on", hybrid_block=T, time_block=T))
    assert blk.drude_blk is not None
    if cfg.use_pml or cfg.use_tfsf:
        assert blk.hybrid is not None and blk.hybrid["drude"]
    else:
        assert blk.hybrid is None and blk.tb == T
    blk.perform_steps()
    ref = _scheme(dataclasses.replace(cfg, blocked_drude="off", hybrid_block=1, time_block=1))
    assert ref.drude_blk is None
    ref.perform_steps()
    _close(blk, ref)
    # the medium matters: the same run in vacuum ends elsewhere
    vac = _scheme(dataclasses.replace(cfg, use_metamaterials=False, hybrid_block=1, time_block=1))
    vac.perform_steps()
    assert float((vac.F[0]["Ez"] - ref.F[0]["Ez"]).abs().max()) > 1e-3 * float(ref.F[0]["Ez"].abs().max())


def test_drude_blocked_state_round_trip():
    """named_state() moves the pass state into the chain levels (the
    checkpoint format); the next pass reads it back; a whole-grid stepped
    step in between runs the chain on it."""
    cfg = SchemeConfig(time_steps=17, **BASE)
    ref = _scheme(dataclasses.replace(cfg, blocked_drude="off", hybrid_block=1, time_block=1))
    ref.perform_steps()
    blk = _scheme(dataclasses.replace(cfg, blocked_drude="on", time_block=4))
    blk.advance(8)
    saved = {k: v.clone() for k, v in blk.named_state().items()}
    assert blk.drude_blk["loc"] == "chain"
    blk.advance(1)
    blk.step()  # whole-grid stepped step: the chain on the exported state
    blk.advance(7)
    _close(blk, ref)
    # resume from the saved arrays into a fresh blocked run
    res = _scheme(dataclasses.replace(cfg, blocked_drude="on", time_block=4))
    for k, v in res.named_state().items():
        v.copy_(saved[k])
    res.t = 8
    res.advance(9)
    _close(res, ref)
