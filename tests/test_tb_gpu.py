"""Temporally blocked kernel (yee3d_tb.hip) vs the torch fp64 oracle and vs
repeated single fused steps on the GPU."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

pytestmark = pytest.mark.gpu


def _scheme(cfg, backend, device, dtype):
    s = YeeScheme(cfg, make_ops(backend, None, device, dtype))
    s.init_scheme()
    s.init_grids()
    return s


def _randomize(s, seed=3):
    g = torch.Generator().manual_seed(seed)
    for c in s.comps:
        v = torch.randn(s.F[0][c].shape, generator=g, dtype=torch.float64)
        s.F[0][c].copy_(v.to(s.F[0][c].dtype))
        s.F_alt[0][c].copy_(s.F[0][c])


CASES = [
    # size, T, scene, output box (None = whole), source
    ((20, 30, 24), 2, "vacuum", None, True),
    ((37, 29, 520), 2, "vacuum", None, True),       # 3 z tiles, 3 y tiles
    ((70, 18, 256), 2, "sphere", None, False),      # x chunks, per-cell coefficients
    ((24, 26, 28), 3, "vacuum", ((3, 4, 4), (21, 22, 24)), True),
    ((24, 20, 264), 4, "sphere", ((4, 4, 8), (20, 16, 256)), False),
    ((30, 21, 20), 1, "vacuum", None, True),
    # thin z shell of a decomposed rank with the source inside it
    ((20, 20, 36), 2, "vacuum", ((0, 0, 2), (20, 20, 4)), "shell"),
    ((20, 20, 36), 2, "vacuum", ((0, 0, 4), (20, 20, 34)), "shell"),
]


CASES_MR = CASES + [
    ((26, 70, 140), 5, "vacuum", None, True),       # 3 y tiles of the 2-row kernel, 3 z tiles
    ((22, 40, 72), 6, "sphere", ((6, 6, 8), (16, 34, 64)), False),
    ((20, 36, 68), 6, "vacuum", ((0, 0, 0), (20, 36, 68)), True),
]


@pytest.mark.parametrize("vec,rows,xcd,mrows,variant", [(0, 0, 1, 1, 0), (0, 0, 0, 1, 0), (2, 1, 1, 1, 0),
                                                        (2, 2, 1, 1, 0), (4, 1, 1, 1, 0), (4, 2, 0, 1, 0),
                                                        (0, 0, 0, 2, 0), (0, 0, 0, 2, 1), (0, 0, 0, 2, 2),
                                                        (0, 0, 0, 2, 3), (0, 0, 0, 2, 4)])
@pytest.mark.parametrize("size,T,scene,obox,src", CASES_MR)
def test_tb_op_vs_torch(gpu, size, T, scene, obox, src, vec, rows, xcd, mrows, variant):
    if T > 4 and mrows != 2:
        pytest.skip("the single-row kernel stops at 4 steps per pass")
    cfg = SchemeConfig(scheme="3d", size=size, scene=scene, sphere_radius=min(size) / 3.0,
                       sphere_center=tuple(v / 2.0 for v in size), dtype="f32", use_fused=True)
    a = _scheme(cfg, "hip", gpu, torch.float32)
    a.ops.tb_xchunk = 16
    a.ops.tb_vec = vec
    a.ops.tb_rows = rows
    a.ops.tb_xcd = xcd
    a.ops.tb_mrows = mrows
    a.ops.tb_variant = variant
    b = _scheme(dataclasses.replace(cfg, dtype="f64"), "torch", "cpu", torch.float64)
    _randomize(a)
    _randomize(b)
    upd = {c: a.local_box(c) for c in a.comps}
    ob = obox if obox is not None else ((0, 0, 0), tuple(size))
    srcs = None
    if src == "shell":
        srcs = [("Ez", (10, 10, 2), 0.5 + 0.25 * l) for l in range(T)]
    elif src:
        li = tuple(v // 2 for v in size)
        srcs = [("Ez", li, 0.5 + 0.25 * l) for l in range(T)]
    a.ops.tb_step(a.F[0], a.F_alt[0], upd, ob, a.cb, T, srcs)
    b.ops.tb_step(b.F[0], b.F_alt[0], upd, ob, b.cb, T, srcs)
    torch.cuda.synchronize()
    for c in a.comps:
        x = a.F_alt[0][c].double().cpu()
        y = b.F_alt[0][c]
        err = float((x - y).abs().max())
        assert err <= 2e-5 * (float(y.abs().max()) + 1.0), (c, err)


@pytest.mark.parametrize("T", [2, 3, 4, 5, 6])
def test_tb_scheme_matches_fused(gpu, T):
    """Scheme-level: time_block=T over 11 steps == 11 single fused steps."""
    cfg = SchemeConfig(scheme="3d", size=(48, 40, 300), scene="vacuum", dtype="f32", use_fused=True,
                       time_steps=11)
    a = _scheme(dataclasses.replace(cfg, time_block=T), "hip", gpu, torch.float32)
    b = _scheme(cfg, "hip", gpu, torch.float32)
    assert a.tb == T
    a.perform_steps()
    b.perform_steps()
    torch.cuda.synchronize()
    for c in a.comps:
        x, y = a.F[0][c], b.F[0][c]
        err = float((x - y).abs().max())
        assert err <= 1e-6 * (float(y.abs().max()) + 1e-30), (c, err)


F64_CASES = [
    ((20, 30, 22), 2, "vacuum", None, True),
    ((37, 29, 150), 3, "vacuum", None, True),      # 3 z tiles, 3 y tiles
    ((40, 18, 61), 3, "sphere", None, False),      # per-cell coefficients, odd nz
    ((24, 26, 28), 4, "vacuum", ((4, 4, 4), (20, 22, 24)), True),
    ((20, 20, 36), 2, "vacuum", ((0, 0, 2), (20, 20, 4)), "shell"),
]


@pytest.mark.parametrize("size,T,scene,obox,src", F64_CASES)
def test_tb_f64_vs_torch(gpu, size, T, scene, obox, src):
    """fp64 blocked kernel (yee3d_tb64.hip) vs the fp64 torch oracle."""
    cfg = SchemeConfig(scheme="3d", size=size, scene=scene, sphere_radius=min(size) / 3.0,
                       sphere_center=tuple(v / 2.0 for v in size), dtype="f64", use_fused=True)
    a = _scheme(cfg, "hip", gpu, torch.float64)
    a.ops.tb_xchunk = 16
    b = _scheme(cfg, "torch", "cpu", torch.float64)
    _randomize(a)
    _randomize(b)
    upd = {c: a.local_box(c) for c in a.comps}
    ob = obox if obox is not None else ((0, 0, 0), tuple(size))
    srcs = None
    if src == "shell":
        srcs = [("Ez", (10, 10, 2), 0.5 + 0.25 * l) for l in range(T)]
    elif src:
        srcs = [("Ez", tuple(v // 2 for v in size), 0.5 + 0.25 * l) for l in range(T)]
    a.ops.tb_step(a.F[0], a.F_alt[0], upd, ob, a.cb, T, srcs)
    b.ops.tb_step(b.F[0], b.F_alt[0], upd, ob, b.cb, T, srcs)
    torch.cuda.synchronize()
    for c in a.comps:
        x = a.F_alt[0][c].cpu()
        y = b.F_alt[0][c]
        err = float((x - y).abs().max())
        assert err <= 1e-12 * (float(y.abs().max()) + 1.0), (c, err)


@pytest.mark.parametrize("T", [2, 3, 4])
def test_tb_f64_scheme_matches_fused(gpu, T):
    cfg = SchemeConfig(scheme="3d", size=(40, 36, 90), scene="vacuum", dtype="f64", use_fused=True, time_steps=11)
    a = _scheme(dataclasses.replace(cfg, time_block=T), "hip", gpu, torch.float64)
    b = _scheme(cfg, "hip", gpu, torch.float64)
    assert a.tb == T
    a.perform_steps()
    b.perform_steps()
    torch.cuda.synchronize()
    for c in a.comps:
        x, y = a.F[0][c], b.F[0][c]
        err = float((x - y).abs().max())
        assert err <= 1e-12 * (float(y.abs().max()) + 1e-300), (c, err)
