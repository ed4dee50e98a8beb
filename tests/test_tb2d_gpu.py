"""2D (TMz / TEz) temporally blocked kernel (yee2d_tb.hip) vs the torch fp64
oracle, and the blocked 2D scheme vs stepping on the GPU."""
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
    if not hasattr(s, "F_alt"):
        s.F_alt = [{c: s._zeros() for c in s.comps} for _ in range(s.planes)]
    return s


def _randomize(s, seed=5):
    g = torch.Generator().manual_seed(seed)
    for c in s.comps:
        v = torch.randn(s.F[0][c].shape, generator=g, dtype=torch.float64)
        s.F[0][c].copy_(v.to(s.F[0][c].dtype))
        s.F_alt[0][c].copy_(s.F[0][c])


CASES = [
    # size (nx, ny), T, scene, output box (None = whole), source component
    ((40, 64), 1, "vacuum", None, "E"),
    ((40, 64), 2, "vacuum", None, "E"),
    ((33, 520), 4, "vacuum", None, "E"),          # 3 y runs of 248 / 240 cells
    ((37, 520), 8, "vacuum", None, "H"),
    ((70, 300), 3, "sphere", ((5, 6, 0), (60, 290, 1)), None),  # per-cell coefficients, x chunks
    ((50, 244), 5, "sphere", None, "E2"),
    ((24, 28), 7, "vacuum", ((0, 3, 0), (24, 25, 1)), "H"),
    ((30, 1024), 6, "vacuum", ((8, 0, 0), (22, 1024, 1)), "E"),
]
SRC = {"tmz": {"E": "Ez", "H": "Hx", "E2": "Ez"}, "tez": {"E": "Ex", "H": "Hz", "E2": "Ey"}}


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("mode", ["tmz", "tez"])
@pytest.mark.parametrize("size,T,scene,obox,src", CASES + [((41, 254), 6, "vacuum", None, "H")])
def test_tb2d_op_vs_torch(gpu, mode, size, T, scene, obox, src, dtype):
    nx, ny = size
    if dtype == "f32" and ny % 4:
        pytest.skip("fp32 rows are whole float4 lanes")
    dt = torch.float32 if dtype == "f32" else torch.float64
    cfg = SchemeConfig(scheme=mode, size=(nx, ny, 1), scene=scene, sphere_radius=min(size) / 3.0,
                       sphere_center=(nx / 2.0, ny / 2.0, 0.5), dtype=dtype, use_fused=True)
    a = _scheme(cfg, "hip", gpu, dt)
    a.ops.tb_xchunk = 16
    b = _scheme(dataclasses.replace(cfg, dtype="f64"), "torch", "cpu", torch.float64)
    _randomize(a)
    _randomize(b)
    upd = {c: a.local_box(c) for c in a.comps}
    ob = obox if obox is not None else ((0, 0, 0), (nx, ny, 1))
    srcs = None
    if src is not None:
        srcs = [(SRC[mode][src], (nx // 2, ny // 2 + 1, 0), 0.5 + 0.25 * l) for l in range(T)]
    a.ops.tb_step(a.F[0], a.F_alt[0], upd, ob, a.cb, T, srcs)
    b.ops.tb_step(b.F[0], b.F_alt[0], upd, ob, b.cb, T, srcs)
    torch.cuda.synchronize()
    for c in a.comps:
        x = a.F_alt[0][c].double().cpu()
        y = b.F_alt[0][c]
        err = float((x - y).abs().max())
        assert err <= (2e-5 if dtype == "f32" else 1e-12) * (float(y.abs().max()) + 1.0), (c, err)


@pytest.mark.parametrize("mode,T,dtype", [("tmz", 4, "f32"), ("tmz", 8, "f32"), ("tez", 4, "f32"),
                                          ("tez", 8, "f32"), ("tmz", 6, "f64"), ("tez", 5, "f64")])
def test_tb2d_scheme_matches_stepped(gpu, mode, T, dtype):
    """Scheme-level: time_block=T over 21 steps (a short tail pass) == 21
    split-kernel steps, with the reference's point source."""
    dt = torch.float32 if dtype == "f32" else torch.float64
    cfg = SchemeConfig(scheme=mode, size=(300, 260, 1), dtype=dtype, use_fused=True, time_steps=21)
    a = _scheme(dataclasses.replace(cfg, time_block=T), "hip", gpu, dt)
    b = _scheme(dataclasses.replace(cfg, time_block=1), "hip", gpu, dt)
    assert a.tb == T and b.tb == 1
    a.perform_steps()
    b.perform_steps()
    torch.cuda.synchronize()
    scale = max(float(b.F[0][c].abs().max()) for c in b.comps)
    for c in a.comps:
        x, y = a.F[0][c], b.F[0][c]
        err = float((x - y).abs().max())
        assert err <= (1e-5 if dtype == "f32" else 1e-12) * scale, (c, err, scale)


@pytest.mark.parametrize("kinds", ["E", "H", "EH"])
@pytest.mark.parametrize("mode", ["tmz", "tez"])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_tb2d_per_kind_coefs(gpu, mode, kinds, dtype):
    """Per-cell coefficients on one kind only (the other kind passes null
    arrays and its scalar: no constant planes) or on both, vs the torch
    oracle."""
    from fdtd3d_amd.ops.coef import Coef
    nx, ny = 36, 264
    dt = torch.float32 if dtype == "f32" else torch.float64
    cfg = SchemeConfig(scheme=mode, size=(nx, ny, 1), scene="vacuum", dtype=dtype, use_fused=True)
    a = _scheme(cfg, "hip", gpu, dt)
    b = _scheme(dataclasses.replace(cfg, dtype="f64"), "torch", "cpu", torch.float64)
    g = torch.Generator().manual_seed(5)
    for c in a.comps:
        if c[0] not in kinds:
            continue
        cell = 0.3 + 0.7 * torch.rand((nx, ny, 1), generator=g, dtype=torch.float64)
        a.cb[c] = Coef(scalar=a.cb[c].scalar, cell=cell.to(dt).to(gpu))
        b.cb[c] = Coef(scalar=b.cb[c].scalar, cell=cell.to(dt).double())
    _randomize(a)
    _randomize(b)
    upd = {c: a.local_box(c) for c in a.comps}
    ob = ((0, 0, 0), (nx, ny, 1))
    T = 4
    a.ops.tb_step(a.F[0], a.F_alt[0], upd, ob, a.cb, T, None)
    b.ops.tb_step(b.F[0], b.F_alt[0], upd, ob, b.cb, T, None)
    torch.cuda.synchronize()
    for c in a.comps:
        x = a.F_alt[0][c].double().cpu()
        y = b.F_alt[0][c]
        err = float((x - y).abs().max())
        assert err <= (2e-5 if dtype == "f32" else 1e-12) * (float(y.abs().max()) + 1.0), (c, err)
