"""Temporally blocked kernel (yee3d_tb.hip) vs the torch fp64 oracle and vs
repeated single fused steps on the GPU."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops
from fdtd3d_amd.ops.coef import Coef

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
    ((22, 40, 72), 5, "sphere", ((6, 6, 8), (16, 34, 64)), False),
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
    a.ops.tb_sparse = mrows != 1  # single-row runs keep the full per-cell planes
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


SPARSE_BOXES = [((6, 10, 30), (20, 37, 101)), ((0, 0, 0), (11, 50, 8)), ((25, 44, 128), (30, 50, 136))]


@pytest.mark.parametrize("kinds", ["E", "H", "EH"])
@pytest.mark.parametrize("T", [1, 3, 5])
@pytest.mark.parametrize("box", SPARSE_BOXES)
def test_tb_sparse_coefs(gpu, kinds, T, box):
    """Sparse per-cell coefficients (float4 box arrays, multi-row kernel):
    per-cell E only (dielectric), H only (magnetic, scalar E), or both; one
    component of each per-cell kind stays scalar; boxes inside the grid, on
    its low corner and on its high corner."""
    size = (30, 50, 136)
    cfg = SchemeConfig(scheme="3d", size=size, scene="vacuum", dtype="f32", use_fused=True)
    a = _scheme(cfg, "hip", gpu, torch.float32)
    b = _scheme(dataclasses.replace(cfg, dtype="f64"), "torch", "cpu", torch.float64)
    g = torch.Generator().manual_seed(11)
    sl = tuple(slice(box[0][d], box[1][d]) for d in range(3))
    for c in ("Ex", "Ez", "Hy", "Hz"):
        if c[0] not in kinds:
            continue
        cell = torch.ones(size, dtype=torch.float64)
        cell[sl] = 0.3 + 0.7 * torch.rand(cell[sl].shape, generator=g, dtype=torch.float64)
        cell32 = cell.float()
        a.cb[c] = Coef(scalar=a.cb[c].scalar, cell=cell32.to(gpu))
        b.cb[c] = Coef(scalar=b.cb[c].scalar, cell=cell32.double())
    _randomize(a)
    _randomize(b)
    upd = {c: a.local_box(c) for c in a.comps}
    ob = ((0, 0, 0), size)
    srcs = [("Ez", (15, 25, 68), 0.5 + 0.25 * l) for l in range(T)]
    a.ops.tb_step(a.F[0], a.F_alt[0], upd, ob, a.cb, T, srcs)
    b.ops.tb_step(b.F[0], b.F_alt[0], upd, ob, b.cb, T, srcs)
    torch.cuda.synchronize()
    ce = a.cb["Ex"]._sparse4 if "E" in kinds else None
    if ce is not None:
        assert tuple(ce[1][0]) == box[0] and tuple(ce[1][1]) == box[1], ce[1]
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
    ((30, 70, 75), 5, "vacuum", None, True),      # 3 x 4 half-wave tiles at T = 5
    ((26, 41, 33), 5, "sphere", None, False),
]


@pytest.mark.parametrize("half", [1, 0])
@pytest.mark.parametrize("size,T,scene,obox,src", F64_CASES)
def test_tb_f64_vs_torch(gpu, size, T, scene, obox, src, half):
    """fp64 blocked kernel (yee3d_tb64.hip, both tile shapes) vs the fp64
    torch oracle."""
    cfg = SchemeConfig(scheme="3d", size=size, scene=scene, sphere_radius=min(size) / 3.0,
                       sphere_center=tuple(v / 2.0 for v in size), dtype="f64", use_fused=True)
    a = _scheme(cfg, "hip", gpu, torch.float64)
    a.ops.tb_xchunk = 16
    a.ops.tb64_half = half
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


@pytest.mark.parametrize("T", [2, 3, 4, 5])
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


@pytest.mark.parametrize("size,T,scene,obox,src", [c for c in CASES_MR if c[2] == "vacuum"])
@pytest.mark.parametrize("variant,shape", [(0, 1), (4, 1), (0, 2)])
def test_tb_mr_shape8(gpu, size, T, scene, obox, src, variant, shape):
    """8-wave tiles of the plain multi-row kernel (two workgroups per CU):
    x 4 rows (shape 1) and x 2 rows (shape 2, the 16-row tiles of thin y
    boxes) vs the fp64 torch oracle."""
    if shape == 2 and T > 5:
        pytest.skip("16-row tiles: T <= 5")
    cfg = SchemeConfig(scheme="3d", size=size, scene=scene, dtype="f32", use_fused=True)
    a = _scheme(cfg, "hip", gpu, torch.float32)
    a.ops.tb_mrows = 2
    a.ops.tb_mr_shape = shape
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
        srcs = [("Ez", tuple(v // 2 for v in size), 0.5 + 0.25 * l) for l in range(T)]
    a.ops.tb_step(a.F[0], a.F_alt[0], upd, ob, a.cb, T, srcs)
    b.ops.tb_step(b.F[0], b.F_alt[0], upd, ob, b.cb, T, srcs)
    torch.cuda.synchronize()
    for c in a.comps:
        x = a.F_alt[0][c].double().cpu()
        y = b.F_alt[0][c]
        err = float((x - y).abs().max())
        assert err <= 2e-5 * (float(y.abs().max()) + 1.0), (c, err)


def test_tb_bench_scale(gpu):
    """The bench configuration itself: 1024^3 fp32 with the automatic x chunks
    (171-plane chunks at T=5), 10 steps as two blocked passes == 10 fused
    single steps, from random fields."""
    cfg = SchemeConfig(scheme="3d", size=(1024, 1024, 1024), scene="vacuum", dtype="f32", use_fused=True,
                       time_steps=10)
    runs = []
    for T in (5, 1):
        s = _scheme(dataclasses.replace(cfg, time_block=T), "hip", gpu, torch.float32)
        assert s.tb == T and s.ops.tb_xchunk == 0
        s.randomize_fields(seed=2)
        s.perform_steps()
        torch.cuda.synchronize()
        runs.append(s)
    a, b = runs
    for c in a.comps:
        err = float((a.F[0][c] - b.F[0][c]).abs().max())
        scale = max(float(b.F[0][o].abs().max()) for o in b.comps if o[0] == c[0])
        assert err <= 1e-6 * scale, (c, err, scale)
    del runs, a, b
    torch.cuda.empty_cache()


def test_tb_periodic_between_passes(gpu):
    """Periodic work no longer forces single steps: a T=5 blocked run with
    work every 7 steps (passes cut at 7, 14, ...) sees the same fields at each
    firing as the fused single-step run, and still takes blocked passes."""
    cfg = SchemeConfig(scheme="3d", size=(40, 36, 96), scene="vacuum", dtype="f32", use_fused=True, time_steps=23)
    rec = {}
    for T in (5, 1):
        s = _scheme(dataclasses.replace(cfg, time_block=T), "hip", gpu, torch.float32)
        s.randomize_fields(seed=4)
        log = []
        s.add_periodic(7, 0, lambda sc, t, log=log: log.append((t, sc.F[0]["Ez"].double().sum().item(),
                                                              sc.F[0]["Hy"].double().abs().sum().item())))
        launches0 = s.ops.launches
        s.perform_steps()
        torch.cuda.synchronize()
        rec[T] = (log, s.ops.launches - launches0)
    (la, na), (lb, nb) = rec[5], rec[1]
    assert [x[0] for x in la] == [7, 14, 21] == [x[0] for x in lb]
    for x, y in zip(la, lb):
        assert abs(x[1] - y[1]) <= 1e-4 * (abs(y[1]) + 1) and abs(x[2] - y[2]) <= 1e-5 * y[2], (x, y)
    assert na < nb  # blocked passes (7 = 5 + 2 per period), not 23 single steps
