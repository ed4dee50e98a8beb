"""HIP kernels vs the torch fp64 reference ops (GPU only).

Every configuration runs the same scheme twice -- once through the HIP
kernels on the GPU, once through the torch reference backend on the CPU in
float64 -- and compares all field components."""

import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

pytestmark = pytest.mark.gpu


def run(cfg, backend, device, dtype):
    s = YeeScheme(cfg, make_ops(backend, None, device, dtype))
    s.init_scheme()
    s.init_grids()
    s.perform_steps()
    return s


def compare(cfg, gpu, tol=2e-5):
    dt = torch.float32 if cfg.dtype == "f32" else torch.float64
    a = run(cfg, "hip", gpu, dt)
    import dataclasses
    cfg64 = dataclasses.replace(cfg, dtype="f64")
    b = run(cfg64, "torch", "cpu", torch.float64)
    assert a.ops.launches > 0
    for p in range(a.planes):
        for c in a.comps:
            x = a.F[p][c].double().cpu()
            y = b.F[p][c]
            # scale by the largest field of the same kind (E or H): components
            # that stay ~0 by symmetry would otherwise compare noise to noise
            scale = max(float(b.F[p][o].abs().max()) for o in b.comps if o[0] == c[0]) + 1e-300
            err = float((x - y).abs().max())
            assert err <= tol * scale, (c, err, scale)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("nz", [70, 72])
def test_vacuum_3d(gpu, dtype, nz):
    # (nz % 4 == 0: fp32 float4 / fp64 double4 lanes; else the scalar kernels)
    compare(SchemeConfig(scheme="3d", size=(37, 45, nz), time_steps=25, scene="vacuum", dtype=dtype,
                         use_fused=False), gpu, 2e-5 if dtype == "f32" else 1e-12)


def test_dielectric_sphere_3d(gpu):
    compare(SchemeConfig(scheme="3d", size=(48, 48, 48), time_steps=20, scene="sphere", sphere_radius=10,
                         sphere_center=(24.5, 24.5, 24.5), dtype="f32"), gpu)


def test_upml_tfsf_3d(gpu):
    compare(SchemeConfig(scheme="3d", size=(40, 40, 40), time_steps=20, use_pml=True, use_tfsf=True,
                         pml_size=(5, 5, 5), tfsf_size=(10, 10, 10), dtype="f32", theta=60, phi=30, psi=45), gpu,
            5e-5)


def test_cpml_3d(gpu):
    compare(SchemeConfig(scheme="3d", size=(40, 44, 36), time_steps=30, use_pml=True, pml_type="cpml",
                         pml_size=(6, 6, 6), scene="vacuum", dtype="f32"), gpu, 5e-5)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_cpml_fused_sphere_tfsf(gpu, dtype):
    """CPML folded into the 4-cell-lane update kernels (yee3d_cpml.hip, fp32
    float4 / fp64 double4): per-cell coefficients, z slabs straddling lanes,
    kappa / alpha."""
    compare(SchemeConfig(scheme="3d", size=(36, 40, 52), time_steps=30, use_pml=True, pml_type="cpml",
                         use_tfsf=True, pml_size=(7, 6, 7), tfsf_size=(12, 12, 14), scene="sphere",
                         sphere_radius=5, sphere_center=(18.5, 20.5, 26.5), dtype=dtype, cpml_kappa_max=3.0,
                         cpml_alpha_max=0.05), gpu, 5e-5 if dtype == "f32" else 1e-10)


def test_cpml_tfsf_3d(gpu):
    compare(SchemeConfig(scheme="3d", size=(40, 40, 40), time_steps=25, use_pml=True, pml_type="cpml",
                         use_tfsf=True, pml_size=(6, 6, 6), tfsf_size=(12, 12, 12), scene="sphere",
                         sphere_radius=6, sphere_center=(20.5, 20.5, 20.5), dtype="f64"), gpu, 1e-10)


def test_chain_wide_upml_drude_f32(gpu):
    """Chain boxes wider than a wave row in z (x / y slabs, the dispersive
    box) and narrow z slabs in one run, fp32."""
    compare(SchemeConfig(scheme="3d", size=(40, 36, 132), time_steps=14, use_pml=True, use_metamaterials=True,
                         pml_size=(5, 5, 6), scene="drude-sphere", sphere_radius=9,
                         sphere_center=(20.0, 18.0, 66.0), dtype="f32"), gpu, 5e-5)
    compare(SchemeConfig(scheme="3d", size=(36, 40, 128), time_steps=14, use_pml=True, use_tfsf=True,
                         pml_size=(6, 5, 6), tfsf_size=(10, 10, 12), scene="sphere", sphere_radius=7,
                         sphere_center=(18.5, 20.5, 64.5), dtype="f32"), gpu, 5e-5)


def test_drude_3d(gpu):
    compare(SchemeConfig(scheme="3d", size=(64, 64, 36), time_steps=12, use_pml=True, use_metamaterials=True,
                         pml_size=(5, 5, 5), dtype="f64"), gpu, 1e-10)


@pytest.mark.parametrize("dtype,hybrid", [("f64", 1), ("f32", 1), ("f32", 0)])
def test_2d_drude_upml_tfsf(gpu, dtype, hybrid):
    """2D TMz Drude sphere (the reference's SchemeTMz.cpp:307-572 Ez PML + Drude
    path) with UPML and a TF/SF plane wave on the HIP chain kernels -- stepped
    (hybrid 1) and with the automatic hybrid passes (hybrid 0: 2D blocked core
    around the dispersive box) -- vs the fp64 torch oracle.  The sphere sits
    in the wave's path, so the dispersive update shapes the fields (the field
    energy differs from the run without metamaterials)."""
    cfg = SchemeConfig(scheme="tmz", size=(96, 88, 1), time_steps=120, use_pml=True, pml_size=(8, 8, 1),
                       use_tfsf=True, tfsf_size=(14, 14, 1), scene="drude-sphere", use_metamaterials=True,
                       sphere_center=(48.0, 44.0, 0.0), sphere_radius=14.0, dtype=dtype, hybrid_block=hybrid)
    compare(cfg, gpu, 1e-10 if dtype == "f64" else 5e-5)


@pytest.mark.parametrize("scheme", ["tmz", "tez"])
def test_2d(gpu, scheme):
    compare(SchemeConfig(scheme=scheme, size=(90, 70, 1), time_steps=40, scene="vacuum", dtype="f32"), gpu)


def test_2d_pml(gpu):
    compare(SchemeConfig(scheme="tmz", size=(80, 80, 1), time_steps=40, use_pml=True, pml_size=(8, 8, 1),
                         dtype="f64"), gpu, 1e-10)


def test_1d(gpu):
    compare(SchemeConfig(scheme="1d", size=(500, 1, 1), time_steps=300, scene="vacuum", source="gaussian",
                         dtype="f32"), gpu)


def test_complex_3d(gpu):
    compare(SchemeConfig(scheme="3d", size=(32, 32, 32), time_steps=10, scene="vacuum", complex_values=True,
                         dtype="f64"), gpu, 1e-12)


def test_amplitude_mode_3d(gpu):
    cfg = SchemeConfig(scheme="3d", size=(32, 32, 32), time_steps=10, amplitude_steps=20, use_amp_mode=True,
                       scene="vacuum", dtype="f64")
    a = run(cfg, "hip", gpu, torch.float64)
    b = run(cfg, "torch", "cpu", torch.float64)
    for c in a.comps:
        assert torch.allclose(a.amp[0][c].cpu(), b.amp[0][c], rtol=1e-10, atol=1e-14)


def test_amplitude_mode_3d_f32_vector(gpu):
    """fp32 amplitude mode through the float4 amplitude kernel (nz % 4 == 0,
    aux_kernels.hip k_amplitude_many_v4) against the fp32 torch oracle, and
    the same stable step."""
    cfg = SchemeConfig(scheme="3d", size=(36, 32, 40), time_steps=10, amplitude_steps=30, use_amp_mode=True,
                       scene="vacuum", dtype="f32", amplitude_check_steps=4)
    a = run(cfg, "hip", gpu, torch.float32)
    b = run(cfg, "torch", "cpu", torch.float32)
    for c in a.comps:
        # a near-silent component (Hz of the Ez line source) is compared on its kind's scale
        scale = max(float(b.amp[0][o].abs().max()) for o in b.comps if o[0] == c[0]) + 1e-30
        assert float((a.amp[0][c].cpu() - b.amp[0][c]).abs().max()) <= 1e-5 * scale, c
    assert getattr(a, "amplitude_stable_step", None) == getattr(b, "amplitude_stable_step", None)


@pytest.mark.parametrize("T", [2, 3])
def test_amplitude_blocked_passes(gpu, T, monkeypatch):
    """Amplitude mode on blocked passes (csrc/tb3d_mr.h AmpDev: the update
    of every step folded into the pass, maxima handed from level to level in
    LDS) against per-step stepping with the separate amplitude kernel: the
    same maxima, fields and per-step changed counts (fp32; counts may differ
    by the few cells whose growth sits at the threshold within round-off)."""
    import fdtd3d_amd.models.scheme as sch
    cfg = SchemeConfig(scheme="3d", size=(48, 40, 64), time_steps=10, amplitude_steps=45, use_amp_mode=True,
                       scene="vacuum", dtype="f32", amplitude_check_steps=8)
    runs = {}
    for t in (T, 1):
        monkeypatch.setattr(sch, "AMP_TB_STEPS", t)
        s = YeeScheme(cfg, make_ops("hip", None, gpu, torch.float32))
        s.init_scheme()
        s.init_grids()
        assert s._amp_blocked_steps() == t
        s.advance(cfg.time_steps)
        s.perform_amplitude_steps()
        torch.cuda.synchronize()
        runs[t] = s
    a, b = runs[T], runs[1]
    assert len(a.amplitude_counts) == len(b.amplitude_counts) == 45
    tot = sum(b.amplitude_counts)
    assert tot > 1000
    assert sum(abs(x - y) for x, y in zip(a.amplitude_counts, b.amplitude_counts)) <= 1e-3 * tot + 5, \
        (a.amplitude_counts, b.amplitude_counts)
    for c in a.comps:
        scale = max(float(b.amp[0][o].abs().max()) for o in b.comps if o[0] == c[0]) + 1e-30
        assert float((a.amp[0][c] - b.amp[0][c]).abs().max()) <= 2e-5 * scale, c
        fs = max(float(b.F[0][o].abs().max()) for o in b.comps if o[0] == c[0]) + 1e-30
        assert float((a.F[0][c] - b.F[0][c]).abs().max()) <= 2e-5 * fs, c


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_fused_vacuum_3d(gpu, dtype):
    compare(SchemeConfig(scheme="3d", size=(50, 37, 131), time_steps=21, scene="vacuum", dtype=dtype,
                         use_fused=True), gpu, 2e-5 if dtype == "f32" else 1e-12)


def test_fused_dielectric_complex_3d(gpu):
    compare(SchemeConfig(scheme="3d", size=(45, 40, 70), time_steps=15, scene="sphere", sphere_radius=9,
                         sphere_center=(20.5, 22.5, 30.5), complex_values=True, dtype="f64", use_fused=True), gpu,
            1e-12)


WINDOWS = {
    # z span 37 -> 16 lanes per z row (4 rows per wave)
    "mid": ({"Ex": ((2, 3, 5), (17, 21, 31)), "Ey": ((3, 1, 6), (19, 20, 33)), "Ez": ((1, 2, 1), (18, 22, 37))},
            {"Hx": ((2, 3, 5), (17, 21, 31)), "Hy": ((3, 1, 6), (19, 20, 33)), "Hz": ((1, 2, 1), (18, 22, 38))}),
    # z-thin slab (z span <= 32 -> 8 lanes per row, 8 rows per wave), high z end
    "thin": ({"Ex": ((2, 3, 130), (17, 21, 149)), "Ey": ((3, 1, 131), (19, 20, 150)),
              "Ez": ((1, 2, 129), (18, 22, 147))},
             {"Hx": ((2, 3, 130), (17, 21, 150)), "Hy": ((3, 1, 131), (19, 20, 149)),
              "Hz": ((1, 2, 129), (18, 22, 147))}),
    # wide rows (64 lanes) with a partial last row
    "wide": ({"Ex": ((2, 3, 5), (17, 21, 141)), "Ey": ((3, 1, 6), (19, 20, 143)), "Ez": ((1, 2, 1), (18, 22, 149))},
             {"Hx": ((2, 3, 5), (17, 21, 141)), "Hy": ((3, 1, 6), (19, 20, 143)), "Hz": ((1, 2, 1), (18, 22, 148))}),
}


@pytest.mark.parametrize("win", sorted(WINDOWS))
def test_vec4_windows_match_scalar(gpu, win):
    """float4 split kernels vs scalar split kernels on odd windows (box edges
    not multiple of 4, lanes past the box feeding neighbours, short z rows
    stacked several per wave)."""
    from fdtd3d_amd.ops.hip_ops import HipOps
    shape = (20, 24, 152)
    torch.manual_seed(0)
    base = {c: torch.randn(shape, dtype=torch.float32, device=gpu) for c in
            ("Ex", "Ey", "Ez", "Hx", "Hy", "Hz")}
    from fdtd3d_amd.layout.yee import YeeLayout
    from fdtd3d_amd.ops.coef import Coef
    lay = YeeLayout(shape)
    boxes_e, boxes_h = WINDOWS[win]
    cb = {c: Coef(0.3) for c in base}
    out = []
    for v4 in (False, True):
        ops = HipOps(lay, gpu, torch.float32, vec4=v4)
        f = {c: t.clone() for c, t in base.items()}
        ops.curl_update("E", boxes_e, f, f, cb)
        ops.curl_update("H", boxes_h, f, f, cb)
        out.append(f)
    for c in base:
        assert torch.allclose(out[0][c], out[1][c], rtol=1e-5, atol=1e-5), c


def test_fused_matches_split_bitwise(gpu):
    """fp32 fused kernel vs fp32 split kernels: same arithmetic per cell."""
    cfg = SchemeConfig(scheme="3d", size=(64, 64, 64), time_steps=10, scene="vacuum", dtype="f32")
    import dataclasses
    a = run(cfg, "hip", gpu, torch.float32)
    b = run(dataclasses.replace(cfg, use_fused=True), "hip", gpu, torch.float32)
    assert b.fused
    for c in a.comps:
        scale = float(a.F[0][c].abs().max()) + 1e-30
        assert float((a.F[0][c] - b.F[0][c]).abs().max()) <= 1e-6 * scale


def test_drude_lut_bitwise(gpu):
    """The Drude chain's material-ID + LUT coefficients (one byte per cell)
    give bit-identical fields to the five per-cell coefficient arrays, and
    the scene really compresses (a handful of tuples)."""
    cfg = SchemeConfig(scheme="3d", size=(48, 40, 64), time_steps=10, use_pml=True, use_metamaterials=True,
                       pml_size=(5, 5, 6), scene="drude-sphere", sphere_radius=10,
                       sphere_center=(24.0, 20.0, 32.0), dtype="f32")
    res = []
    for lut in (True, False):
        s = YeeScheme(cfg, make_ops("hip", None, gpu, torch.float32))
        s.ops.drude_lut = lut
        s.init_scheme()
        s.init_grids()
        s.perform_steps()
        torch.cuda.synchronize()
        if lut:
            ids, tab = s.upml["Ez"]["_drude_lut"]
            assert ids is not None and ids.dtype == torch.uint8 and 2 <= tab.shape[0] <= 8
            # lean initialisation: no per-cell coefficient arrays, no D1 for H
            assert s.upml["Ez"]["b0"].cell is None
            assert s.upml["Hx"].get("D1") is None and len(s.upml["Hx"]["D"][0]) == 2
        res.append({c: s.F[0][c].cpu() for c in s.comps})
    for c in res[0]:
        assert torch.equal(res[0][c], res[1][c]), c


@pytest.mark.parametrize("pml", [False, True])
def test_drude_row_split_gpu(gpu, pml):
    """Dispersive chain launches with the per-row material z ranges (plain
    update on the rest of the bounding box, chain_kernels.hip RowRanges) vs the
    chain on the whole box, from random fields, and vs the fp64 torch oracle."""
    # z = 128: the z PML chain boxes of fp32 runs widen to 32-cell row segments
    # (scheme._init_chain_regions z_align), which must leave the sphere clear
    cfg = SchemeConfig(scheme="3d", size=(48, 40, 128), time_steps=9, use_pml=pml, use_metamaterials=True,
                       pml_size=(5, 5, 6), scene="drude-sphere", sphere_radius=11,
                       sphere_center=(24.0, 19.0, 62.0), dtype="f32", hybrid_block=1)
    res = []
    for backend, dev, dt, rows in (("hip", gpu, torch.float32, True), ("hip", gpu, torch.float32, False),
                                   ("torch", "cpu", torch.float64, True)):
        s = YeeScheme(dataclasses.replace(cfg, dtype="f32" if dt == torch.float32 else "f64"),
                      make_ops(backend, None, dev, dt))
        s.ops.chain_rows = rows
        s.init_scheme()
        s.init_grids()
        s.randomize_fields(seed=11)
        s.perform_steps()
        if backend == "hip":
            torch.cuda.synchronize()
            used = any(L[4] is not None for plan in s._chain_plan_cache.values() for ls, _ in plan["chain"]
                       for L in ls)
            assert used == rows
        res.append({c: s.F[0][c].double().cpu() for c in s.comps})
    for c in res[0]:
        scale = max(float(res[2][o].abs().max()) for o in res[2] if o[0] == c[0])
        assert float((res[0][c] - res[1][c]).abs().max()) <= 2e-5 * scale, (c, "rows vs whole box")
        assert float((res[0][c] - res[2][c]).abs().max()) <= 2e-5 * scale, (c, "rows vs fp64 oracle")


def test_tfsf_apply_many_vs_tables(gpu):
    """The merged TF/SF launch (int32 offsets, folded weights, first-fit
    grouping: the layers of one component in successive launches) applies
    the same corrections as one launch per table."""
    cfg = SchemeConfig(scheme="3d", size=(40, 36, 44), time_steps=1, use_tfsf=True, scene="vacuum", dtype="f32",
                       tfsf_size=(6, 7, 8), theta=35, phi=20, psi=10)
    s = YeeScheme(cfg, make_ops("hip", None, gpu, torch.float32))
    s.init_scheme()
    s.init_grids()
    g = torch.Generator(device="cpu").manual_seed(5)
    inc = torch.randn(s.einc[0].numel(), generator=g).to(gpu)
    for kind, comps in (("E", s.e_comps), ("H", s.h_comps)):
        base = {c: torch.randn(s.F[0][c].shape, generator=g).to(gpu) for c in comps}
        a = {c: base[c].clone() for c in comps}
        b = {c: base[c].clone() for c in comps}
        items = []
        for c in comps:
            for tab in s.tfsf[c]:
                s.ops.tfsf_apply(a[c], tab, inc, ((0, 0, 0), tuple(a[c].shape)))
                items.append((b[c], tab))
        assert len(items) >= 3
        n0 = s.ops.launches
        s.ops.tfsf_apply_many(items, inc)
        assert s.ops.launches - n0 < len(items)
        torch.cuda.synchronize()
        for c in comps:
            d = float((a[c] - b[c]).abs().max())
            corr = float((a[c] - base[c]).abs().max())
            assert corr > 0  # corrections landed
            # fp32 round-off of (coef w0) inc0 + (coef w1) inc1 vs coef (w0 inc0 + w1 inc1)
            assert d <= 1e-5 * max(corr, float(base[c].abs().max())), (kind, c, d, corr)


@pytest.mark.parametrize("hb", [1, 3])
def test_chain_v4_vs_scalar(gpu, hb):
    """Non-dispersive UPML chain in 4-cell z groups (chain_kernels.hip
    k_chain3d_v4, per-element box / folded-plain masks) vs the one-cell-per-
    thread kernel, stepped (z slabs widened to 32-cell rows) and hybrid (thin
    plain boxes folded into the z slab launches), from random fields, and vs
    the fp64 torch oracle."""
    from fdtd3d_amd.ops.hip_ops import load_library
    lib = load_library()
    cfg = SchemeConfig(scheme="3d", size=(72, 64, 128), time_steps=7, use_pml=True, use_tfsf=True, scene="vacuum",
                       pml_size=(5, 6, 7), tfsf_size=(8, 8, 8), theta=30, phi=20, psi=10, dtype="f32",
                       hybrid_block=hb)
    res = []
    try:
        for backend, dev, dt, v4 in (("hip", gpu, torch.float32, 1), ("hip", gpu, torch.float32, 0),
                                     ("torch", "cpu", torch.float64, 1)):
            lib.fdtd_set_chain_v4(v4)
            c = dataclasses.replace(cfg, dtype="f32" if dt == torch.float32 else "f64",
                                    hybrid_block=hb if backend == "hip" else 1)
            s = YeeScheme(c, make_ops(backend, None, dev, dt))
            s.init_scheme()
            s.init_grids()
            s.randomize_fields(seed=4)
            s.perform_steps()
            if backend == "hip":
                torch.cuda.synchronize()
                assert (s.hybrid is not None) == (hb > 1)
            res.append({k: s.F[0][k].double().cpu() for k in s.comps})
    finally:
        lib.fdtd_set_chain_v4(0)  # the library default (measured slower, kept as a knob)
    for k in res[0]:
        scale = max(float(res[2][o].abs().max()) for o in res[2] if o[0] == k[0])
        assert float((res[0][k] - res[1][k]).abs().max()) <= 2e-5 * scale, (k, "v4 vs scalar")
        assert float((res[0][k] - res[2][k]).abs().max()) <= 2e-5 * scale, (k, "v4 vs fp64 oracle")
