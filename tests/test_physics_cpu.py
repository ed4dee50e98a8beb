"""Analytic physics checks (CPU, torch reference backend).

The reference has no physics validation.  These tests pin
the solver to known results: propagation speed, cavity eigenfrequencies,
energy conservation, absorbing-boundary reflection and TF/SF leakage.
"""

import math

import numpy as np
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops
from fdtd3d_amd.utils.constants import EPS0, MU0, SPEED_OF_LIGHT


def make(cfg):
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    return s


def test_1d_gaussian_pulse_speed():
    """BASELINE config 1: 1D vacuum, Gaussian pulse -- the peak travels at c
    (numerical dispersion of a well-resolved pulse is negligible)."""
    cfg = SchemeConfig(scheme="1d", size=(2000, 1, 1), time_steps=0, scene="vacuum", source="gaussian",
                       gaussian_width=20, gaussian_delay=80)
    s = make(cfg)
    src = 1000
    s.perform_steps(300)
    ez = s.F[0]["Ez"][:, 0, 0]
    right = int(torch.argmax(ez[src + 5:]).item()) + src + 5
    # after the pulse peak left the source (t = delay), it moved c*dt*(T - delay)
    expected = src + s.courant * (300 - 80)
    assert abs(right - expected) <= 2, (right, expected)


def test_cavity_resonance_tmz():
    """PEC-bounded 2D TMz cavity: the dominant mode after a broadband kick is
    TM11 with f = c/2 * sqrt((1/a)^2 + (1/b)^2) (up to Yee dispersion)."""
    n = 40
    cfg = SchemeConfig(scheme="tmz", size=(n, n, 1), time_steps=0, scene="vacuum", source="gaussian",
                       gaussian_width=4, gaussian_delay=12)
    s = make(cfg)
    # smooth off-centre blob: excites the low modes, TM11 the lowest and strongest
    rec = []
    s.point_source = None
    x = torch.arange(n, dtype=torch.float64) + 0.5
    X, Y = torch.meshgrid(x, x, indexing="ij")
    blob = torch.exp(-((X - 16) ** 2 + (Y - 18) ** 2) / 30.0)
    s.F[0]["Ez"][1:, 1:, 0] = blob[1:, 1:]
    steps = 4096
    for _ in range(steps):
        s.step()
        rec.append(float(s.F[0]["Ez"][13, 17, 0]))
    sig = np.array(rec) - np.mean(rec)
    spec = np.abs(np.fft.rfft(sig * np.hanning(steps)))
    freqs = np.fft.rfftfreq(steps, d=s.dt)
    peaks = [freqs[i] for i in range(2, len(spec) - 1)
             if spec[i] > spec[i - 1] and spec[i] > spec[i + 1] and spec[i] > 0.1 * spec.max()]
    # The reference's computation ranges (YeeGridLayout.h:131-182) make the low
    # border an electric wall (Ez index 0 never updated, at x = 0.5) and the high
    # border a magnetic wall (Hy index N-1 never updated, at x = N): a
    # quarter-wave cavity of length L = (N - 0.5) dx with modes
    # f = c / (2L) * sqrt((m + 1/2)^2 + (n + 1/2)^2).
    L = (n - 0.5) * s.dx
    expect = sorted(SPEED_OF_LIGHT / (2 * L) * math.sqrt((m + 0.5) ** 2 + (q + 0.5) ** 2)
                    for m in range(3) for q in range(3))
    for f in peaks[:3]:
        rel = min(abs(f - e) / e for e in expect)
        assert rel < 0.02, (f, expect[:4])
    assert abs(peaks[0] - expect[0]) / expect[0] < 0.02


def test_energy_conservation_pec_cavity():
    """Closed PEC cavity, source off: discrete EM energy stays constant."""
    cfg = SchemeConfig(scheme="3d", size=(20, 22, 24), time_steps=0, scene="vacuum")
    s = make(cfg)
    s.point_source = None
    g = torch.Generator().manual_seed(1)
    for c in ("Ex", "Ey", "Ez"):
        lo, hi = s.layout.global_range(c)
        sl = tuple(slice(lo[d], hi[d]) for d in range(3))
        s.F[0][c][sl] = torch.randn(s.F[0][c][sl].shape, generator=g, dtype=torch.float64)

    def staggered_energy_step():
        """Leapfrog's exactly conserved discrete energy
        eps0 |E^{n+1}|^2 + mu0 H^{n+1/2} . H^{n+3/2}, measured across one step."""
        h_old = {c: s.F[0][c].clone() for c in ("Hx", "Hy", "Hz")}
        s.step()
        e = sum(float((s.F[0][c] ** 2).sum()) for c in ("Ex", "Ey", "Ez")) * EPS0
        h = sum(float((h_old[c] * s.F[0][c]).sum()) for c in ("Hx", "Hy", "Hz")) * MU0
        return 0.5 * (e + h)

    e0 = staggered_energy_step()
    vals = [staggered_energy_step() for _ in range(200)]
    assert max(abs(v - e0) / e0 for v in vals) < 1e-10


def _reflection(pml_type):
    def run(size, use_pml):
        cfg = SchemeConfig(scheme="tmz", size=size, time_steps=0, scene="vacuum", use_pml=use_pml,
                           pml_type=pml_type, pml_size=(10, 10, 1), source="gaussian", gaussian_width=6,
                           gaussian_delay=25)
        return make(cfg)
    small = run((80, 80, 1), True)
    big = run((400, 400, 1), False)
    small.point_source = ("Ez", (40, 40, 0), (40, 40, 0))
    big.point_source = ("Ez", (200, 200, 0), (200, 200, 0))
    err, peak = 0.0, 0.0
    for t in range(260):
        small.step()
        big.step()
        if t % 4 == 0:
            a = small.F[0]["Ez"][10:70, 10:70, 0]
            b = big.F[0]["Ez"][170:230, 170:230, 0]
            peak = max(peak, float(b.abs().max()))
            err = max(err, float((a - b).abs().max()))
    return err / peak


def test_upml_reflection():
    assert _reflection("upml") < 2e-2


def test_cpml_reflection():
    assert _reflection("cpml") < 2e-2


def test_tfsf_leakage_3d():
    """Plane wave through an empty TF/SF box: the scattered-field region stays
    (almost) empty while the total-field region carries the full wave."""
    cfg = SchemeConfig(scheme="3d", size=(40, 40, 40), time_steps=120, scene="vacuum", use_pml=True,
                       pml_type="cpml", pml_size=(6, 6, 6), use_tfsf=True, tfsf_size=(11, 11, 11),
                       theta=70, phi=25, psi=40)
    s = make(cfg)
    s.perform_steps()
    ez = s.F[0]["Ez"]
    inside = float(ez[14:26, 14:26, 14:26].abs().max())
    outside = max(float(ez[7:9, 7:33, 7:33].abs().max()), float(ez[31:33, 7:33, 7:33].abs().max()))
    assert inside > 0.3
    assert outside < 0.05 * inside, (outside, inside)


def test_amplitude_check_period(monkeypatch):
    """Amplitude mode with the changed counts read back once per 8 steps
    finds the same first stable step as a check after every step and, from a
    near-convergence snapshot, stops exactly there with the same fields
    (reference intent of Scheme3D.cpp:2945-3333); without a snapshot the run
    ends with the stable step's check period."""
    import torch
    from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
    from fdtd3d_amd.ops import make_ops

    def run(k):
        cfg = SchemeConfig(scheme="3d", size=(16, 16, 16), time_steps=60, amplitude_steps=300, use_amp_mode=True,
                           scene="vacuum", dtype="f64", use_pml=True, pml_size=(4, 4, 4), amplitude_check_steps=k)
        s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
        s.init_scheme()
        s.init_grids()
        s.advance(cfg.time_steps)
        taken = s.perform_amplitude_steps()
        return s, (taken, getattr(s, "amplitude_stable_step", None), s.amplitude_converged)

    s1, r1 = run(1)
    s8, r8 = run(8)
    assert r1[2] and r8[2], (r1, r8)
    assert r1[1] == r8[1] == r1[0] == r8[0], (r1, r8)
    assert s1.t == s8.t and s1.amplitude_counts == s8.amplitude_counts
    for c in s1.comps:
        assert torch.equal(s1.F[0][c], s8.F[0][c]), c
        assert torch.equal(s1.amp[0][c], s8.amp[0][c]), c
    # no snapshot: the run ends with the period of the stable step
    monkeypatch.setattr(YeeScheme, "AMP_SNAPSHOT_SHARE", 0.0)
    s0, r0 = run(8)
    assert r0[1] == r1[1] and r0[0] in (r1[1], -(-r1[1] // 8) * 8), (r0, r1)


def test_capacity_plan_drude_upml():
    """The capacity plan of a Drude sphere + UPML run (scheme.capacity_plan):
    two field sets on the HIP path, three D levels + D1 for the three
    dispersive E components only, two D levels for H, all region-local
    (models/regions.py: the PML slabs and the dispersive box) -- and the
    resident arrays of the torch run stay within the plan's UPML / D1 terms
    and well below full-grid levels."""
    from fdtd3d_amd.models.regions import RegionLevel
    import torch
    from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
    from fdtd3d_amd.ops import make_ops
    cfg = SchemeConfig(scheme="3d", size=(64, 60, 56), dtype="f32", use_pml=True, use_metamaterials=True,
                       pml_size=(5, 5, 5), scene="drude-sphere", sphere_radius=7, sphere_center=(32.0, 30.0, 28.0),
                       time_steps=2)
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float32))
    s.init_scheme()
    s.init_grids()
    cells = 64 * 60 * 56
    plan = s.mem_plan
    assert plan["fields"] == 24 * cells
    assert plan["upml_D"] < 4 * cells * (3 * 3 + 2 * 3)
    assert plan["drude_D1"] < 3 * 4 * cells * 3
    assert all(isinstance(t, RegionLevel) for c in s.comps for t in s.upml[c]["D"][0])
    d = sum(t.cells() * 4 for c in s.comps for t in s.upml[c]["D"][0])
    d1 = sum(t.cells() * 4 for c in s.comps if s.upml[c].get("D1") is not None for t in s.upml[c]["D1"][0])
    assert d <= plan["upml_D"] and d1 <= plan["drude_D1"], (d, plan["upml_D"], d1, plan["drude_D1"])
    assert d >= 0.6 * plan["upml_D"] and d1 >= 0.3 * plan["drude_D1"], (d, plan["upml_D"], d1, plan["drude_D1"])
    assert all(s.upml[c].get("D1") is None for c in s.h_comps)
    # the material grids are released once the coefficients exist
    assert not s.sampler._cache and all(v is None for v in s.mat.values())
    s.perform_steps()


def test_amplitude_blocked_passes_match_stepped(monkeypatch):
    """Amplitude mode on blocked passes (the amplitude update of every step
    folded into the pass, csrc/tb3d_mr.h AmpDev; torch oracle of
    ``tb_amp_step``) equals per-step stepping with the separate update: same
    first stable step, same counts, same maxima and fields (fp64, bitwise
    arithmetic of the same single steps)."""
    import fdtd3d_amd.models.scheme as sch
    res = {}
    for T in (1, 2, 3):
        monkeypatch.setattr(sch, "AMP_TB_STEPS", T)
        cfg = SchemeConfig(scheme="3d", size=(20, 16, 24), time_steps=6, amplitude_steps=400, use_amp_mode=True,
                           scene="vacuum", dtype="f64", amplitude_check_steps=8)
        s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
        s.init_scheme()
        s.init_grids()
        assert s._amp_blocked_steps() == T
        s.advance(cfg.time_steps)
        taken = s.perform_amplitude_steps()
        res[T] = (taken, s.amplitude_converged, getattr(s, "amplitude_stable_step", None),
                  {c: s.amp[0][c].clone() for c in s.comps}, {c: s.F[0][c].clone() for c in s.comps})
    for T in (2, 3):
        assert res[T][:3] == res[1][:3], (T, res[T][:3], res[1][:3])
        for c in res[1][3]:
            assert torch.allclose(res[T][3][c], res[1][3][c], rtol=1e-12, atol=0), c
            assert torch.allclose(res[T][4][c], res[1][4][c], rtol=1e-12, atol=1e-300), c
