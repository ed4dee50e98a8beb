"""CPU unit tests: settings/CLI, coordinates, layout tables, topology,
materials, I/O formats, checkpoint/resume, NTFF, driver."""

import io
import math
import os

import numpy as np
import pytest
import torch

from fdtd3d_amd.utils import settings as S
from fdtd3d_amd.utils.coordinates import GridCoordinate, GridCoordinate3D, GridCoordinateFP3D, convert_coord


# ------------------------------------------------------------------ settings
REFERENCE_FLAGS = [
    "--2d", "--3d", "--log-level", "--sizex", "--sizey", "--sizez", "--same-size", "--pml-sizex", "--pml-sizey",
    "--pml-sizez", "--same-size-pml", "--tfsf-sizex", "--tfsf-sizey", "--tfsf-sizez", "--same-size-tfsf",
    "--ntff-sizex", "--ntff-sizey", "--ntff-sizez", "--same-size-ntff", "--time-steps", "--amplitude-time-steps",
    "--angle-teta", "--angle-phi", "--angle-psi", "--buffer-size", "--num-cuda-gpus", "--parallel-grid",
    "--optimal-topology", "--available-topologies", "--topology-sizex", "--topology-sizey", "--topology-sizez",
    "--same-size-topology", "--use-double-material-precision", "--use-tfsf", "--use-ntff", "--use-pml",
    "--use-metamaterials", "--use-amp-mode", "--dx", "--wavelength", "--save-res", "--save-materials",
    "--save-interm-res", "--interm-save-step", "--save-scattered-field-res", "--save-scattered--field-interm",
    "--cmd-from-file", "--save-cmd-to-file",
]


def test_every_reference_flag_is_accepted():
    for f in REFERENCE_FLAGS:
        assert f in S.OPTIONS_BY_CLI, f


def test_reference_defaults():
    s = S.Settings()
    assert (s.sizeX, s.sizeY, s.sizeZ) == (100, 100, 100)
    assert (s.pmlSizeX, s.tfsfSizeX, s.ntffSizeX) == (10, 20, 15)
    assert s.numTimeSteps == 100 and s.numAmplitudeTimeSteps == 10
    assert s.incidentWaveAngle1 == 90.0 and s.incidentWaveAngle2 == 0.0 and s.incidentWaveAngle3 == 90.0
    assert s.gridStep == 0.0005 and s.sourceWaveLength == 0.02
    assert s.bufferSize == 1 and s.intermediateSaveStep == 100
    assert s.fileWithAvailableTopologies == "nofile"
    assert s.getSizeX() == 100 and s.getPMLSizeX() == 10 and s.getDoUsePML() is False


def test_parse_and_same_size_semantics():
    st, s = S.setup_from_cmd(["--sizex", "64", "--same-size", "--sizez", "32", "--pml-sizex", "7",
                              "--same-size-pml", "--ntff-sizex", "9", "--same-size-ntff", "--use-pml", "--2d"],
                             out=io.StringIO())
    assert st == S.EXIT_OK
    assert (s.sizeX, s.sizeY, s.sizeZ) == (64, 64, 32)
    assert (s.pmlSizeY, s.pmlSizeZ) == (7, 7)
    # reference bug Settings.cpp:133-136 fixed: ntff copies ntff, tfsf untouched
    assert (s.ntffSizeY, s.ntffSizeZ, s.tfsfSizeY) == (9, 9, 20)
    assert s.doUsePML and s.dimension == 2


def test_unknown_option_and_help_version():
    out = io.StringIO()
    st, _ = S.setup_from_cmd(["--nope"], out=out)
    assert st == S.EXIT_UNKNOWN_OPTION and "Unknown option [--nope]" in out.getvalue()
    out = io.StringIO()
    st, _ = S.setup_from_cmd(["--help"], out=out)
    assert st == S.EXIT_BREAK_ARG_PARSING
    for f in REFERENCE_FLAGS:
        assert f in out.getvalue()
    out = io.StringIO()
    st, _ = S.setup_from_cmd(["--version"], out=out)
    assert st == S.EXIT_BREAK_ARG_PARSING and "0.2.2" in out.getvalue()


def test_cmd_file_roundtrip(tmp_path):
    f = tmp_path / "cmd.txt"
    out = io.StringIO()
    st, s = S.setup_from_cmd(["--3d", "--sizex", "48", "--use-pml", "--save-cmd-to-file", str(f)], out=out)
    assert st == S.EXIT_OK
    assert f.read_text().split() == ["--3d", "--sizex", "48", "--use-pml"]
    st, s2 = S.setup_from_cmd(["--cmd-from-file", str(f)], out=io.StringIO())
    assert st == S.EXIT_OK and s2.sizeX == 48 and s2.doUsePML
    # not combinable with other options, not nestable
    st, _ = S.setup_from_cmd(["--cmd-from-file", str(f), "--3d"], out=io.StringIO())
    assert st == S.EXIT_ERROR
    g = tmp_path / "nested.txt"
    g.write_text("--cmd-from-file\n%s\n" % f)
    st, _ = S.setup_from_cmd(["--cmd-from-file", str(g)], out=io.StringIO())
    assert st == S.EXIT_ERROR


def test_validation():
    st, _ = S.setup_from_cmd(["--angle-teta", "120"], out=io.StringIO())
    assert st != S.EXIT_OK
    st, _ = S.setup_from_cmd(["--dtype", "f16"], out=io.StringIO())
    assert st != S.EXIT_OK


# ---------------------------------------------------------------- coordinates
def test_coordinates_all_component_semantics():
    a, b = GridCoordinate3D(1, 2, 3), GridCoordinate3D(2, 3, 4)
    assert a < b and b > a and not (a < GridCoordinate3D(2, 3, 3))
    assert (a + b).as_tuple() == (3, 5, 7) and (b - a).as_tuple() == (1, 1, 1)
    # reference bug GridCoordinate3D.h:111: != compared z with ==
    assert GridCoordinate3D(1, 2, 3) != GridCoordinate3D(1, 2, 4)
    assert not (GridCoordinate3D(1, 2, 3) != GridCoordinate3D(1, 2, 3))
    assert a.calculate_total_coord() == 6 and b.get_max() == 4
    assert convert_coord(GridCoordinateFP3D(1.0, 2.0, 3.0)) == a
    with pytest.raises(Exception):
        convert_coord(GridCoordinateFP3D(1.5, 2.0, 3.0))


# --------------------------------------------------------------------- layout
def test_yee_layout_tables():
    from fdtd3d_amd.layout.yee import YeeLayout
    L = YeeLayout((10, 12, 14))
    assert L.global_range("Ex") == ((0, 1, 1), (9, 12, 14))
    assert L.global_range("Hz") == ((0, 0, 1), (9, 11, 14))
    assert L.coord_fp("Ey", (0, 0, 0)).as_tuple() == (0.5, 1.0, 0.5)
    T = YeeLayout((10, 12, 1), scheme="tmz")
    assert T.components == ("Ez", "Hx", "Hy")
    assert T.global_range("Ez") == ((1, 1, 0), (10, 12, 1))
    assert T.curl_terms("Hx") == (("Ez", 1, -1),)
    P = YeeLayout((20, 20, 20), pml_size=(4, 4, 4))
    assert P.is_in_pml((3.5, 10, 10)) and not P.is_in_pml((4.0, 10, 10)) and P.is_in_pml((16.0, 10, 10))
    # incident projections are an orthonormal triad for any angles
    R = YeeLayout((20, 20, 20), theta=0.7, phi=0.3, psi=1.1)
    e = np.array([R.incident_projection(c) for c in ("Ex", "Ey", "Ez")])
    h = np.array([R.incident_projection(c) for c in ("Hx", "Hy", "Hz")])
    k = np.array(R.incident_direction())
    assert abs(np.linalg.norm(e) - 1) < 1e-12 and abs(np.linalg.norm(h) - 1) < 1e-12
    assert abs(e @ h) < 1e-12 and abs(e @ k) < 1e-12 and abs(h @ k) < 1e-12


def test_phase_velocity_and_sphere():
    from fdtd3d_amd.layout.approximation import approximate_sphere, phase_velocity_incident_wave_3d
    from fdtd3d_amd.utils.constants import SPEED_OF_LIGHT
    # numerical phase velocity is below c and approaches c as resolution grows
    v40 = phase_velocity_incident_wave_3d(0.0005, 0.02, 0.5, 40, math.pi / 2, 0)
    v10 = phase_velocity_incident_wave_3d(0.002, 0.02, 0.5, 10, math.pi / 2, 0)
    assert v10 < v40 < SPEED_OF_LIGHT
    # oblique incidence via Newton agrees with the axis-aligned special case in the limit
    vo = phase_velocity_incident_wave_3d(0.0005, 0.02, 0.5, 40, 1.0, 0.3)
    assert abs(vo - v40) / v40 < 2e-3
    x = torch.tensor([0.0, 19.4, 20.0, 20.6, 30.0], dtype=torch.float64)
    e = approximate_sphere(x, torch.zeros_like(x), torch.zeros_like(x), (0, 0, 0), 20.0, 2.0)
    assert e[0] == 2.0 and e[-1] == 1.0 and abs(float(e[2]) - 1.5) < 1e-12


def test_sigma_profile_matches_reference_grading():
    from fdtd3d_amd.layout.materials import sigma_profile_1d
    p = sigma_profile_1d(41, 5, 0.0005, False)
    assert p[5:36].max() == 0.0
    assert (np.diff(p[:5]) < 0).all() and p[0] > 0
    # right PML starts at eps index N+1-P (reference Scheme3D.cpp:3700-3712)
    assert p[36] > 0 and p[35] == 0 and p[40] == p[0]


# ------------------------------------------------------------------- topology
def test_topology_optimizer_and_chunks():
    from fdtd3d_amd.parallel.topology import ParallelGridCore, buffer_directions, chunk_bounds, opposite
    c = ParallelGridCore.create((1024, 1024, 1024), 8)
    assert c.topology == (2, 2, 2)
    c = ParallelGridCore.create((2048, 1024, 1024), 8)
    assert c.topology == (2, 2, 2)
    c = ParallelGridCore.create((1024, 1024, 1024), 2)
    assert sorted(c.topology) == [1, 1, 2]
    c = ParallelGridCore.create((100, 40, 40), 4, "x")
    assert c.topology == (4, 1, 1)
    c = ParallelGridCore.create((64, 64, 64), 8, "xyz", requested=(8, 1, 1), optimal=False)
    assert c.topology == (8, 1, 1)
    assert chunk_bounds(10, 3, 0) == (0, 3) and chunk_bounds(10, 3, 2) == (6, 10)
    d = ParallelGridCore((16, 16, 16), 8, (2, 2, 2)).domain(7, 2)
    assert d.coords == (1, 1, 1) and d.lo == (8, 8, 8) and d.ghost_lo == (2, 2, 2) and d.ghost_hi == (0, 0, 0)
    assert d.neighbors[0] == (6, -1)
    dirs = buffer_directions()
    assert len(dirs) == 26 and dirs["LDB"] == (-1, -1, -1) and opposite("LU") == "RD"
    assert len(buffer_directions((0, 1))) == 8


# -------------------------------------------------------------------- I/O
def test_dat_roundtrip_and_layout(tmp_path):
    from fdtd3d_amd.io.dat import DATDumper, DATLoader
    from fdtd3d_amd.io.naming import GridFileType
    t = torch.arange(2 * 3 * 4, dtype=torch.float64).reshape(2, 3, 4)
    files = DATDumper(7, GridFileType.CURRENT, 3, "Ez", str(tmp_path)).dump_grid(t)
    assert os.path.basename(files[0]) == "current[7]_rank-3_Ez.dat"
    raw = np.fromfile(files[0], dtype=np.float64)
    assert raw.tolist() == list(range(24))  # z fastest, headerless
    back = DATLoader(7, GridFileType.CURRENT, 3, "Ez", str(tmp_path)).load_grid((2, 3, 4), torch.float64)
    assert torch.equal(back, t)
    im = -t.float()
    files = DATDumper(1, GridFileType.ALL, 0, "c", str(tmp_path)).dump_grid(t.float(), im)
    assert len(files) == 3 and os.path.getsize(files[0]) == 24 * 8  # complex<float>
    re2, im2 = DATLoader(1, GridFileType.CURRENT, 0, "c", str(tmp_path)).load_grid((2, 3, 4), torch.float32, True)
    assert torch.equal(re2, t.float()) and torch.equal(im2, im)


def test_bmp_roundtrip(tmp_path):
    from fdtd3d_amd.io.bmp import BMPDumper, BMPLoader, palette_rgb
    from fdtd3d_amd.io.naming import GridFileType
    x = torch.linspace(-1, 1, 37 * 21, dtype=torch.float64).reshape(37, 21, 1)
    d = BMPDumper(5, GridFileType.CURRENT, 0, "Ez", str(tmp_path))
    files = d.dump_grid(x, dim=2)
    assert os.path.basename(files[0]) == "current[5]_rank-0_Ez-Re.bmp"
    back = BMPLoader(5, GridFileType.CURRENT, 0, "Ez", str(tmp_path)).load_grid((37, 21, 1), -1.0, 1.0)
    assert float((back - x).abs().max()) < 2.0 / 255 * 1.01
    px = palette_rgb(np.array([-1.0, 0.0, 1.0]), -1.0, 1.0)
    assert px[0].tolist() == [0, 0, 255] and px[2].tolist() == [255, 0, 0]
    cube = torch.randn(6, 5, 4, dtype=torch.float64)
    files = BMPDumper(0, GridFileType.CURRENT, 0, "c", str(tmp_path)).dump_grid(cube, dim=3)
    assert len(files) == 4 and files[2].endswith("current[0]_rank-0_c2-Re.bmp")
    back = BMPLoader(0, GridFileType.CURRENT, 0, "c", str(tmp_path)).load_grid((6, 5, 4), float(cube.min()),
                                                                                  float(cube.max()))
    assert float((back - cube).abs().max()) < (float(cube.max() - cube.min())) / 255 * 2


def test_txt_roundtrip(tmp_path):
    from fdtd3d_amd.io.naming import GridFileType
    from fdtd3d_amd.io.txt import TXTDumper, read_txt
    t = torch.randn(3, 4, 5, dtype=torch.float64)
    f = TXTDumper(0, GridFileType.CURRENT, 0, "Hx", str(tmp_path)).dump_grid(t)[0]
    lines = [l for l in open(f).read().split("\n") if l]
    assert len(lines) == 60 and lines[0].split()[:3] == ["0", "0", "0"]
    assert torch.allclose(read_txt(f, (3, 4, 5)), t)


# ------------------------------------------------------- checkpoint / resume
def test_checkpoint_resume_bitwise(tmp_path):
    from fdtd3d_amd.io.checkpoint import load_checkpoint, save_checkpoint
    from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
    from fdtd3d_amd.ops import make_ops
    cfg = SchemeConfig(scheme="3d", size=(24, 24, 24), time_steps=20, use_pml=True, use_tfsf=True,
                       use_metamaterials=True, pml_size=(4, 4, 4), tfsf_size=(7, 7, 7))

    def mk():
        s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
        s.init_scheme()
        s.init_grids()
        return s

    full = mk()
    full.perform_steps(20)
    half = mk()
    half.perform_steps(11)
    save_checkpoint(half, str(tmp_path))
    resumed = mk()
    assert load_checkpoint(resumed, str(tmp_path)) == 11
    resumed.perform_steps(9)
    for c in full.comps:
        assert torch.equal(full.F[0][c], resumed.F[0][c]), c


# ------------------------------------------------------------------- NTFF
def _run(cfg):
    from fdtd3d_amd.models.scheme import YeeScheme
    from fdtd3d_amd.ops import make_ops
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    s.perform_steps()
    return s


def test_ntff_dipole_pattern():
    """z-directed source: strong, nearly isotropic radiation in the xy plane,
    a null along the dipole axis."""
    from fdtd3d_amd.models.ntff import ntff_power, reference_angles
    from fdtd3d_amd.models.scheme import SchemeConfig
    cfg = SchemeConfig(scheme="3d", size=(40, 40, 40), time_steps=200, scene="vacuum", use_pml=True,
                       pml_type="cpml", pml_size=(8, 8, 8), complex_values=True, ntff_size=(11, 11, 11),
                       wavelength=0.01)
    s = _run(cfg)
    phis = reference_angles()
    assert phis.numel() == 181
    re = {c: s.F[0][c] for c in s.comps}
    im = {c: s.F[1][c] for c in s.comps}
    p = ntff_power(re, im, cfg.size, cfg.ntff_size, s.dx, s.wavelength, math.pi / 2, phis)
    p0 = ntff_power(re, im, cfg.size, cfg.ntff_size, s.dx, s.wavelength, 0.01, phis)
    assert torch.isfinite(p).all() and float(p.min()) > 0
    assert float(p.std() / p.mean()) < 0.2
    assert float(p0.mean()) < 1e-2 * float(p.mean())


def test_ntff_extinction_of_plane_wave():
    """A closed NTFF surface inside the total-field region of a TF/SF plane wave
    with no scatterer radiates nothing (equivalence principle): J and M
    contributions must cancel, which checks positions, signs and phases."""
    from fdtd3d_amd.models.ntff import ETA0, ntff_power, reference_angles
    from fdtd3d_amd.models.scheme import SchemeConfig
    cfg = SchemeConfig(scheme="3d", size=(48, 48, 48), time_steps=260, scene="vacuum", use_pml=True,
                       wavelength=0.01, pml_type="cpml", pml_size=(8, 8, 8), complex_values=True, use_tfsf=True,
                       tfsf_size=(11, 11, 11), ntff_size=(15, 15, 15))
    s = _run(cfg)
    re = {c: s.F[0][c] for c in s.comps}
    im = {c: s.F[1][c] for c in s.comps}
    p = ntff_power(re, im, cfg.size, cfg.ntff_size, s.dx, s.wavelength, math.pi / 2, reference_angles())
    # scale: one face of the box radiating alone
    k = 2 * math.pi / s.wavelength
    area = ((48 - 30) * s.dx) ** 2
    one_face = k * k / (8 * math.pi) * (area * 1.0) ** 2
    assert float(p.max()) < 1e-2 * one_face


# ------------------------------------------------------------------ driver
def test_driver_end_to_end(tmp_path):
    from fdtd3d_amd.runner import run
    out = io.StringIO()
    rc = run(["--3d", "--sizex", "24", "--same-size", "--time-steps", "12", "--use-pml", "--pml-sizex", "4",
              "--same-size-pml", "--save-res", "--save-as-dat", "--output-dir", str(tmp_path), "--json",
              "--checkpoint-dir", str(tmp_path / "ck")], out=out)
    assert rc == 0
    txt = out.getvalue()
    assert "Total time =" in txt and "Grid size: 24x24x24" in txt and "Mcells/s" in txt
    assert (tmp_path / "current[12]_rank-0_Ez.dat").exists()
    rc = run(["--3d", "--sizex", "24", "--same-size", "--time-steps", "20", "--use-pml", "--pml-sizex", "4",
              "--same-size-pml", "--load-from-file", str(tmp_path / "ck")], out=io.StringIO())
    assert rc == 0
    rc = run(["--2d", "--2d-mode", "tez", "--sizex", "40", "--same-size", "--time-steps", "10"], out=io.StringIO())
    assert rc == 0
    assert run(["--help"], out=io.StringIO()) == 0


def test_phase_profiler_report():
    import io
    from fdtd3d_amd.runner import run
    out = io.StringIO()
    assert run(["--3d", "--sizex", "16", "--same-size", "--time-steps", "4", "--use-pml", "--pml-sizex", "3",
                "--same-size-pml", "--profile-phases", "--backend", "torch", "--device", "cpu", "--json"],
               out=out) == 0
    text = out.getvalue()
    assert "Phase timings" in text
    import json
    rec = json.loads([l for l in text.splitlines() if l.startswith("{")][-1])
    assert rec["phases"]["E"]["calls"] == 4 and rec["phases"]["H"]["calls"] == 4


# ---------------------------------------------------------------- periodic work
def test_periodic_hooks_fire_on_schedule():
    """YeeScheme.add_periodic: fires after every step t with (t - offset) %
    period == 0, across several advance() calls, in registration order."""
    from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
    from fdtd3d_amd.ops import make_ops
    cfg = SchemeConfig(scheme="3d", size=(8, 8, 8), dtype="f64", scene="vacuum", time_steps=0)
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    seen = []
    s.add_periodic(10, 1, lambda sc, t: seen.append(("a", t, sc.t)))
    s.add_periodic(7, 0, lambda sc, t: seen.append(("b", t, sc.t)))
    s.advance(12)
    s.advance(13)
    assert [x for x in seen if x[0] == "a"] == [("a", 1, 1), ("a", 11, 11), ("a", 21, 21)]
    assert [x for x in seen if x[0] == "b"] == [("b", 7, 7), ("b", 14, 14), ("b", 21, 21)]
    assert seen.index(("a", 21, 21)) < seen.index(("b", 21, 21))
    assert s.t == 25
