"""Standalone native driver (csrc/main.cpp) on the GPU vs the Python driver
on the torch CPU backend: identical final fields for the plain Yee schemes."""
import io
import os
import subprocess

import numpy as np
import pytest

from fdtd3d_amd import native
from fdtd3d_amd.runner import run as py_run

CASES = {
    "3d_fused_vacuum": ["--3d", "--sizex", "28", "--sizey", "20", "--sizez", "24", "--time-steps", "12",
                        "--scene", "vacuum"],
    "3d_tb2_vacuum": ["--3d", "--sizex", "28", "--sizey", "20", "--sizez", "24", "--time-steps", "13",
                      "--scene", "vacuum", "--time-block", "2", "--warmup-steps", "3"],
    "3d_split_vacuum": ["--3d", "--sizex", "28", "--sizey", "20", "--sizez", "24", "--time-steps", "12",
                        "--scene", "vacuum", "--split-kernels"],
    "3d_fused_sphere": ["--3d", "--sizex", "32", "--same-size", "--time-steps", "15", "--scene", "sphere",
                        "--sphere-center-x", "16", "--sphere-center-y", "16", "--sphere-center-z", "16",
                        "--sphere-radius", "6", "--sphere-eps", "4"],
    "2d_tmz": ["--2d", "--sizex", "60", "--sizey", "50", "--time-steps", "25", "--scene", "vacuum"],
    "2d_tez": ["--2d", "--2d-mode", "tez", "--sizex", "60", "--sizey", "50", "--time-steps", "25",
               "--scene", "vacuum"],
    "1d": ["--1d", "--sizex", "300", "--time-steps", "40", "--scene", "vacuum", "--source", "gaussian",
           "--gaussian-width", "8", "--gaussian-delay", "30"],
    # blocked 2D passes (ny % 4 == 0; 23 steps = 4 passes of 5 + a tail of 3) and the per-step kernels
    "2d_tmz_tb5": ["--2d", "--sizex", "60", "--sizey", "52", "--time-steps", "23", "--scene", "vacuum",
                   "--time-block", "5"],
    "2d_tez_tb": ["--2d", "--2d-mode", "tez", "--sizex", "44", "--sizey", "64", "--time-steps", "25",
                  "--scene", "vacuum"],
    "2d_tmz_split": ["--2d", "--sizex", "60", "--sizey", "52", "--time-steps", "25", "--scene", "vacuum",
                     "--split-kernels"],
    "1d_split": ["--1d", "--sizex", "300", "--time-steps", "40", "--scene", "vacuum", "--source", "gaussian",
                 "--gaussian-width", "8", "--gaussian-delay", "30", "--split-kernels"],
    # CPML (3D fp32, folded float4 kernels): slabs of different thickness per axis, kappa / alpha
    "3d_cpml": ["--3d", "--sizex", "36", "--sizey", "32", "--sizez", "40", "--time-steps", "30", "--scene", "vacuum",
                "--use-pml", "--pml-type", "cpml", "--pml-sizex", "6", "--pml-sizey", "5", "--pml-sizez", "7"],
    "3d_cpml_sphere_kappa": ["--3d", "--sizex", "32", "--same-size", "--time-steps", "24", "--scene", "sphere",
                             "--sphere-center-x", "16", "--sphere-center-y", "16", "--sphere-center-z", "16",
                             "--sphere-radius", "5", "--sphere-eps", "3", "--use-pml", "--pml-type", "cpml",
                             "--pml-sizex", "6", "--same-size-pml", "--cpml-kappa-max", "3",
                             "--cpml-alpha-max", "0.05"],
    # 3D CPML on z rows of a size not divisible by 4: the scalar split kernels + the generic slab corrections
    "3d_cpml_tfsf_z42": ["--3d", "--sizex", "30", "--sizey", "28", "--sizez", "42", "--time-steps", "24", "--scene",
                         "sphere", "--sphere-center-x", "15", "--sphere-center-y", "14", "--sphere-center-z", "21",
                         "--sphere-radius", "4", "--sphere-eps", "3", "--use-pml", "--pml-type", "cpml",
                         "--pml-sizex", "5", "--same-size-pml", "--cpml-kappa-max", "2", "--cpml-alpha-max", "0.05",
                         "--use-tfsf", "--tfsf-sizex", "9", "--same-size-tfsf", "--angle-teta", "50", "--angle-phi",
                         "30", "--angle-psi", "20"],
    # TF/SF plane wave (oblique incidence; fp32 and fp64), and CPML + TF/SF (BASELINE config 3, fp32)
    "3d_tfsf": ["--3d", "--sizex", "36", "--sizey", "32", "--sizez", "40", "--time-steps", "30", "--scene", "sphere",
                "--sphere-center-x", "18", "--sphere-center-y", "16", "--sphere-center-z", "20", "--sphere-radius",
                "4", "--sphere-eps", "2", "--use-tfsf", "--tfsf-sizex", "8", "--tfsf-sizey", "7", "--tfsf-sizez", "9",
                "--angle-teta", "50", "--angle-phi", "30", "--angle-psi", "20"],
    "3d_cpml_tfsf": ["--3d", "--sizex", "40", "--same-size", "--time-steps", "30", "--scene", "vacuum",
                     "--use-pml", "--pml-type", "cpml", "--pml-sizex", "6", "--same-size-pml", "--use-tfsf",
                     "--tfsf-sizex", "10", "--same-size-tfsf", "--angle-teta", "60", "--angle-phi", "10",
                     "--angle-psi", "5"],
    # hybrid passes (blocked core + stepped CPML / TF/SF shell, csrc/main.cpp hybrid_pass): grids large
    # enough for the core to hold a quarter of the cells; 23 steps = 4 passes of 5 + a 3-step tail
    "3d_cpml_tfsf_hybrid": ["--3d", "--sizex", "104", "--same-size", "--time-steps", "23", "--scene", "vacuum",
                            "--use-pml", "--pml-type", "cpml", "--pml-sizex", "6", "--same-size-pml", "--use-tfsf",
                            "--tfsf-sizex", "10", "--same-size-tfsf", "--angle-teta", "60", "--angle-phi", "10",
                            "--angle-psi", "5"],
    "3d_cpml_point_hybrid": ["--3d", "--sizex", "72", "--sizey", "76", "--sizez", "80", "--time-steps", "17",
                             "--scene", "vacuum", "--use-pml", "--pml-type", "cpml", "--pml-sizex", "6",
                             "--pml-sizey", "7", "--pml-sizez", "5", "--hybrid-block", "4"],
    # hybrid passes with the UPML (chain slabs whole in every shell step, plain kernels on the windows' inner
    # parts)
    "3d_upml_tfsf_hybrid": ["--3d", "--sizex", "104", "--same-size", "--time-steps", "23", "--scene", "vacuum",
                            "--use-pml", "--pml-sizex", "5", "--same-size-pml", "--use-tfsf", "--tfsf-sizex", "10",
                            "--same-size-tfsf", "--angle-teta", "50", "--angle-phi", "20", "--angle-psi", "10"],
    "3d_upml_point_hybrid": ["--3d", "--sizex", "72", "--sizey", "76", "--sizez", "80", "--time-steps", "17",
                             "--scene", "vacuum", "--use-pml", "--pml-sizex", "6", "--pml-sizey", "7", "--pml-sizez",
                             "5", "--hybrid-block", "4"],
    # TF/SF without absorbing layers: hybrid passes with the TF/SF band in the stepped shell
    "3d_tfsf_hybrid": ["--3d", "--sizex", "100", "--sizey", "96", "--sizez", "104", "--time-steps", "23", "--scene",
                       "vacuum", "--use-tfsf", "--tfsf-sizex", "9", "--tfsf-sizey", "8", "--tfsf-sizez", "10",
                       "--angle-teta", "40", "--angle-phi", "25", "--angle-psi", "15"],
    # hybrid passes around a Drude sphere (the dispersive box cut out of the core, its chain whole in every
    # shell step), with the UPML and without absorbing layers (the core reaches the domain faces)
    "3d_drude_upml_hybrid": ["--3d", "--sizex", "96", "--sizey", "88", "--sizez", "92", "--time-steps", "23",
                             "--scene", "drude-sphere", "--use-metamaterials", "--use-pml", "--pml-sizex", "5",
                             "--same-size-pml", "--sphere-center-x", "48", "--sphere-center-y", "44",
                             "--sphere-center-z", "46", "--sphere-radius", "6"],
    "3d_drude_hybrid": ["--3d", "--sizex", "80", "--same-size", "--time-steps", "17", "--scene", "drude-sphere",
                        "--use-metamaterials", "--sphere-center-x", "40", "--sphere-center-y", "38",
                        "--sphere-center-z", "41", "--sphere-radius", "7", "--hybrid-block", "4"],
    # UPML in the reference's D/B form (fused chain kernel) + oblique TF/SF, a dielectric sphere with the
    # UPML (per-cell 1/(eps eps0) in the chain), Drude and Lorentz spheres + UPML (uint8 index + table)
    "3d_upml_tfsf": ["--3d", "--sizex", "36", "--sizey", "32", "--sizez", "40", "--time-steps", "30",
                     "--scene", "vacuum", "--use-pml", "--pml-sizex", "5", "--pml-sizey", "4", "--pml-sizez", "6",
                     "--use-tfsf", "--tfsf-sizex", "9", "--tfsf-sizey", "8", "--tfsf-sizez", "10",
                     "--angle-teta", "60", "--angle-phi", "20", "--angle-psi", "30"],
    "3d_upml_sphere": ["--3d", "--sizex", "32", "--same-size", "--time-steps", "24", "--scene", "sphere",
                       "--sphere-center-x", "16", "--sphere-center-y", "16", "--sphere-center-z", "16",
                       "--sphere-radius", "5", "--sphere-eps", "3", "--use-pml", "--pml-sizex", "5",
                       "--same-size-pml"],
    "3d_drude_upml": ["--3d", "--sizex", "40", "--sizey", "36", "--sizez", "32", "--time-steps", "24",
                      "--scene", "drude-sphere", "--use-metamaterials", "--use-pml", "--pml-sizex", "5",
                      "--same-size-pml", "--sphere-center-x", "20", "--sphere-center-y", "18",
                      "--sphere-center-z", "16", "--sphere-radius", "7"],
    "3d_lorentz_upml_tfsf": ["--3d", "--sizex", "40", "--same-size", "--time-steps", "24", "--scene",
                             "drude-sphere", "--use-metamaterials", "--dispersion", "lorentz", "--lorentz-omega0",
                             "0.7", "--use-pml", "--pml-sizex", "5", "--same-size-pml", "--sphere-center-x", "20",
                             "--sphere-center-y", "20", "--sphere-center-z", "20", "--sphere-radius", "6",
                             "--use-tfsf", "--tfsf-sizex", "9", "--same-size-tfsf"],
    # 2D absorbing layers and TF/SF (generic slab / chain kernels, csrc/main.cpp Pml2d): the reference's
    # UPML with an oblique plane wave, the CPML with kappa / alpha, dielectric cylinders (per-cell coefficients)
    "2d_tmz_upml_tfsf": ["--2d", "--sizex", "60", "--sizey", "52", "--time-steps", "30", "--scene", "vacuum",
                         "--use-pml", "--pml-sizex", "6", "--pml-sizey", "5", "--use-tfsf", "--tfsf-sizex", "10",
                         "--tfsf-sizey", "9", "--angle-phi", "30"],
    "2d_tez_cpml": ["--2d", "--2d-mode", "tez", "--sizex", "60", "--sizey", "52", "--time-steps", "30",
                    "--scene", "vacuum", "--use-pml", "--pml-type", "cpml", "--pml-sizex", "6", "--pml-sizey", "7",
                    "--cpml-kappa-max", "2", "--cpml-alpha-max", "0.05"],
    "2d_tmz_cpml_tfsf_sphere": ["--2d", "--sizex", "64", "--sizey", "56", "--time-steps", "30", "--scene", "sphere",
                                "--sphere-center-x", "32", "--sphere-center-y", "28", "--sphere-radius", "7",
                                "--sphere-eps", "3", "--use-pml", "--pml-type", "cpml", "--pml-sizex", "6",
                                "--same-size-pml", "--use-tfsf", "--tfsf-sizex", "11", "--tfsf-sizey", "10",
                                "--angle-phi", "20", "--angle-psi", "90"],
    "2d_tez_upml_sphere": ["--2d", "--2d-mode", "tez", "--sizex", "56", "--sizey", "60", "--time-steps", "30",
                           "--scene", "sphere", "--sphere-center-x", "28", "--sphere-center-y", "30",
                           "--sphere-radius", "6", "--sphere-eps", "4", "--use-pml", "--pml-sizex", "5",
                           "--pml-sizey", "6"],
    # 2D hybrid passes (yee2d_tb.hip core + stepped strips): CPML + oblique TF/SF, UPML + point source
    "2d_tmz_cpml_tfsf_hybrid": ["--2d", "--sizex", "200", "--sizey", "192", "--time-steps", "23", "--scene",
                                "vacuum", "--use-pml", "--pml-type", "cpml", "--pml-sizex", "6", "--same-size-pml",
                                "--use-tfsf", "--tfsf-sizex", "10", "--tfsf-sizey", "12", "--angle-phi", "35"],
    "2d_tez_upml_point_hybrid": ["--2d", "--2d-mode", "tez", "--sizex", "180", "--sizey", "176", "--time-steps",
                                 "17", "--scene", "vacuum", "--use-pml", "--pml-sizex", "8", "--pml-sizey", "7",
                                 "--hybrid-block", "5"],
    # amplitude mode: 3D vacuum (fp32: blocked passes with the running maxima folded in), CPML (per step),
    # 2D with the CPML until the stable state (fp64: the same converged step as the Python driver)
    "3d_amp": ["--3d", "--sizex", "32", "--sizey", "28", "--sizez", "24", "--time-steps", "6", "--scene", "vacuum",
               "--use-amp-mode", "--amplitude-time-steps", "20"],
    "3d_amp_cpml": ["--3d", "--sizex", "32", "--sizey", "28", "--sizez", "24", "--time-steps", "5", "--scene",
                    "vacuum", "--use-amp-mode", "--amplitude-time-steps", "13", "--use-pml", "--pml-type", "cpml",
                    "--pml-sizex", "5", "--same-size-pml"],
    "2d_tmz_amp_cpml": ["--2d", "--sizex", "60", "--sizey", "52", "--time-steps", "10", "--scene", "vacuum",
                        "--use-amp-mode", "--amplitude-time-steps", "300", "--use-pml", "--pml-type", "cpml"],
}
# (round 6: the native hybrid passes run in both precisions -- fp64 blocked core, Drude pass and CPML windows)
FP32_ONLY = set()
# the converged step depends on running-maximum comparisons at round-off level: fp64 only
FP64_ONLY = {"2d_tmz_amp_cpml"}

COMPS = {"3d": ["Ex", "Ey", "Ez", "Hx", "Hy", "Hz"], "tmz": ["Ez", "Hx", "Hy"], "tez": ["Ex", "Ey", "Hz"],
         "1d": ["Ez", "Hy"]}


def _shape(argv):
    def get(flag, default):
        return int(argv[argv.index(flag) + 1]) if flag in argv else default
    nx = get("--sizex", 100)
    same = "--same-size" in argv
    if "--1d" in argv:
        return (nx, 1, 1), "1d"
    if "--2d" in argv:
        return (nx, nx if same else get("--sizey", 100), 1), ("tez" if "tez" in argv else "tmz")
    return (nx, nx if same else get("--sizey", 100), nx if same else get("--sizez", 100)), "3d"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("case", list(CASES))
def test_native_driver_matches_python(case, dtype, tmp_path, gpu):
    exe = native.executable()
    assert os.path.exists(exe), "native fdtd3d executable missing (run python -m fdtd3d_amd.ops.build)"
    if case in FP32_ONLY and dtype != "f32":
        pytest.skip("native hybrid passes: fp32")
    if case in FP64_ONLY and dtype != "f64":
        pytest.skip("converged amplitude step compared in fp64")
    argv = CASES[case] + ["--dtype", dtype, "--save-res", "--save-as-dat"]
    nd, pd = tmp_path / "native", tmp_path / "py"
    nd.mkdir()
    pd.mkdir()
    r = subprocess.run([exe] + argv + ["--output-dir", str(nd)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Mcells/s" in r.stdout
    assert ("hybrid passes" in r.stdout) == case.endswith("_hybrid"), r.stdout
    pbuf = io.StringIO()
    assert py_run(argv[:-4] + ["--dtype", "f64", "--save-res", "--save-as-dat", "--backend", "torch",
                               "--device", "cpu", "--output-dir", str(pd)], out=pbuf) == 0
    shape, scheme = _shape(argv)
    steps = int(argv[argv.index("--time-steps") + 1])
    if "--use-amp-mode" in argv:
        # the same amplitude steps (and converged step) in both drivers
        na = [l for l in r.stdout.splitlines() if l.startswith("Amplitude mode:")]
        pa = [l for l in pbuf.getvalue().splitlines() if l.startswith("Amplitude mode:")]
        assert na and na == pa, (na, pa)
        steps += int(na[0].split("after ")[1].split()[0]) if "not reached" in na[0] else \
            int(na[0].split("(")[1].split()[0])
    ndt = np.float32 if dtype == "f32" else np.float64
    errs = {}
    for c in COMPS[scheme]:
        name = "current[%d]_rank-0_%s.dat" % (steps, c)
        a = np.fromfile(nd / name, dtype=ndt).astype(np.float64).reshape(shape)
        b = np.fromfile(pd / name, dtype=np.float64).reshape(shape)
        errs[c] = (np.abs(a - b).max(), np.abs(b).max())
    for kind in "EH":
        peak = max(v[1] for c, v in errs.items() if c[0] == kind)
        tol = 1e-11 if dtype == "f64" else 2e-5
        for c, (err, _) in errs.items():
            if c[0] == kind:
                assert err <= tol * peak + 1e-300, (c, err, peak)


NTFF_ARGV = ["--3d", "--sizex", "40", "--same-size", "--time-steps", "31", "--scene", "sphere", "--sphere-center-x",
             "20", "--sphere-center-y", "20", "--sphere-center-z", "20", "--sphere-radius", "5", "--sphere-eps", "3",
             "--use-pml", "--pml-sizex", "5", "--same-size-pml", "--use-tfsf", "--tfsf-sizex", "9",
             "--same-size-tfsf", "--use-ntff", "--ntff-sizex", "12", "--same-size-ntff", "--ntff-step", "10"]


def _ntff_lines(text):
    out = []
    for line in text.splitlines():
        if line.startswith("=== t="):
            head, val = line.rsplit("===", 1)
            out.append((head.strip(), float(val)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_native_ntff_matches_python(dtype, gpu):
    """The native driver's NTFF scattered power diagram (native_physics.h) at
    the reference's angles and report steps against the Python driver's
    (models/ntff.py) on the torch CPU backend, same UPML + TF/SF + sphere run."""
    exe = native.executable()
    assert os.path.exists(exe)
    r = subprocess.run([exe] + NTFF_ARGV + ["--dtype", dtype], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    buf = io.StringIO()
    assert py_run(NTFF_ARGV + ["--dtype", "f64", "--backend", "torch", "--device", "cpu"], out=buf) == 0
    a, b = _ntff_lines(r.stdout), _ntff_lines(buf.getvalue())
    assert len(a) == len(b) == 4 * 181, (len(a), len(b))  # t = 0, 10, 20, 30
    assert [h for h, _ in a] == [h for h, _ in b]
    peak = max(abs(v) for _, v in b)
    assert peak > 0
    tol = 1e-9 if dtype == "f64" else 2e-4
    for (h, x), (_, y) in zip(a, b):
        assert abs(x - y) <= tol * peak, (h, x, y, peak)


@pytest.mark.gpu
def test_native_parallel_grid_checkpoint(tmp_path):
    """Checkpoints of a decomposed native run (2x2x1 ranks, the gathered grid in the serial form): resumed by
    the decomposed native run, by the single-rank native run and by the Python driver, every one ends on the
    fields of the Python driver's full run (fp64)."""
    exe = native.executable()
    argv = ["--3d", "--sizex", "28", "--sizey", "20", "--sizez", "24", "--scene", "vacuum", "--time-block", "3",
            "--dtype", "f64"]
    par = ["--parallel-grid", "--topology-sizex", "2", "--topology-sizey", "2"]
    py = ["--backend", "torch", "--device", "cpu"]
    k, n = 7, 19
    d = {x: tmp_path / x for x in ("a", "par", "one", "py", "full")}

    def nat(extra):
        r = subprocess.run([exe] + argv + extra, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        return r.stdout

    out = nat(par + ["--time-steps", str(2 * k + 1), "--checkpoint-dir", str(d["a"]), "--checkpoint-step", str(k)])
    assert "Number of processes: 4" in out
    for t in (k, 2 * k, 2 * k + 1):
        side = d["a"] / ("checkpoint[%d]_rank-0.json" % t)
        assert side.exists(), t
        if t != k:
            side.unlink()
    out = nat(par + ["--time-steps", str(n), "--load-from-file", str(d["a"]), "--checkpoint-dir", str(d["par"])])
    assert "Number of time steps: %d (%d timed" % (n, n - k) in out, out
    nat(["--time-steps", str(n), "--load-from-file", str(d["a"]), "--checkpoint-dir", str(d["one"])])
    assert py_run(argv + py + ["--time-steps", str(n), "--load-from-file", str(d["a"]), "--checkpoint-dir",
                               str(d["py"])], out=io.StringIO()) == 0
    assert py_run(argv + py + ["--time-steps", str(n), "--checkpoint-dir", str(d["full"])], out=io.StringIO()) == 0
    shape = (28, 20, 24)
    for kind in "EH":
        errs, peak = [], 0.0
        for c in "xyz":
            name = "current[%d]_rank-0_%s%s.dat" % (n, kind, c)
            ref = np.fromfile(d["full"] / name, dtype=np.float64).reshape(shape)
            peak = max(peak, np.abs(ref).max())
            errs += [np.abs(np.fromfile(d[x] / name, dtype=np.float64).reshape(shape) - ref).max()
                     for x in ("par", "one", "py")]
        assert peak > 0
        assert max(errs) <= 1e-11 * peak, (kind, errs, peak)


COMPLEX = {
    "3d_cpml_tfsf": CASES["3d_cpml_tfsf"],
    "3d_vacuum_blocked": ["--3d", "--sizex", "32", "--sizey", "28", "--sizez", "24", "--time-steps", "13", "--scene",
                          "vacuum"],
    "3d_drude_upml": CASES["3d_drude_upml"],
    "2d_tmz_upml_tfsf": CASES["2d_tmz_upml_tfsf"],
    "1d_gauss": ["--1d", "--sizex", "300", "--time-steps", "40", "--scene", "vacuum", "--source", "gaussian",
                 "--gaussian-width", "8", "--gaussian-delay", "30"],
}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("case", list(COMPLEX))
def test_native_complex_matches_python(case, dtype, tmp_path):
    """Complex fields natively (the real and imaginary planes as two real runs, sin / cos source) against the
    Python driver's complex run (torch CPU, fp64): the interleaved complex DAT outputs agree."""
    exe = native.executable()
    argv = COMPLEX[case] + ["--complex-field-values", "--save-res", "--save-as-dat"]
    nd, pd = tmp_path / "native", tmp_path / "py"
    nd.mkdir()
    pd.mkdir()
    r = subprocess.run([exe] + argv + ["--dtype", dtype, "--output-dir", str(nd)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Complex field values: 1" in r.stdout, r.stdout
    assert py_run(argv + ["--dtype", "f64", "--backend", "torch", "--device", "cpu", "--output-dir", str(pd)],
                  out=io.StringIO()) == 0
    shape, scheme = _shape(argv)
    steps = int(argv[argv.index("--time-steps") + 1])
    ndt = np.complex64 if dtype == "f32" else np.complex128
    tol = 1e-11 if dtype == "f64" else 2e-5
    for kind in "EH":
        errs, peak = [], 0.0
        for c in [c for c in COMPS[scheme] if c[0] == kind]:
            name = "current[%d]_rank-0_%s.dat" % (steps, c)
            a = np.fromfile(nd / name, dtype=ndt).astype(np.complex128).reshape(shape)
            b = np.fromfile(pd / name, dtype=np.complex128).reshape(shape)
            errs.append(np.abs(a - b).max())
            peak = max(peak, np.abs(b).max())
        assert peak > 0
        assert max(errs) <= tol * peak, (kind, errs, peak)


AMP_MULTI = {
    "amp_2x2x1": (CASES["3d_amp"], ["--topology-sizex", "2", "--topology-sizey", "2"]),
    "amp_cpml_2x1x2": (CASES["3d_amp_cpml"], ["--topology-sizex", "2", "--topology-sizez", "2"]),
    # until the stable state (the near-convergence snapshot and the redone period over the ranks)
    "amp_2d_tmz_cpml_2x2": (CASES["2d_tmz_amp_cpml"], ["--topology-sizex", "2", "--topology-sizey", "2"]),
    # (the single-rank run: stable after 1015 steps)
    "amp_cpml_stable_2x2x1": (["--3d", "--sizex", "20", "--same-size", "--time-steps", "5", "--scene", "vacuum",
                               "--use-amp-mode", "--amplitude-time-steps", "1200", "--use-pml", "--pml-type", "cpml",
                               "--pml-sizex", "5", "--same-size-pml"],
                              ["--topology-sizex", "2", "--topology-sizey", "2"]),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(AMP_MULTI))
def test_native_parallel_grid_amplitude(case, tmp_path):
    """Amplitude mode of a decomposed native run (running maxima per rank, changed counts summed over the ranks
    per check period): the same amplitude steps and final fields as the single-rank native run (fp64)."""
    exe = native.executable()
    base, topo = AMP_MULTI[case]
    argv = base + ["--dtype", "f64", "--save-res", "--save-as-dat"]
    outs = {}
    for lab, extra in (("one", []), ("par", ["--parallel-grid"] + topo)):
        d = tmp_path / lab
        d.mkdir()
        r = subprocess.run([exe] + argv + extra + ["--output-dir", str(d)], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        outs[lab] = [l for l in r.stdout.splitlines() if l.startswith("Amplitude mode:")]
    assert outs["one"] and outs["one"] == outs["par"], outs
    line = outs["one"][0]
    steps = int(base[base.index("--time-steps") + 1])
    steps += int(line.split("after ")[1].split()[0]) if "not reached" in line else int(line.split("(")[1].split()[0])
    if case.endswith("stable_2x2x1"):
        assert "stable after" in line, line
    shape, scheme = _shape(argv)
    for kind in "EH":
        errs, peak = [], 0.0
        for c in [c[1] for c in COMPS[scheme] if c[0] == kind]:
            name = "current[%d]_rank-0_%s%s.dat" % (steps, kind, c)
            a = np.fromfile(tmp_path / "par" / name, dtype=np.float64).reshape(shape)
            b = np.fromfile(tmp_path / "one" / name, dtype=np.float64).reshape(shape)
            errs.append(np.abs(a - b).max())
            peak = max(peak, np.abs(b).max())
        assert peak > 0
        assert max(errs) <= 1e-12 * peak, (kind, errs, peak)


@pytest.mark.gpu
def test_native_ntff_parallel_grid():
    """The NTFF diagram of a decomposed native run (2x2x1 ranks: UPML chain + TF/SF + sphere on the split half
    steps, the grid gathered for each report) equals the single-rank native run's to fp64 round-off."""
    exe = native.executable()
    argv = NTFF_ARGV + ["--dtype", "f64"]
    one = subprocess.run([exe] + argv, capture_output=True, text=True, timeout=300)
    assert one.returncode == 0, one.stdout + one.stderr
    par = subprocess.run([exe] + argv + ["--parallel-grid", "--topology-sizex", "2", "--topology-sizey", "2"],
                         capture_output=True, text=True, timeout=300)
    assert par.returncode == 0, par.stdout + par.stderr
    assert "Number of processes: 4" in par.stdout
    a, b = _ntff_lines(par.stdout), _ntff_lines(one.stdout)
    assert len(a) == len(b) == 4 * 181, (len(a), len(b))
    assert [h for h, _ in a] == [h for h, _ in b]
    peak = max(abs(v) for _, v in b)
    assert peak > 0
    for (h, x), (_, y) in zip(a, b):
        assert abs(x - y) <= 1e-11 * peak, (h, x, y, peak)


# parallel grids of the native driver (csrc/native_multi.h run_multi): 3 / 4 / 8 ranks of one process on one
# GPU (ghost boxes packed, copied and unpacked on the device; peer xGMI copies on a multi-GPU node), 23 steps =
# passes + a tail; x slabs, x-y and x-z grids (edge messages) and a 2x2x2 grid (corner messages); the 4-rank x
# case puts the source on a rank's first plane (its lower neighbour's ghosts hold it too)
MULTI = {
    "f32_vacuum_3ranks": ["--3d", "--sizex", "40", "--sizey", "24", "--sizez", "32", "--time-steps", "23",
                          "--scene", "vacuum", "--parallel-grid", "--topology-sizex", "3", "--dtype", "f32"],
    "f64_sphere_4ranks": ["--3d", "--sizex", "36", "--sizey", "20", "--sizez", "24", "--time-steps", "23",
                          "--scene", "sphere", "--sphere-center-x", "17", "--sphere-center-y", "10",
                          "--sphere-center-z", "12", "--sphere-radius", "5", "--sphere-eps", "3", "--parallel-grid",
                          "--topology-sizex", "4", "--time-block", "3", "--dtype", "f64"],
    "f32_vacuum_2x2x1": ["--3d", "--sizex", "40", "--sizey", "36", "--sizez", "32", "--time-steps", "23",
                         "--scene", "vacuum", "--parallel-grid", "--topology-sizex", "2", "--topology-sizey", "2",
                         "--dtype", "f32"],
    "f32_sphere_2x1x2": ["--3d", "--sizex", "36", "--sizey", "24", "--sizez", "40", "--time-steps", "23",
                         "--scene", "sphere", "--sphere-center-x", "18", "--sphere-center-y", "11",
                         "--sphere-center-z", "19", "--sphere-radius", "6", "--sphere-eps", "3", "--parallel-grid",
                         "--topology-sizex", "2", "--topology-sizez", "2", "--time-block", "4", "--dtype", "f32"],
    "f64_vacuum_2x2x2": ["--3d", "--sizex", "28", "--sizey", "24", "--sizez", "32", "--time-steps", "23",
                         "--scene", "vacuum", "--parallel-grid", "--topology-sizex", "2", "--topology-sizey", "2",
                         "--topology-sizez", "2", "--time-block", "3", "--dtype", "f64"],
    # physics over ranks (split half steps, face ghosts after every half step): rank borders across the CPML
    # slabs, the TF/SF faces (oblique incidence) and a dielectric sphere
    "f32_cpml_tfsf_2x2x1": ["--3d", "--sizex", "40", "--sizey", "36", "--sizez", "32", "--time-steps", "23",
                            "--scene", "vacuum", "--use-pml", "--pml-type", "cpml", "--pml-sizex", "6",
                            "--pml-sizey", "5", "--pml-sizez", "4", "--use-tfsf", "--tfsf-sizex", "10",
                            "--tfsf-sizey", "9", "--tfsf-sizez", "8", "--angle-teta", "60", "--angle-phi", "20",
                            "--angle-psi", "30", "--parallel-grid", "--topology-sizex", "2", "--topology-sizey", "2",
                            "--dtype", "f32"],
    "f64_cpml_tfsf_sphere_2x1x2": ["--3d", "--sizex", "36", "--sizey", "32", "--sizez", "40", "--time-steps", "23",
                                   "--scene", "sphere", "--sphere-center-x", "17", "--sphere-center-y", "15",
                                   "--sphere-center-z", "21", "--sphere-radius", "5", "--sphere-eps", "3",
                                   "--use-pml", "--pml-type", "cpml", "--pml-sizex", "5", "--same-size-pml",
                                   "--cpml-kappa-max", "2", "--cpml-alpha-max", "0.05", "--use-tfsf",
                                   "--tfsf-sizex", "9", "--same-size-tfsf", "--angle-teta", "50", "--angle-phi", "30",
                                   "--angle-psi", "20", "--parallel-grid", "--topology-sizex", "2",
                                   "--topology-sizez", "2", "--dtype", "f64"],
    "f32_cpml_point_3x1x1": ["--3d", "--sizex", "42", "--sizey", "30", "--sizez", "32", "--time-steps", "23",
                             "--scene", "vacuum", "--use-pml", "--pml-type", "cpml", "--pml-sizex", "6",
                             "--pml-sizey", "5", "--pml-sizez", "4", "--parallel-grid", "--topology-sizex", "3",
                             "--dtype", "f32"],
    "f64_tfsf_1x2x2": ["--3d", "--sizex", "32", "--sizey", "40", "--sizez", "48", "--time-steps", "23",
                       "--scene", "vacuum", "--use-tfsf", "--tfsf-sizex", "8", "--tfsf-sizey", "9", "--tfsf-sizez",
                       "10", "--angle-teta", "40", "--angle-phi", "25", "--angle-psi", "15", "--parallel-grid",
                       "--topology-sizey", "2", "--topology-sizez", "2", "--dtype", "f64"],
    # the UPML D/B chain and dispersive spheres over ranks: the chain on each rank's part of the PML slabs and
    # the sphere's box (region-local levels), a sphere across two rank borders, a Lorentz sphere with TF/SF
    "f64_upml_tfsf_2x2x1": ["--3d", "--sizex", "36", "--sizey", "32", "--sizez", "40", "--time-steps", "23",
                            "--scene", "vacuum", "--use-pml", "--pml-sizex", "5", "--pml-sizey", "4", "--pml-sizez",
                            "6", "--use-tfsf", "--tfsf-sizex", "9", "--tfsf-sizey", "8", "--tfsf-sizez", "10",
                            "--angle-teta", "60", "--angle-phi", "20", "--angle-psi", "30", "--parallel-grid",
                            "--topology-sizex", "2", "--topology-sizey", "2", "--dtype", "f64"],
    "f32_drude_upml_2x1x2": ["--3d", "--sizex", "40", "--sizey", "36", "--sizez", "32", "--time-steps", "23",
                             "--scene", "drude-sphere", "--use-metamaterials", "--use-pml", "--pml-sizex", "5",
                             "--same-size-pml", "--sphere-center-x", "20", "--sphere-center-y", "18",
                             "--sphere-center-z", "16", "--sphere-radius", "7", "--parallel-grid",
                             "--topology-sizex", "2", "--topology-sizez", "2", "--dtype", "f32"],
    "f64_lorentz_upml_tfsf_1x2x2": ["--3d", "--sizex", "40", "--same-size", "--time-steps", "23", "--scene",
                                    "drude-sphere", "--use-metamaterials", "--dispersion", "lorentz",
                                    "--lorentz-omega0", "0.7", "--use-pml", "--pml-sizex", "5", "--same-size-pml",
                                    "--sphere-center-x", "20", "--sphere-center-y", "21", "--sphere-center-z", "19",
                                    "--sphere-radius", "6", "--use-tfsf", "--tfsf-sizex", "9", "--same-size-tfsf",
                                    "--parallel-grid", "--topology-sizey", "2", "--topology-sizez", "2",
                                    "--dtype", "f64"],
    # 2D schemes over x / y rank grids (the 2D kernels, CPML slabs / UPML strips per rank)
    "f64_tmz_upml_tfsf_2x2": ["--2d", "--sizex", "60", "--sizey", "52", "--time-steps", "23", "--scene", "vacuum",
                              "--use-pml", "--pml-sizex", "6", "--pml-sizey", "5", "--use-tfsf", "--tfsf-sizex",
                              "10", "--tfsf-sizey", "9", "--angle-phi", "30", "--parallel-grid", "--topology-sizex",
                              "2", "--topology-sizey", "2", "--dtype", "f64"],
    "f32_tez_cpml_sphere_2x1": ["--2d", "--2d-mode", "tez", "--sizex", "56", "--sizey", "60", "--time-steps", "23",
                                "--scene", "sphere", "--sphere-center-x", "28", "--sphere-center-y", "30",
                                "--sphere-radius", "6", "--sphere-eps", "4", "--use-pml", "--pml-type", "cpml",
                                "--pml-sizex", "5", "--pml-sizey", "6", "--cpml-kappa-max", "2", "--cpml-alpha-max",
                                "0.05", "--parallel-grid", "--topology-sizex", "2", "--dtype", "f32"],
    "f64_tmz_upml_sphere_1x3": ["--2d", "--sizex", "64", "--sizey", "66", "--time-steps", "23", "--scene", "sphere",
                                "--sphere-center-x", "30", "--sphere-center-y", "33", "--sphere-radius", "7",
                                "--sphere-eps", "3", "--use-pml", "--pml-sizex", "5", "--pml-sizey", "6",
                                "--parallel-grid", "--topology-sizey", "3", "--dtype", "f64"],
    # 1D: x slabs (the Ez / Hy kernels per rank)
    "f64_1d_x3": ["--1d", "--sizex", "300", "--time-steps", "40", "--scene", "vacuum", "--source", "gaussian",
                  "--gaussian-width", "8", "--gaussian-delay", "30", "--parallel-grid", "--topology-sizex", "3",
                  "--dtype", "f64"],
    "f32_1d_sphere_x4": ["--1d", "--sizex", "320", "--time-steps", "40", "--scene", "sphere", "--sphere-center-x",
                         "150", "--sphere-radius", "30", "--sphere-eps", "4", "--parallel-grid", "--topology-sizex",
                         "4", "--dtype", "f32"],
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(MULTI))
def test_native_parallel_grid_matches_python(case, tmp_path, gpu):
    exe = native.executable()
    argv = MULTI[case] + ["--save-res", "--save-as-dat"]
    nd, pd = tmp_path / "native", tmp_path / "py"
    nd.mkdir()
    pd.mkdir()
    r = subprocess.run([exe] + argv + ["--output-dir", str(nd)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Parallel grid: 1" in r.stdout, r.stdout
    if any(f in argv for f in ("--use-pml", "--use-tfsf", "--use-metamaterials", "--1d", "--2d")):
        assert "split half-step kernels" in r.stdout and "face ghosts" in r.stdout, r.stdout
    else:
        assert "26-neighbour ghost boxes" in r.stdout, r.stdout
    ranks = 1
    serial = [a for a in argv if a not in ("--parallel-grid",)]
    for flag in ("--topology-sizex", "--topology-sizey", "--topology-sizez"):
        if flag in serial:
            i = serial.index(flag)
            ranks *= int(serial[i + 1])
            serial = serial[:i] + serial[i + 2:]
    assert "Number of processes: %d" % ranks in r.stdout
    i = serial.index("--dtype")
    dtype = serial[i + 1]
    serial = serial[:i] + serial[i + 2:]
    assert py_run(serial + ["--dtype", "f64", "--backend", "torch", "--device", "cpu", "--output-dir", str(pd)],
                  out=io.StringIO()) == 0
    shape, scheme = _shape(argv)
    steps = int(argv[argv.index("--time-steps") + 1])
    ndt = np.float32 if dtype == "f32" else np.float64
    for kind in "EH":
        errs = []
        for c in [c[1] for c in COMPS[scheme] if c[0] == kind]:
            name = "current[%d]_rank-0_%s%s.dat" % (steps, kind, c)
            a = np.fromfile(nd / name, dtype=ndt).astype(np.float64).reshape(shape)
            b = np.fromfile(pd / name, dtype=np.float64).reshape(shape)
            errs.append((np.abs(a - b).max(), np.abs(b).max()))
        peak = max(e[1] for e in errs)
        assert peak > 0
        tol = 1e-11 if dtype == "f64" else 2e-5
        for err, _ in errs:
            assert err <= tol * peak, (kind, err, peak)


# checkpoints written and resumed by either driver (csrc/main.cpp ckpt_save / ckpt_load, io/checkpoint.py):
# plain media, whose state is the field components; (argv, resume step, final step)
CKPT = {
    "3d_blocked_vacuum": (["--3d", "--sizex", "28", "--sizey", "20", "--sizez", "24", "--scene", "vacuum",
                           "--time-block", "3"], 7, 19),
    "3d_sphere": (["--3d", "--sizex", "32", "--same-size", "--scene", "sphere", "--sphere-center-x", "16",
                   "--sphere-center-y", "16", "--sphere-center-z", "16", "--sphere-radius", "6", "--sphere-eps", "4"],
                  6, 15),
    "2d_tmz": (["--2d", "--sizex", "60", "--sizey", "52", "--scene", "vacuum", "--time-block", "5"], 9, 23),
    "1d": (["--1d", "--sizex", "300", "--scene", "vacuum", "--source", "gaussian", "--gaussian-width", "8",
            "--gaussian-delay", "30"], 13, 40),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(CKPT))
def test_native_checkpoint_roundtrip(case, tmp_path, gpu):
    """A native checkpoint resumed by the native driver and by the Python
    driver, and the full run, end on the same fields (fp64)."""
    exe = native.executable()
    argv, k, n = CKPT[case]
    argv = argv + ["--dtype", "f64"]
    py = ["--backend", "torch", "--device", "cpu"]
    d = {x: tmp_path / x for x in ("a", "nat", "py", "full")}

    def nat(extra):
        r = subprocess.run([exe] + argv + extra, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        return r.stdout

    # periodic checkpoints every k steps (at k, 2k) and the final one; the resume takes the latest, so the
    # later ones go before resuming
    nat(["--time-steps", str(2 * k + 1), "--checkpoint-dir", str(d["a"]), "--checkpoint-step", str(k)])
    for t in (k, 2 * k, 2 * k + 1):
        side = d["a"] / ("checkpoint[%d]_rank-0.json" % t)
        assert side.exists(), t
        if t != k:
            side.unlink()
    out = nat(["--time-steps", str(n), "--load-from-file", str(d["a"]), "--checkpoint-dir", str(d["nat"])])
    assert "Number of time steps: %d (%d timed" % (n, n - k) in out, out
    assert py_run(argv + py + ["--time-steps", str(n), "--load-from-file", str(d["a"]), "--checkpoint-dir",
                               str(d["py"])], out=io.StringIO()) == 0
    assert py_run(argv + py + ["--time-steps", str(n), "--checkpoint-dir", str(d["full"])], out=io.StringIO()) == 0
    shape, scheme = _shape(argv)
    for kind in "EH":
        got = {}
        for c in COMPS[scheme]:
            if c[0] != kind:
                continue
            name = "current[%d]_rank-0_%s.dat" % (n, c)
            ref = np.fromfile(d["full"] / name, dtype=np.float64).reshape(shape)
            got[c] = [np.abs(np.fromfile(d[x] / name, dtype=np.float64).reshape(shape) - ref).max()
                      for x in ("nat", "py")] + [np.abs(ref).max()]
        peak = max(v[-1] for v in got.values())
        assert peak > 0
        for c, v in got.items():
            assert max(v[:2]) <= 1e-11 * peak, (c, v)
    # the other direction: a checkpoint the PYTHON driver wrote (indent=1 sidecar with multi-line lists,
    # __version__, origin / topology / sub_step) resumed by the native driver
    d["pyck"], d["nat2"] = tmp_path / "pyck", tmp_path / "nat2"
    assert py_run(argv + py + ["--time-steps", str(k), "--checkpoint-dir", str(d["pyck"])], out=io.StringIO()) == 0
    out = nat(["--time-steps", str(n), "--load-from-file", str(d["pyck"]), "--checkpoint-dir", str(d["nat2"])])
    assert "Number of time steps: %d (%d timed" % (n, n - k) in out, out
    # (scaled by the kind's peak, as above: a component the source never drives -- Hz of an Ez point
    # source -- holds only round-off, ~1e-20)
    for kind in "EH":
        err, peak = {}, 0.0
        for c in COMPS[scheme]:
            if c[0] != kind:
                continue
            name = "current[%d]_rank-0_%s.dat" % (n, c)
            ref = np.fromfile(d["full"] / name, dtype=np.float64).reshape(shape)
            got = np.fromfile(d["nat2"] / name, dtype=np.float64).reshape(shape)
            err[c] = np.abs(got - ref).max()
            peak = max(peak, np.abs(ref).max())
        assert peak > 0
        for c, e in err.items():
            assert e <= 1e-11 * peak, (c, e, peak)
