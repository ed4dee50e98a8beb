"""Native C++ runtime vs its Python mirror: settings parser and topology
optimiser must agree exactly (same settings.inc table, same cost model)."""
import io
import itertools
import os
import subprocess

import pytest

from fdtd3d_amd import native
from fdtd3d_amd.parallel.topology import optimal_topology as py_topology
from fdtd3d_amd.utils.settings import Settings

ARGVS = [
    [],
    ["--3d", "--same-size", "--sizex", "64", "--time-steps", "7"],
    ["--sizex", "80", "--same-size", "--use-pml", "--pml-type", "cpml", "--cpml-kappa-max", "3.5"],
    ["--2d", "--2d-mode", "tez", "--dx", "0.001", "--wavelength", "0.03", "--courant", "0.7"],
    ["--1d", "--sizex", "1000", "--dtype", "f32", "--source", "gaussian", "--gaussian-width", "12.5"],
    ["--use-tfsf", "--tfsf-sizex", "7", "--same-size-tfsf", "--angle-teta", "30", "--angle-phi", "45",
     "--angle-psi", "10"],
    ["--use-ntff", "--ntff-sizex", "9", "--same-size-ntff", "--ntff-step", "3"],
    ["--parallel-grid", "--topology", "xy", "--topology-sizex", "2", "--same-size-topology",
     "--buffer-size", "3", "--num-cuda-gpus", "8"],
    ["--save-res", "--save-as-dat", "--save-as-bmp", "--dumper-pallete", "gray", "--output-dir", "/tmp/x"],
    ["--scene", "sphere", "--sphere-eps", "4", "--sphere-radius", "11.5", "--sphere-center-x", "20"],
    ["--use-metamaterials", "--dispersion", "lorentz", "--lorentz-omega0", "0.25", "--split-kernels"],
]


@pytest.fixture(scope="module")
def host():
    return native.load_host_library()


@pytest.mark.parametrize("argv", ARGVS, ids=range(len(ARGVS)))
def test_settings_parity(host, argv):
    st, nat = native.parse_settings(argv)
    s = Settings()
    pst = s.set_from_cmd(argv, out=io.StringIO())
    assert st == pst == 0, nat
    py = s.as_dict()
    assert set(py) <= set(nat)
    for k, v in py.items():
        if isinstance(v, float):
            assert nat[k] == pytest.approx(v, rel=1e-15), k
        else:
            assert nat[k] == v, k


def test_settings_errors(host):
    assert native.parse_settings(["--bogus"])[0] == 2
    assert native.parse_settings(["--sizex"])[0] == 1
    assert native.parse_settings(["--sizex", "abc"])[0] == 1
    assert native.parse_settings(["--help"])[0] == 3
    st, msg = native.parse_settings(["--version"])
    assert st == 3 and "0.2.2" in msg


def test_cmd_from_file(host, tmp_path):
    p = tmp_path / "cmd.txt"
    p.write_text("--sizex 33\n--same-size\n--use-pml\n")
    st, nat = native.parse_settings(["--cmd-from-file", str(p)])
    assert st == 0 and nat["sizeZ"] == 33 and nat["doUsePML"] is True
    # nested files are rejected
    q = tmp_path / "nested.txt"
    q.write_text("--cmd-from-file %s\n" % p)
    assert native.parse_settings(["--cmd-from-file", str(q)])[0] == 1


def test_topology_parity(host):
    sizes = [(1024, 1024, 1024), (100, 200, 50), (64, 64, 8), (7, 300, 300), (2, 2, 2), (1000, 1, 1)]
    axes_sets = [(0, 1, 2), (0,), (1,), (0, 1), (1, 2)]
    for size, n, axes in itertools.product(sizes, [1, 2, 3, 4, 6, 8, 12, 16], axes_sets):
        assert native.optimal_topology(size, n, axes) == py_topology(size, n, axes), (size, n, axes)


def test_native_executable_cli(host):
    exe = native.executable()
    if not os.path.exists(exe):
        pytest.skip("fdtd3d executable not built")
    r = subprocess.run([exe, "--version"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "Version" in r.stdout
    r = subprocess.run([exe, "--no-such-flag"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    r = subprocess.run([exe, "--1d", "--use-tfsf"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "python -m fdtd3d_amd" in r.stderr
    # CPML runs natively in 3D (whole 4-cell z rows, fp32 / fp64) and in 2D, the UPML in 3D and 2D, the Drude
    # chain and NTFF in 3D, parallel grids for 3D plain media, CPML, UPML, Drude spheres and TF/SF; decomposed 3D
    # CPML on z rows of a size not divisible by 4, 2D metamaterials, metamaterials outside the drude-sphere scene, amplitude
    # mode with NTFF go to the Python driver
    for argv in (["--3d", "--use-pml", "--pml-type", "cpml", "--dtype", "f64", "--sizez", "42", "--parallel-grid"],
                 ["--2d", "--use-ntff"],
                 ["--2d", "--use-pml", "--use-metamaterials"],
                 ["--3d", "--use-metamaterials", "--use-pml", "--scene", "reference"],
                 ["--3d", "--use-amp-mode", "--use-ntff"], ["--3d", "--parallel-grid", "--use-amp-mode", "--use-ntff"],
                 ["--1d", "--parallel-grid", "--use-tfsf"], ["--3d", "--complex-field-values", "--use-amp-mode"],
                 ["--3d", "--complex-field-values", "--parallel-grid"],
                 ["--3d", "--use-pml", "--use-tfsf", "--pml-sizex", "10", "--tfsf-sizex", "8"],
                 ["--3d", "--use-pml", "--pml-type", "cpml", "--dtype", "f32", "--checkpoint-dir", "/tmp/ck"],
                 ["--3d", "--parallel-grid", "--use-pml", "--pml-type", "cpml", "--checkpoint-dir", "/tmp/ck"],
                 ["--2d", "--use-tfsf", "--load-from-file", "/tmp/ck"]):
        r = subprocess.run([exe] + argv, capture_output=True, text=True, timeout=60)
        assert r.returncode == 2 and "python -m fdtd3d_amd" in r.stderr, argv


def test_cmake_configures_and_builds_host_runtime(tmp_path):
    """The CMake build (reference CMakeLists.txt counterpart) configures for
    gfx950 and builds the host runtime library; the full kernel build is the
    same compiler line as ``ops/build.py`` and runs in the GPU session."""
    import shutil
    if shutil.which("cmake") is None or not os.path.exists("/opt/rocm/llvm/bin/clang++"):
        pytest.skip("cmake / ROCm clang not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    b = str(tmp_path / "build")
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    r = subprocess.run(["cmake", "-S", root, "-B", b] + gen, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "gfx950" in open(os.path.join(b, "CMakeCache.txt")).read()
    r = subprocess.run(["cmake", "--build", b, "--target", "fdtd3d_host", "-j", "4"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert os.path.exists(os.path.join(b, "libfdtd3d_host.so"))


def test_host_runtime_under_sanitizers(tmp_path):
    """Host C++ runtime (settings parser, topology optimiser, DAT/BMP writers)
    built with AddressSanitizer + UndefinedBehaviorSanitizer and exercised by
    tests/native/host_selftest.cpp; any report aborts the run."""
    import shutil
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "fdtd3d_amd", "csrc")
    exe = str(tmp_path / "host_selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=all", "-I", csrc, os.path.join(root, "tests", "native", "host_selftest.cpp"),
           os.path.join(csrc, "host_native.cpp"), os.path.join(csrc, "settings_native.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    # verify_asan_link_order=0: the environment may preload its own library ahead of the runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "0 failed checks" in r.stdout
