"""In-tree build of the native libraries.

* ``libfdtd3d_hip.so`` -- every HIP kernel (``csrc/*.hip``) compiled for
  gfx950 plus the C ABI the Python ops call through ctypes.  Linked against the
  HIP runtime by SONAME (``libamdhip64.so.7``), so inside a Python process it
  binds to the runtime PyTorch already loaded.
* ``libfdtd3d_host.so`` -- host-only C++ runtime pieces (settings parser,
  topology optimiser, BMP/DAT writers) shared by the standalone driver.
* ``fdtd3d`` -- the standalone native driver (``csrc/main.cpp``).

Objects are rebuilt only when a source or header is newer.  Usage::

    python -m fdtd3d_amd.ops.build [--force] [-j N]
"""

from __future__ import annotations

import argparse
import glob
import re
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from typing import List

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(CSRC, "build")
LIB_HIP = os.path.join(PKG_DIR, "libfdtd3d_hip.so")
LIB_HOST = os.path.join(PKG_DIR, "libfdtd3d_host.so")
EXE = os.path.join(PKG_DIR, "fdtd3d")

ARCH = os.environ.get("FDTD3D_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-munsafe-fp-atomics",
             "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
HOST_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]


def _headers() -> List[str]:
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.inc"))


_INCLUDE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(src: str, seen=None) -> List[str]:
    """``src`` plus the in-tree headers it includes, transitively (a change
    to the native driver's headers then rebuilds main.cpp only)."""
    seen = set() if seen is None else seen
    if src in seen:
        return []
    seen.add(src)
    out = [src]
    try:
        text = open(src).read()
    except OSError:
        return out
    for name in _INCLUDE.findall(text):
        h = os.path.join(CSRC, name)
        if os.path.exists(h):
            out += _deps(h, seen)
    return out


def _stale(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n  %s\n%s" % (" ".join(cmd), r.stdout))
    if r.stdout.strip():
        # keep compiler warnings visible but short
        sys.stderr.write(r.stdout[-4000:])


def hip_sources() -> List[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def host_sources() -> List[str]:
    return sorted(s for s in glob.glob(os.path.join(CSRC, "*.cpp")) if os.path.basename(s) != "main.cpp")


def build(force: bool = False, jobs: int = 8, verbose: bool = False, exe: bool = True,
          hip: bool = True) -> None:
    """Incremental build; ``hip=False`` builds only the host library."""
    os.makedirs(BUILD_DIR, exist_ok=True)

    def obj(src: str, hip: bool) -> str:
        o = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        if force or _stale(o, _deps(src)):
            cc = HIPCC if hip else "g++"
            flags = HIP_FLAGS if hip else HOST_FLAGS
            cmd = [cc] + flags + ["-I", CSRC, "-c", src, "-o", o]
            if not hip:
                cmd = ["g++"] + flags + ["-I", CSRC, "-c", src, "-o", o]
            if verbose:
                print(" ".join(cmd))
            _run(cmd)
        return o

    hs = hip_sources() if hip else []
    cs = host_sources()
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        hip_objs = list(ex.map(lambda s: obj(s, True), hs))
        host_objs = list(ex.map(lambda s: obj(s, False), cs))

    if hip and (force or _stale(LIB_HIP, hip_objs)):
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", LIB_HIP] + hip_objs)
    if host_objs and (force or _stale(LIB_HOST, host_objs)):
        _run(["g++", "-shared", "-fPIC", "-o", LIB_HOST] + host_objs)
    main_cpp = os.path.join(CSRC, "main.cpp")
    if hip and exe and os.path.exists(main_cpp):
        main_o = obj(main_cpp, True)
        if force or _stale(EXE, [main_o] + hip_objs + host_objs):
            _run([HIPCC, "--offload-arch=" + ARCH, "-o", EXE, main_o] + hip_objs + host_objs)


def clean() -> None:
    shutil.rmtree(BUILD_DIR, ignore_errors=True)
    for p in (LIB_HIP, LIB_HOST, EXE):
        if os.path.exists(p):
            os.remove(p)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args(argv)
    if a.clean:
        clean()
        return 0
    build(force=a.force, jobs=a.j, verbose=a.v)
    return 0


if __name__ == "__main__":
    sys.exit(main())
