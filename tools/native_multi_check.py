#!/usr/bin/env python3
"""Native --parallel-grid vs the native single-rank run on variants of one
config (debug aid): max |diff| per component and where."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "fdtd3d_amd", "fdtd3d")
SHAPE = (36, 32, 40)
BASE = ["--3d", "--sizex", "36", "--sizey", "32", "--sizez", "40", "--time-steps", "23", "--save-res",
        "--save-as-dat"]
SPH = ["--scene", "sphere", "--sphere-center-x", "17", "--sphere-center-y", "15", "--sphere-center-z", "21",
       "--sphere-radius", "5", "--sphere-eps", "3"]
CPML = ["--use-pml", "--pml-type", "cpml", "--pml-sizex", "5", "--same-size-pml"]
KAP = ["--cpml-kappa-max", "2", "--cpml-alpha-max", "0.05"]
TFSF = ["--use-tfsf", "--tfsf-sizex", "9", "--same-size-tfsf", "--angle-teta", "50", "--angle-phi", "30",
        "--angle-psi", "20"]
VAC = ["--scene", "vacuum"]
UPML = ["--use-pml", "--pml-sizex", "5", "--same-size-pml"]
DRU = ["--scene", "drude-sphere", "--use-metamaterials", "--sphere-center-x", "17", "--sphere-center-y", "15",
       "--sphere-center-z", "21", "--sphere-radius", "5"]
VARIANTS = [
    ("f64 vac upml 2x1x2", VAC + UPML + ["--dtype", "f64"], (2, 1, 2)),
    ("f64 vac upml tfsf 1x2x1", VAC + UPML + TFSF + ["--dtype", "f64"], (1, 2, 1)),
    ("f64 sph upml 2x1x1", SPH + UPML + ["--dtype", "f64"], (2, 1, 1)),
    ("f64 drude upml 2x1x2", DRU + UPML + ["--dtype", "f64"], (2, 1, 2)),
    ("f64 drude 1x1x2", DRU + ["--dtype", "f64"], (1, 1, 2)),
    ("f32 drude upml 2x2x1", DRU + UPML + ["--dtype", "f32"], (2, 2, 1)),
]
VARIANTS_CPML = [
    ("f64 sph cpml kap tfsf 2x1x2", SPH + CPML + KAP + TFSF + ["--dtype", "f64"], (2, 1, 2)),
    ("f64 sph cpml kap tfsf 2x1x1", SPH + CPML + KAP + TFSF + ["--dtype", "f64"], (2, 1, 1)),
    ("f64 sph cpml kap tfsf 1x1x2", SPH + CPML + KAP + TFSF + ["--dtype", "f64"], (1, 1, 2)),
    ("f32 sph cpml kap tfsf 1x1x2", SPH + CPML + KAP + TFSF + ["--dtype", "f32"], (1, 1, 2)),
    ("f64 vac cpml 1x1x2", VAC + CPML + ["--dtype", "f64"], (1, 1, 2)),
    ("f64 vac cpml 1x2x1", VAC + CPML + ["--dtype", "f64"], (1, 2, 1)),
    ("f64 vac tfsf 1x1x2", VAC + TFSF + ["--dtype", "f64"], (1, 1, 2)),
    ("f64 sph tfsf 1x1x2", SPH + TFSF + ["--dtype", "f64"], (1, 1, 2)),
    ("f32 vac cpml 1x1x2", VAC + CPML + ["--dtype", "f32"], (1, 1, 2)),
]


def run(args, out):
    r = subprocess.run([EXE] + BASE + args + ["--output-dir", out], capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        print(r.stdout, r.stderr)
        sys.exit(1)


for name, args, topo in VARIANTS:
    with tempfile.TemporaryDirectory() as d:
        a, b = os.path.join(d, "a"), os.path.join(d, "b")
        os.mkdir(a)
        os.mkdir(b)
        run(args + ["--parallel-grid", "--topology-sizex", str(topo[0]), "--topology-sizey", str(topo[1]),
                    "--topology-sizez", str(topo[2])], a)
        run(args, b)
        dt = np.float64 if "f64" in args else np.float32
        diffs = []
        for c in ("Ex", "Ey", "Ez", "Hx", "Hy", "Hz"):
            x = np.fromfile(os.path.join(a, "current[23]_rank-0_%s.dat" % c), dtype=dt).reshape(SHAPE)
            y = np.fromfile(os.path.join(b, "current[23]_rank-0_%s.dat" % c), dtype=dt).reshape(SHAPE)
            dd = np.abs(x.astype(np.float64) - y)
            idx = np.unravel_index(np.argmax(dd), dd.shape)
            diffs.append("%s %.2e@%s/%.2e" % (c, dd.max(), tuple(int(v) for v in idx), np.abs(y).max()))
        print(name, " ".join(diffs), flush=True)
