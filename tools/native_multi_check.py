#!/usr/bin/env python3
"""Native x-slab parallel grid vs the native single-rank run on variants of
one config (debug aid): max |diff| per component."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "fdtd3d_amd", "fdtd3d")
BASE = ["--3d", "--sizex", "36", "--sizey", "20", "--sizez", "24", "--time-steps", "23", "--save-res",
        "--save-as-dat"]
SPH = ["--scene", "sphere", "--sphere-center-x", "17", "--sphere-center-y", "10", "--sphere-center-z", "12",
       "--sphere-radius", "5", "--sphere-eps", "3"]
VARIANTS = [
    ("f64 vacuum 4r tb3", ["--scene", "vacuum", "--dtype", "f64", "--time-block", "3"], 4),
    ("f32 sphere 4r tb3", SPH + ["--dtype", "f32", "--time-block", "3"], 4),
    ("f64 sphere 1r tb3", SPH + ["--dtype", "f64", "--time-block", "3"], 1),
    ("f64 sphere 4r tb4", SPH + ["--dtype", "f64"], 4),
    ("f64 sphere 4r tb3", SPH + ["--dtype", "f64", "--time-block", "3"], 4),
]


def run(args, out):
    r = subprocess.run([EXE] + BASE + args + ["--output-dir", out], capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        print(r.stdout, r.stderr)
        sys.exit(1)


for name, args, ranks in VARIANTS:
    with tempfile.TemporaryDirectory() as d:
        a, b = os.path.join(d, "a"), os.path.join(d, "b")
        os.mkdir(a)
        os.mkdir(b)
        run(args + ["--parallel-grid", "--topology-sizex", str(ranks)], a)
        run(args, b)
        dt = np.float64 if "f64" in args else np.float32
        diffs = []
        for c in ("Ex", "Ey", "Ez", "Hx", "Hy", "Hz"):
            x = np.fromfile(os.path.join(a, "current[23]_rank-0_%s.dat" % c), dtype=dt).reshape(36, 20, 24)
            y = np.fromfile(os.path.join(b, "current[23]_rank-0_%s.dat" % c), dtype=dt).reshape(36, 20, 24)
            dd = np.abs(x.astype(np.float64) - y)
            idx = np.unravel_index(np.argmax(dd), dd.shape)
            diffs.append("%s %.2e@%s/%.2e" % (c, dd.max(), tuple(int(v) for v in idx), np.abs(y).max()))
        print(name, " ".join(diffs), flush=True)
