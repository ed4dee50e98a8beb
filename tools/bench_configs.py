#!/usr/bin/env python3
"""Run every BASELINE.json config through the driver and tabulate Mcells/s.

    python tools/bench_configs.py [--only NAME ...] [--out gpurun_out/configs.md]

Each config runs as its own ``python -m fdtd3d_amd ... --json`` process under
a time limit; the JSON summary line is parsed.  The 8-GPU 2048x1024x1024
config is driven by ``bench.py`` under torchrun on an 8-GPU node and is not
launched here.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

C512 = ["--3d", "--sizex", "512", "--same-size", "--dtype", "f32", "--warmup-steps", "10"]
CONFIGS = [
    ("1d-cpu", "1D vacuum, 10000 cells, Gaussian pulse, torch CPU path",
     ["--1d", "--sizex", "10000", "--time-steps", "2000", "--scene", "vacuum", "--source", "gaussian",
      "--backend", "torch", "--device", "cpu", "--dtype", "f64"]),
    ("1d-hip", "1D vacuum, 10000 cells, Gaussian pulse, HIP",
     ["--1d", "--sizex", "10000", "--time-steps", "2000", "--scene", "vacuum", "--source", "gaussian",
      "--dtype", "f64", "--warmup-steps", "10"]),
    ("1d-hip-long", "1D vacuum, 10000 cells, Gaussian pulse, HIP, 100 000 steps (one resident launch)",
     ["--1d", "--sizex", "10000", "--time-steps", "100000", "--scene", "vacuum", "--source", "gaussian",
      "--dtype", "f64", "--warmup-steps", "10"]),
    ("3d-512-vacuum", "3D vacuum 512^3, point dipole, fp32",
     C512 + ["--time-steps", "200", "--scene", "vacuum"]),
    ("1d-hip-graph", "1D vacuum, 10000 cells, Gaussian pulse, HIP graphs of the per-step kernels",
     ["--1d", "--sizex", "10000", "--time-steps", "2000", "--scene", "vacuum", "--source", "gaussian",
      "--dtype", "f64", "--warmup-steps", "60", "--use-hip-graph", "--split-kernels"]),
    ("3d-512-vacuum-tb4", "3D vacuum 512^3, point dipole, fp32, 4 steps per pass",
     C512 + ["--time-steps", "210", "--scene", "vacuum", "--time-block", "4"]),
    ("3d-512-cpml-tfsf", "3D 512^3, CPML (10 cells) + TF/SF plane wave, fp32",
     C512 + ["--time-steps", "100", "--scene", "vacuum", "--use-pml", "--pml-type", "cpml", "--use-tfsf"]),
    ("3d-512-upml-tfsf", "3D 512^3, UPML (10 cells, reference D/B form) + TF/SF, fp32",
     C512 + ["--time-steps", "100", "--scene", "vacuum", "--use-pml", "--use-tfsf"]),
    ("3d-512-drude", "3D 512^3 Drude sphere (r=128) in vacuum, UPML, fp32",
     C512 + ["--time-steps", "100", "--scene", "drude-sphere", "--use-metamaterials", "--use-pml",
             "--sphere-center-x", "256", "--sphere-center-y", "256", "--sphere-center-z", "256",
             "--sphere-radius", "128"]),
    ("3d-512-drude-nopml", "3D 512^3 Drude sphere (r=128) in vacuum, no PML (BASELINE config 4 as named), fp32",
     C512 + ["--time-steps", "100", "--scene", "drude-sphere", "--use-metamaterials",
             "--sphere-center-x", "256", "--sphere-center-y", "256", "--sphere-center-z", "256",
             "--sphere-radius", "128"]),
    ("3d-512-sphere", "3D 512^3 dielectric sphere (eps=4, r=128), fp32",
     C512 + ["--time-steps", "200", "--scene", "sphere", "--sphere-eps", "4",
             "--sphere-center-x", "256", "--sphere-center-y", "256", "--sphere-center-z", "256",
             "--sphere-radius", "128"]),
    ("2d-tmz-16k", "2D TMz 16384^2 vacuum, fp32 (blocked, 7 steps per pass)",
     ["--2d", "--sizex", "16384", "--sizey", "16384", "--time-steps", "600", "--warmup-steps", "14", "--scene",
      "vacuum", "--dtype", "f32"]),
    ("2d-tmz-16k-f64", "2D TMz 16384^2 vacuum, fp64 (blocked, 7 steps per pass)",
     ["--2d", "--sizex", "16384", "--sizey", "16384", "--time-steps", "600", "--warmup-steps", "14", "--scene",
      "vacuum", "--dtype", "f64"]),
    ("2d-tmz-8k-upml-tfsf", "2D TMz 8192^2, UPML + TF/SF, fp32 (hybrid blocking)",
     ["--2d", "--sizex", "8192", "--sizey", "8192", "--time-steps", "210", "--warmup-steps", "14", "--scene",
      "vacuum", "--use-pml", "--use-tfsf", "--dtype", "f32"]),
    ("3d-512-cpml-point", "3D 512^3, CPML (10 cells), point dipole, fp32",
     C512 + ["--time-steps", "100", "--scene", "vacuum", "--use-pml", "--pml-type", "cpml"]),
    ("3d-512-tfsf", "3D 512^3 vacuum + TF/SF plane wave, no PML, fp32 (in-kernel TF/SF, T=4)",
     C512 + ["--time-steps", "200", "--scene", "vacuum", "--use-tfsf"]),
    ("3d-512-ntff", "3D 512^3 vacuum, point dipole, NTFF diagram every 100 steps, fp32",
     C512 + ["--time-steps", "210", "--scene", "vacuum", "--use-ntff", "--ntff-sizex", "15", "--ntff-sizey", "15",
             "--ntff-sizez", "15"]),
    ("3d-512-vacuum-f64", "3D vacuum 512^3, point dipole, fp64",
     ["--3d", "--sizex", "512", "--same-size", "--dtype", "f64", "--warmup-steps", "10", "--time-steps", "200",
      "--scene", "vacuum"]),
    ("3d-512-sphere-tb4", "3D 512^3 dielectric sphere (eps=4, r=128), fp32, 4 steps per pass",
     C512 + ["--time-steps", "210", "--scene", "sphere", "--sphere-eps", "4",
             "--sphere-center-x", "256", "--sphere-center-y", "256", "--sphere-center-z", "256",
             "--sphere-radius", "128", "--time-block", "4"]),
]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--out", default="")
    ap.add_argument("--timeout", type=int, default=300)
    a = ap.parse_args(argv)
    rows = []
    for name, desc, args in CONFIGS:
        if a.only and name not in a.only:
            continue
        cmd = [sys.executable, "-m", "fdtd3d_amd"] + args + ["--json"]
        t0 = time.time()
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=a.timeout)
        wall = time.time() - t0
        res = None
        for line in r.stdout.splitlines():
            if line.startswith("{"):
                res = json.loads(line)
        if r.returncode != 0 or res is None:
            print("%s FAILED rc=%d\n%s\n%s" % (name, r.returncode, r.stdout[-2000:], r.stderr[-2000:]))
            return 1
        res.update(name=name, desc=desc, wall=wall, args=" ".join(args))
        print(json.dumps(res), flush=True)
        rows.append(res)
    if a.out:
        with open(a.out, "w") as f:
            f.write("| config | Mcells/s | timed steps | seconds | backend | command |\n|---|---:|---:|---:|---|---|\n")
            for r in rows:
                f.write("| %s | %.1f | %d | %.3f | %s | `%s` |\n" % (r["desc"], r["mcells_per_s"], r["steps"],
                                                                  r["seconds"], r["backend"], r["args"]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
