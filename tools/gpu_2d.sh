#!/bin/bash
# 2D TMz / TEz throughput (8192^2, fp32 and fp64).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for args in "--dtype f32" "--dtype f64" "--dtype f32 --2d-mode tez" "--dtype f32 --use-hip-graph"; do
  timeout -k 10 200 python -m fdtd3d_amd --2d --sizex 8192 --sizey 8192 --time-steps 200 --warmup-steps 10 --scene vacuum --json $args > gpurun_out/2d.log 2>&1 || { tail -5 gpurun_out/2d.log; exit 1; }
  echo "[2d $args] $(grep -o '"mcells_per_s": [0-9.]*' gpurun_out/2d.log)"
done
