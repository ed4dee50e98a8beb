#!/bin/bash
# 2D TMz / TEz with PML + TF/SF (8192^2): stepped vs hybrid blocking.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python -m fdtd3d_amd --2d --sizex 8192 --sizey 8192 --time-steps 210 --warmup-steps 14 --scene vacuum \
    --use-pml --use-tfsf --json "$@" > gpurun_out/2dp.log 2>&1 || { tail -5 gpurun_out/2dp.log; exit 1; }
  echo "[2d pml+tfsf $*] $(grep -o '"mcells_per_s": [0-9.]*' gpurun_out/2dp.log)"
}
run --dtype f32 --hybrid-block 1
run --dtype f32
run --dtype f32 --hybrid-block 4
run --dtype f32 --pml-type cpml --hybrid-block 1
run --dtype f32 --pml-type cpml
run --dtype f64 --hybrid-block 1
run --dtype f64
run --dtype f32 --2d-mode tez
