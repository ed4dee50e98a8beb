#!/bin/bash
# HIP-graph replay (--use-hip-graph) of stepped PML + TF/SF runs vs eager / hybrid.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python -m fdtd3d_amd --scene vacuum --use-pml --use-tfsf --json "$@" > gpurun_out/gp.log 2>&1 || { tail -5 gpurun_out/gp.log; exit 1; }
  echo "[$*] $(grep -o '"mcells_per_s": [0-9.]*' gpurun_out/gp.log)"
}
D2="--2d --sizex 8192 --sizey 8192 --time-steps 250 --warmup-steps 70"
run $D2 --dtype f32 --use-hip-graph
run $D2 --dtype f32 --use-hip-graph --pml-type cpml
run $D2 --dtype f64 --use-hip-graph
D3="--3d --sizex 512 --same-size --time-steps 190 --warmup-steps 70"
run $D3 --dtype f32 --use-hip-graph
run $D3 --dtype f32 --use-hip-graph --pml-type cpml
