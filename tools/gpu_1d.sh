#!/bin/bash
# 1D throughput (BASELINE config 1: 10000 cells, Gaussian pulse): resident
# kernel (default) vs HIP graphs of the per-step kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {
  timeout -k 10 120 python -m fdtd3d_amd --1d --sizex ${N:-10000} --scene vacuum --source gaussian --json "$@" > gpurun_out/1d.log 2>&1 \
    || { tail -5 gpurun_out/1d.log; exit 1; }
  echo "[1d $*] $(grep -o '"mcells_per_s": [0-9.]*' gpurun_out/1d.log)"
}
run --dtype f64 --time-steps 2000 --warmup-steps 10
run --dtype f64 --time-steps 100000 --warmup-steps 10
run --dtype f32 --time-steps 100000 --warmup-steps 10
run --dtype f64 --time-steps 2000 --warmup-steps 60 --use-hip-graph --split-kernels
