#!/bin/bash
# 2D TMz / TEz throughput: blocked kernel steps per pass (yee2d_tb.hip), fp64.
#   SIZE=16384 STEPS=600 CONFIGS="tmz:1 tmz:6 tez:6 tmz-f64:1" bash tools/gpu_2d.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SIZE=${SIZE:-8192}
STEPS=${STEPS:-400}
for cfg in ${CONFIGS:-tmz:1 tmz:2 tmz:4 tmz:6 tmz:8 tez:1 tez:4 tez:8 tmz-f64:1}; do
  mode=${cfg%%:*}; T=${cfg##*:}; dt=f32
  case $mode in *-f64) dt=f64; mode=${mode%-f64};; esac
  timeout -k 10 200 python -m fdtd3d_amd --2d --2d-mode $mode --sizex $SIZE --sizey $SIZE --time-steps $STEPS \
    --warmup-steps 16 --scene vacuum --json --dtype $dt --time-block $T > gpurun_out/2d.log 2>&1 \
    || { tail -5 gpurun_out/2d.log; exit 1; }
  echo "[2d $mode $dt T=$T ${SIZE}^2] $(grep -o '"mcells_per_s": [0-9.]*' gpurun_out/2d.log)"
done
