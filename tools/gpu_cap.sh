#!/bin/bash
# 1024^3 Drude sphere + UPML on ONE GPU (capacity), plus the 512^3 number after the memory diet.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/cap
mkdir -p $O
C="--3d --dtype f32 --warmup-steps 5 --json --scene drude-sphere --use-metamaterials --use-pml"
timeout -k 10 300 python -u -m fdtd3d_amd $C --sizex 512 --same-size --time-steps 60 --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128 --log-level 2 > $O/d512.log 2>&1 || { echo d512 failed; tail -20 $O/d512.log; exit 1; }
grep -E '^\{|capacity' $O/d512.log | cut -c1-400
timeout -k 10 600 python -u -m fdtd3d_amd $C --sizex 1024 --same-size --time-steps 25 --sphere-center-x 512 --sphere-center-y 512 --sphere-center-z 512 --sphere-radius 256 --log-level 2 > $O/d1024.log 2>&1 || { echo d1024 failed; tail -20 $O/d1024.log; exit 1; }
grep -E '^\{|capacity|Throughput|Total time' $O/d1024.log | cut -c1-400
