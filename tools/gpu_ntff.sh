#!/bin/bash
# --use-ntff keeps the blocked passes: 512^3 vacuum, 210 steps (NTFF at steps 1, 101, 201), with and without NTFF.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
C="-m fdtd3d_amd --3d --sizex 512 --same-size --dtype f32 --scene vacuum --warmup-steps 10 --time-steps 210 --json"
for extra in "" "--use-ntff --ntff-sizex 15 --ntff-sizey 15 --ntff-sizez 15"; do
  timeout -k 10 300 python3 $C $extra > gpurun_out/ntff.log 2>&1 || { tail -5 gpurun_out/ntff.log; exit 1; }
  echo "[$extra] $(grep '^{' gpurun_out/ntff.log | cut -c1-200)"
done
