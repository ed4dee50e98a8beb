#!/bin/bash
# Round 5: config 3 stepped-shell launch shape sweep (workgroups per split launch, smallest x chunk)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5u
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -m fdtd3d_amd $C > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(grep -o '"mcells_per_s": [0-9.]*' $O/$lab.log)"
}
run base FDTD3D_SPLIT_WGS=2048
run w1024 FDTD3D_SPLIT_WGS=1024
run w4096 FDTD3D_SPLIT_WGS=4096
run w8192 FDTD3D_SPLIT_WGS=8192
run w16384 FDTD3D_SPLIT_WGS=16384
run mx1 FDTD3D_SPLIT_MINXC=1
run mx4 FDTD3D_SPLIT_MINXC=4
run mx8 FDTD3D_SPLIT_MINXC=8
run base2 FDTD3D_SPLIT_WGS=2048
