#!/bin/bash
# Kernel-trace profiles of the non-vacuum 512^3 configs (python -m fdtd3d_amd).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/prof_cfg
mkdir -p $O
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60"
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run -- python3 -m fdtd3d_amd $C512 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; return 1; }
}
run cpml --scene vacuum --use-pml --pml-type cpml --use-tfsf &&
run upml --scene vacuum --use-pml --use-tfsf &&
run drude --scene drude-sphere --use-metamaterials --use-pml --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128
echo rc=$?
