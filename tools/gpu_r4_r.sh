#!/bin/bash
# Round 4: x planes per workgroup of the split shell kernels (FDTD3D_SPLIT_WGS / _MINXC) on the 512^3 physics
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
for v in "2048 2" "1024 2" "1024 4" "512 4" "4096 2" "2048 4" "8192 1"; do
  set -- $v
  export FDTD3D_SPLIT_WGS=$1 FDTD3D_SPLIT_MINXC=$2
  run cpml_tfsf_$1_$2 --scene vacuum --use-pml --pml-type cpml --use-tfsf || exit 1
  run upml_tfsf_$1_$2 --scene vacuum --use-pml --use-tfsf || exit 1
  run drude_$1_$2 --scene drude-sphere --use-metamaterials --use-pml $SPH || exit 1
done
echo done
