#!/bin/bash
# Round 4: hybrid plan variants on the 512^3 physics configs (band / history, TF/SF in core / shell, T 4 / 5)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]), round(d.get("max_mem_gb",0),1))')"
}
for cfg in "cpml_tfsf:--scene vacuum --use-pml --pml-type cpml --use-tfsf" "cpml_point:--scene vacuum --use-pml --pml-type cpml" "upml_tfsf:--scene vacuum --use-pml --use-tfsf" "drude:--scene drude-sphere --use-metamaterials --use-pml $SPH"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  FDTD3D_HYBRID_BAND=1 run ${lab}_band5 $args || exit 1
  FDTD3D_HYBRID_BAND=1 run ${lab}_band4 $args --hybrid-block 4 || exit 1
  FDTD3D_HIST_TFSF_CORE=0 run ${lab}_hist5_shell $args || exit 1
  FDTD3D_HIST_TFSF_CORE=0 run ${lab}_hist4_shell $args --hybrid-block 4 || exit 1
  run ${lab}_hist4_core $args --hybrid-block 4 || exit 1
done
