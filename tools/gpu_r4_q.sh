#!/bin/bash
# Round 4: steps per hybrid pass (3 / 4 / 5 / 6) on the 512^3 physics configs (shell on 3 streams)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 70 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
for cfg in "cpml_tfsf:--scene vacuum --use-pml --pml-type cpml --use-tfsf" "upml_tfsf:--scene vacuum --use-pml --use-tfsf" "drude:--scene drude-sphere --use-metamaterials --use-pml $SPH" "cpml_point:--scene vacuum --use-pml --pml-type cpml"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  for T in 3 4 5 6; do run ${lab}_T$T $args --hybrid-block $T || exit 1; done
done
echo done
