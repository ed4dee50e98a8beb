#!/bin/bash
# Round 5: physics configs after the shell-stream fork fix -- hybrid T, shell streams, in-core TF/SF with CPML
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ze
mkdir -p $O
B="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json"
C3="$B --scene vacuum --use-pml --pml-type cpml --use-tfsf"
DU="$B --scene drude-sphere --use-metamaterials --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128 --use-pml"
UT="$B --scene vacuum --use-pml --use-tfsf"
run() {
  local lab=$1; shift
  timeout -k 10 300 python -m fdtd3d_amd "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(grep -o '"mcells_per_s": [0-9.]*' $O/$lab.log)"
}
if [ "${SWEEP:-1}" = 2 ]; then
  for r in 1 2; do
    for ss in 3 4 6; do run c3_ss${ss}_$r $C3 --shell-streams $ss; done
    for ss in 3 4 6; do run du_ss${ss}_$r $DU --shell-streams $ss; done
    for ss in 3 4; do run ut_ss${ss}_$r $UT --shell-streams $ss; done
  done
  exit 0
fi
run c3_base $C3
run c3_ss1 $C3 --shell-streams 1
run c3_ss4 $C3 --shell-streams 4
run c3_T4 $C3 --hybrid-block 4
run c3_T6 $C3 --hybrid-block 6
run c3_core $C3 --hybrid-tfsf core
run du_base $DU
run du_ss1 $DU --shell-streams 1
run du_T4 $DU --hybrid-block 4
run ut_base $UT
run ut_ss1 $UT --shell-streams 1
run c3_base2 $C3
