#!/bin/bash
# Round 5: config 3 (512^3 CPML + TF/SF) knob sweep -- steps per hybrid pass and shell streams
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
run() {
  local lab=$1; shift
  timeout -k 10 300 python -m fdtd3d_amd $C "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(grep -o '"mcells_per_s": [0-9.]*' $O/$lab.log)"
}
run base
run hb6 --hybrid-block 6
run ss4 --shell-streams 4
run ss6 --shell-streams 6
run ss2 --shell-streams 2
run base2
