#!/bin/bash
# steady-state kernel tables of the 512^3 UPML + TF/SF and Drude + UPML configs (stepped shell)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
prof() {
  local lab=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$lab -o run -- python3 -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | cut -c1-90)"
  python3 tools/prof_summary.py $(find $O/$lab -name '*results.db' | head -1) --marker k_tb3d --passes 8 > $O/$lab.md 2>&1
  head -14 $O/$lab.md | cut -c1-140
  rm -rf $O/$lab
}
prof upml_tfsf --scene vacuum --use-pml --use-tfsf || exit 1
prof drude_upml --scene drude-sphere --use-metamaterials --use-pml $SPH || exit 1
