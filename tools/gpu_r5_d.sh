#!/bin/bash
# Round 5: kernel times of the TF/SF variant (rocprofv3 kernel trace): plain vs all sets vs no sets vs y/z only,
# 512^3 fp32, T = 5, whole grid (no PML)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json --scene vacuum --time-block 5"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$lab -o run -- python3 -m fdtd3d_amd $C "$@" > $O/prof_$lab.log 2>&1 || { echo "prof $lab failed"; tail -3 $O/prof_$lab.log; return 1; }
}
run plain || exit 1
FDTD3D_TF_EXP=0 run tfsf --use-tfsf || exit 1
FDTD3D_TF_EXP=1 run tfsf_nosets --use-tfsf || exit 1
FDTD3D_TF_EXP=3 run tfsf_yz --use-tfsf || exit 1
FDTD3D_TF_EXP=2 run tfsf_x --use-tfsf || exit 1
echo done
