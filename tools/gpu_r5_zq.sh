#!/bin/bash
# Round 5: x-chunk cap A/B on another box (headline only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zq
mkdir -p $O
B="--steps 20 --warmup 5 --fp64-companion off --physics-companion off"
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py $B > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*')"
}
for r in 1 2 3; do run cap192_$r A=1; run cap256_$r FDTD3D_TB_XCAP=256; done
