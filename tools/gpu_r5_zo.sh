#!/bin/bash
# Round 5: fp32 headline x chunk sweep at 1024^3, T = 5 (alternating with the automatic 256-plane chunks)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zo
mkdir -p $O
B="--steps 20 --warmup 5 --fp64-companion off --physics-companion off"
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py $B > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*')"
}
for r in 1 2; do
  for x in 0 128 171 205 342; do run x${x}_$r FDTD3D_TB_XCHUNK=$x; done
done
