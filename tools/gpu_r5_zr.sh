#!/bin/bash
# Round 5: fp64 1024^3 x chunk 171 vs automatic, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zr
mkdir -p $O
B="--dtype f64 --steps 12 --warmup 4 --fp64-companion off --physics-companion off"
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py $B > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*')"
}
for r in 1 2 3; do run auto_$r A=1; run x171_$r FDTD3D_TB_XCHUNK=171; run x256_$r FDTD3D_TB_XCHUNK=256; done
