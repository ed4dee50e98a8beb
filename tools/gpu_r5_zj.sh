#!/bin/bash
# Round 5: fp64 blocked kernel knobs at 1024^3 (steps per pass, XCD patch order, tile form)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zj
mkdir -p $O
B="--dtype f64 --steps 12 --warmup 4 --fp64-companion off --physics-companion off"
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py $B $EXTRA > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*')"
}
if [ "${SWEEP:-1}" = 2 ]; then
  for r in 1 2; do
    run base_$r A=1
    for p in 2x8 1x8 2x4 2x16 4x8 3x8 1x16; do run p${p}_$r FDTD3D_TB64_PATCH=$p; done
  done
  exit 0
fi
run base A=1
run p4x4 FDTD3D_TB64_PATCH=4x4
run p8x2 FDTD3D_TB64_PATCH=8x2
run p2x8 FDTD3D_TB64_PATCH=2x8
run half0 FDTD3D_TB64_HALF=0
EXTRA="--time-block 3" run T3 A=1
EXTRA="--time-block 5" run T5 A=1
run base2 A=1
