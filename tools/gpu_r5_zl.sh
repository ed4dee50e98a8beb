#!/bin/bash
# Round 5: fp64 x chunk sweep at 1024^3 with the 2x8 patch order; fp32 headline patch A/B repeated
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zl
mkdir -p $O
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py $B > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*')"
}
B="--dtype f64 --steps 12 --warmup 4 --fp64-companion off --physics-companion off"
for r in 1 2; do
  run f64_auto_$r A=1
  for x in 128 205 256 342 512; do run f64_x${x}_$r FDTD3D_TB_XCHUNK=$x; done
done
B="--steps 20 --warmup 5 --fp64-companion off --physics-companion off"
for r in 1 2 3; do run f32_base_$r A=1; run f32_p4x4_$r FDTD3D_TB_PATCH=4x4; done
