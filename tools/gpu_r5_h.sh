#!/bin/bash
# Round 5: blocked Drude pass -- tile shape A/B (8 waves x 2 rows vs 16 x 1) at T = 4 / 5
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json --scene drude-sphere --use-metamaterials $S"
run() {
  local lab=$1; shift
  timeout -k 10 300 python -m fdtd3d_amd $C "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
timeout -k 10 300 python -u -m pytest tests/test_drude_blk_gpu.py -q --timeout 200 --timeout-method thread > $O/tests0.log 2>&1 || { echo "tests shape0 failed"; tail -5 $O/tests0.log; }
FDTD3D_TB_DR_SHAPE=1 timeout -k 10 300 python -u -m pytest tests/test_drude_blk_gpu.py -q --timeout 200 --timeout-method thread > $O/tests1.log 2>&1 || { echo "tests shape1 failed"; tail -5 $O/tests1.log; }
tail -1 $O/tests0.log; tail -1 $O/tests1.log
for sh in 0 1; do
  for T in 4 5; do
    FDTD3D_TB_DR_SHAPE=$sh run drude_s${sh}_T$T --time-block $T || exit 1
    FDTD3D_TB_DR_SHAPE=$sh run drude_upml_s${sh}_T$T --use-pml --hybrid-block $T || exit 1
  done
done
echo done
