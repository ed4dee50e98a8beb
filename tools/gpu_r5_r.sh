#!/bin/bash
# Round 5: Drude passes -- plain launches over the core minus the Drude box side by side with the Drude launch,
# vs the plain launch over everything then the Drude launch (FDTD3D_DRUDE_OVERWRITE=1), alternating on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_drude_blk_gpu.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; }
tail -1 $O/tests.log
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json --scene drude-sphere --use-metamaterials $S"
for r in 1 2; do
  for mode in 0 1; do
    FDTD3D_DRUDE_OVERWRITE=$mode timeout -k 10 300 python -m fdtd3d_amd $C > $O/d_${mode}_$r.log 2>&1 || { echo "failed"; tail -3 $O/d_${mode}_$r.log; exit 1; }
    FDTD3D_DRUDE_OVERWRITE=$mode timeout -k 10 300 python -m fdtd3d_amd $C --use-pml > $O/u_${mode}_$r.log 2>&1 || { echo "failed"; tail -3 $O/u_${mode}_$r.log; exit 1; }
    echo "overwrite=$mode run $r drude $(grep -o '"mcells_per_s": [0-9.]*' $O/d_${mode}_$r.log) drude_upml $(grep -o '"mcells_per_s": [0-9.]*' $O/u_${mode}_$r.log)"
  done
done
