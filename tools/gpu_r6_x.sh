#!/bin/bash
# Round 6 (x): the Drude pass of a hybrid pass on its own stream next to the shell steps (FDTD3D_DRUDE_SIDE=1)
# vs in order: Drude GPU tests, Drude + UPML fp32 / fp64 512^3 rates alternating, kernel-trace-free
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_drude_blk_gpu.py tests/test_hybrid_gpu.py -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
D="--3d --sizex 512 --same-size --warmup-steps 12 --time-steps 48 --json --scene drude-sphere --use-metamaterials --use-pml --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
for rep in 1 2 3; do
  for m in 1 0; do
    FDTD3D_DRUDE_SIDE=$m timeout -k 10 200 python3 -m fdtd3d_amd $D --dtype f32 > $O/du_$m.log 2>&1 || { echo "du $m failed"; tail -5 $O/du_$m.log; exit 1; }
    FDTD3D_DRUDE_SIDE=$m timeout -k 10 200 python3 -m fdtd3d_amd $D --dtype f64 > $O/du64_$m.log 2>&1 || { echo "du64 $m failed"; tail -5 $O/du64_$m.log; exit 1; }
    echo "rep $rep side=$m: drude+upml f32 $(grep -o '"mcells_per_s": [0-9.]*' $O/du_$m.log | cut -d' ' -f2)  f64 $(grep -o '"mcells_per_s": [0-9.]*' $O/du64_$m.log | cut -d' ' -f2)"
  done
done
