#!/bin/bash
# Round 5: native driver with the Drude box in the blocked passes -- parity tests and the two Drude companions
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py tests/test_drude_blk_gpu.py -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; }
tail -1 $O/tests.log
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json --scene drude-sphere --use-metamaterials $S"
for k in drude drude_upml; do
  extra=""; [ $k = drude_upml ] && extra="--use-pml"
  timeout -k 10 300 ./fdtd3d_amd/fdtd3d $C $extra > $O/nat_$k.log 2>&1 || { echo "nat $k failed"; tail -3 $O/nat_$k.log; }
  timeout -k 10 300 python -m fdtd3d_amd $C $extra > $O/py_$k.log 2>&1 || { echo "py $k failed"; tail -3 $O/py_$k.log; }
  echo "$k nat $(grep -o '"mcells_per_s": [0-9.]*' $O/nat_$k.log) py $(grep -o '"mcells_per_s": [0-9.]*' $O/py_$k.log)"
done
echo done
