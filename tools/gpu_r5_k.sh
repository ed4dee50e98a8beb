#!/bin/bash
# Round 5: masked float4 stores in the plain split kernels (no lost updates next to chain launches on other
# streams) -- hybrid / native / Drude tests and the companions through both drivers
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_native_gpu.py tests/test_drude_blk_gpu.py tests/test_hybrid_gpu.py tests/test_hip_gpu.py -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; }
tail -1 $O/tests.log
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
D="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json"
declare -A CF
CF[drude]="$D --scene drude-sphere --use-metamaterials $S"
CF[drude_upml]="$D --scene drude-sphere --use-metamaterials --use-pml $S"
CF[cpml_tfsf]="$D --scene vacuum --use-pml --pml-type cpml --use-tfsf"
CF[upml_tfsf]="$D --scene vacuum --use-pml --use-tfsf"
for k in drude drude_upml cpml_tfsf upml_tfsf; do
  timeout -k 10 300 ./fdtd3d_amd/fdtd3d ${CF[$k]} > $O/nat_$k.log 2>&1 || { echo "nat $k failed"; tail -3 $O/nat_$k.log; }
  timeout -k 10 300 python -m fdtd3d_amd ${CF[$k]} > $O/py_$k.log 2>&1 || { echo "py $k failed"; tail -3 $O/py_$k.log; }
  echo "$k nat $(grep -o '"mcells_per_s": [0-9.]*' $O/nat_$k.log) py $(grep -o '"mcells_per_s": [0-9.]*' $O/py_$k.log)"
done
echo done
