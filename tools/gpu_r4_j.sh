#!/bin/bash
# Round 4: native driver hybrid passes (CPML + TF/SF / point source) --
# parity tests against the Python driver, 512^3 rates of both drivers
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_native_gpu.py -x -q -k "cpml" --timeout 240 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C512="--3d --sizex 512 --same-size --dtype f32 --time-steps 60 --json"
for cfg in "cpml_tfsf:--scene vacuum --use-pml --pml-type cpml --use-tfsf" "cpml_point:--scene vacuum --use-pml --pml-type cpml"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 ./fdtd3d_amd/fdtd3d $C512 --warmup-steps 10 $args > $O/native_$lab.log 2>&1 || { echo "native $lab failed"; tail -3 $O/native_$lab.log; exit 1; }
  echo "native $lab: $(grep -E 'Backend|Throughput' $O/native_$lab.log | tr '\n' ' ')"
  timeout -k 10 200 ./fdtd3d_amd/fdtd3d $C512 --warmup-steps 10 $args --hybrid-block 1 > $O/native_${lab}_stepped.log 2>&1 || { echo "native stepped $lab failed"; exit 1; }
  echo "native $lab stepped: $(grep -E 'Throughput' $O/native_${lab}_stepped.log)"
done
echo done
