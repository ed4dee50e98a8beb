#!/bin/bash
# Round 6 (n): native driver hybrid passes in fp64 (blocked fp64 core, Drude pass, CPML windows): the native GPU
# tests, the fp64 512^3 physics rates native vs Python, then bench.py with the fp64 physics companions
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -k "hybrid" -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 8 --time-steps 32 --json"
C3="--scene vacuum --use-pml --pml-type cpml --use-tfsf"
DR="--scene drude-sphere --use-metamaterials --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
for cfg in "c3:$C3" "dr:$DR" "du:$DR --use-pml"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 ./fdtd3d_amd/fdtd3d $B $args > $O/nat_$lab.log 2>&1 || { echo "native $lab failed"; tail -5 $O/nat_$lab.log; exit 1; }
  timeout -k 10 300 python3 -m fdtd3d_amd $B $args > $O/py_$lab.log 2>&1 || { echo "py $lab failed"; tail -5 $O/py_$lab.log; exit 1; }
  echo "f64 $lab: native $(grep -o '"mcells_per_s": [0-9.]*' $O/nat_$lab.log | cut -d' ' -f2)  python $(grep -o '"mcells_per_s": [0-9.]*' $O/py_$lab.log | cut -d' ' -f2)"
done
s=$(date +%s)
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
e=$(date +%s)
echo "bench wall $((e - s)) s"
tail -1 $O/bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('headline', d['value'], 'fp64', d['fp64']['value'])
for k, v in d['physics'].items(): print(k, v.get('value'), v.get('steps'), v.get('warmup'), v.get('error', ''))
"
