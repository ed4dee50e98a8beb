#!/bin/bash
# Round 4: shell copies on the shell streams -- hybrid GPU tests, 512^3 physics rates
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_hybrid_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 70 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
for cfg in "cpml_tfsf:--scene vacuum --use-pml --pml-type cpml --use-tfsf" "upml_tfsf:--scene vacuum --use-pml --use-tfsf" "drude_upml:--scene drude-sphere --use-metamaterials --use-pml $SPH" "drude:--scene drude-sphere --use-metamaterials $SPH"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  run ${lab} $args || exit 1
  run ${lab}_s1 $args --shell-streams 1 || exit 1
done
echo done
