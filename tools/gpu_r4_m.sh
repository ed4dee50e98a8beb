#!/bin/bash
# Round 4: hybrid shell window launches spread over several streams -- hybrid GPU tests (default 3 streams),
# then the 512^3 physics configs at 1 / 2 / 3 / 4 streams
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_hybrid_gpu.py tests/test_tfsf_tb_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
for cfg in "cpml_tfsf:--scene vacuum --use-pml --pml-type cpml --use-tfsf" "upml_tfsf:--scene vacuum --use-pml --use-tfsf" "drude:--scene drude-sphere --use-metamaterials --use-pml $SPH"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  for n in 1 2 3 4; do run ${lab}_s$n $args --shell-streams $n || exit 1; done
done
echo done
