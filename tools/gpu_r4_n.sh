#!/bin/bash
# Round 4: overlapped hybrid passes (shell in a scratch set next to the core) -- hybrid GPU tests, then the
# 512^3 physics configs with the overlap on / off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_hybrid_gpu.py tests/test_tfsf_tb_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]), round(d.get("max_mem_gb",0),1))')"
}
for cfg in "cpml_tfsf:--scene vacuum --use-pml --pml-type cpml --use-tfsf" "upml_tfsf:--scene vacuum --use-pml --use-tfsf" "drude:--scene drude-sphere --use-metamaterials --use-pml $SPH" "cpml_point:--scene vacuum --use-pml --pml-type cpml"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  run ${lab}_ov $args || exit 1
  run ${lab}_seq $args --shell-overlap off || exit 1
  run ${lab}_ov_s2 $args --shell-streams 2 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cpml -o run -- python3 -m fdtd3d_amd $C512 \
  --scene vacuum --use-pml --pml-type cpml --use-tfsf > $O/prof_cpml.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
