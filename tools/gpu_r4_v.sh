#!/bin/bash
# Round 4: 2D hybrid passes replayed from HIP graphs -- hybrid GPU tests, then 8192^2 TMz physics
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_hybrid_gpu.py tests/test_tb2d_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--2d --sizex 8192 --sizey 8192 --dtype f32 --warmup-steps 10 --time-steps 150 --scene vacuum --json"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $A "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
run cpml_tfsf --use-pml --pml-type cpml --use-tfsf || exit 1
run upml_tfsf_auto --use-pml --use-tfsf || exit 1
run upml_tfsf_h7 --use-pml --use-tfsf --hybrid-block 7 || exit 1
run upml_tfsf_h5 --use-pml --use-tfsf --hybrid-block 5 || exit 1
run cpml_tfsf_f64 --use-pml --pml-type cpml --use-tfsf --dtype f64 || exit 1
run upml_tfsf_f64 --use-pml --use-tfsf --dtype f64 || exit 1
run tez_cpml_tfsf --2d-mode tez --use-pml --pml-type cpml --use-tfsf || exit 1
echo done
