#!/bin/bash
# Blocked CPML / TF-SF shell (hybrid plan v3): GPU tests, then 512^3 configs (auto vs stepped shell).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hybrid_gpu.py -x -v --timeout 120 --timeout-method thread -k "hybrid3 or at_scale or cpml" > $O/tests.log 2>&1
rc=$?
tail -25 $O/tests.log
[ $rc -ne 0 ] && exit $rc
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json"
run() {
  local lab=$1; shift
  timeout -k 10 240 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | cut -c1-200)"
}
for T in ${TS:-5 4}; do
  run cpml_tfsf_T$T --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-block $T || exit 1
  run cpml_point_T$T --scene vacuum --use-pml --pml-type cpml --hybrid-block $T || exit 1
done
run cpml_tfsf_stepped --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-shell stepped || exit 1
