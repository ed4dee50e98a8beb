#!/bin/bash
# Single-pass vs stepped shell on the 512^3 physics configs (+ shell / hybrid GPU tests).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_shell_gpu.py tests/test_hybrid_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local lab=$1; shift
  timeout -k 10 240 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | cut -c1-160)"
}
for mode in ${MODES:-auto stepped}; do
  run cpml_tfsf_$mode --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-shell $mode || exit 1
  run upml_tfsf_$mode --scene vacuum --use-pml --use-tfsf --hybrid-shell $mode || exit 1
  run drude_$mode --scene drude-sphere --use-metamaterials --use-pml $SPH --hybrid-shell $mode || exit 1
  run cpml_point_$mode --scene vacuum --use-pml --pml-type cpml --hybrid-shell $mode || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m fdtd3d_amd $C512 --scene vacuum --use-pml --pml-type cpml --use-tfsf > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
python3 tools/prof_summary.py $(find $O/prof -name '*results.db' | head -1) --marker k_tb3d --passes 8 > $O/cpml_steady.md 2>&1
rm -rf $O/prof
head -24 $O/cpml_steady.md
