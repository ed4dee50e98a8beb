#!/bin/bash
# blocked-shell CPML: correctness subset, then 512^3 rates with the scratch-load knob, + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cpml_tb_gpu.py tests/test_hybrid_gpu.py -x -q --timeout 120 --timeout-method thread -k "xyz or hybrid3" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 40 --json"
run() {
  local lab=$1; shift
  timeout -k 10 240 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | cut -c1-120)"
}
run cpml_tfsf_T5 --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-shell blocked --hybrid-block 5 || exit 1
FDTD3D_CPML_SCR_L1=1 run cpml_tfsf_T5_l1 --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-shell blocked --hybrid-block 5 || exit 1
run cpml_tfsf_T3 --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-shell blocked --hybrid-block 3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m fdtd3d_amd $C512 --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-shell blocked > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
python3 tools/prof_summary.py $(find $O/prof -name '*results.db' | head -1) > $O/prof.md 2>&1
head -8 $O/prof.md | cut -c1-150
rm -rf $O/prof
