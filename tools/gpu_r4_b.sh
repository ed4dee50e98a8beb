#!/bin/bash
# Round 4: history shell + new TF/SF path -- GPU tests, kernel micro-bench, physics configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hybrid_gpu.py tests/test_tfsf_tb_gpu.py tests/test_tb_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $O/tests.log | head -30; exit $rc; }
timeout -k 10 180 python -u tools/mr_bench.py --T 5 > $O/mr5.log 2>&1 || { tail -5 $O/mr5.log; exit 1; }
grep -v amdgpu.ids $O/mr5.log
timeout -k 10 180 python -u tools/mr_bench.py --T 4 > $O/mr4.log 2>&1 || { tail -5 $O/mr4.log; exit 1; }
grep -v amdgpu.ids $O/mr4.log
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local lab=$1; shift
  timeout -k 10 240 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | cut -c1-120)"
}
run cpml_tfsf --scene vacuum --use-pml --pml-type cpml --use-tfsf --profile-phases || exit 1
grep -A12 "Phase timings" $O/cpml_tfsf.log
run cpml_point --scene vacuum --use-pml --pml-type cpml || exit 1
run upml_tfsf --scene vacuum --use-pml --use-tfsf || exit 1
run drude --scene drude-sphere --use-metamaterials --use-pml $SPH || exit 1
run tfsf --scene vacuum --use-tfsf || exit 1
