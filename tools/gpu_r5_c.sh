#!/bin/bash
# Round 5: where the in-kernel TF/SF variant's cost comes from (512^3 fp32 whole grid, no PML).
# FDTD3D_TF_EXP: 0 all sets, 1 no sets (variant structure only), 2 x-face sets only, 3 y/z-face sets only;
# FDTD3D_TB_XCHUNK: x planes per workgroup (many rounds average the face tiles' extra time).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json --scene vacuum"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
for T in 4 5; do
  run plain_T$T --time-block $T || exit 1
  for e in 0 1 2 3; do
    FDTD3D_TF_EXP=$e run tfsf_T${T}_exp$e --use-tfsf --time-block $T || exit 1
  done
  FDTD3D_TB_XCHUNK=128 run plain_T${T}_xc128 --time-block $T || exit 1
  FDTD3D_TB_XCHUNK=128 run tfsf_T${T}_xc128 --use-tfsf --time-block $T || exit 1
done

C2="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for hb in 4 5; do
  timeout -k 10 200 python -m fdtd3d_amd $C2 --hybrid-block $hb > $O/cpml_tfsf_hb$hb.log 2>&1 || { echo "cpml_tfsf hb$hb failed"; tail -3 $O/cpml_tfsf_hb$hb.log; exit 1; }
  echo "cpml_tfsf_hb$hb $(grep '^{' $O/cpml_tfsf_hb$hb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
  timeout -k 10 200 python -m fdtd3d_amd $C2 --hybrid-block $hb --hybrid-tfsf shell > $O/cpml_tfsf_shell_hb$hb.log 2>&1 || exit 1
  echo "cpml_tfsf_shell_hb$hb $(grep '^{' $O/cpml_tfsf_shell_hb$hb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
done
timeout -k 10 600 python -u -m pytest tests/test_tfsf_tb_gpu.py tests/test_hybrid_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo done
