#!/bin/bash
# Round 5: slot-based in-kernel TF/SF (VGPR-lane metadata, per-trip g preload): tests, whole-grid cost,
# hybrid CPML / UPML + TF/SF with the faces in the core vs the shell
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tfsf_tb_gpu.py tests/test_hybrid_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json --scene vacuum"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
for T in 4 5; do
  run plain_T$T --time-block $T || exit 1
  run tfsf_T$T --use-tfsf --time-block $T || exit 1
  FDTD3D_TF_EXP=1 run tfsf_T${T}_nosets --use-tfsf --time-block $T || exit 1
  FDTD3D_TF_EXP=3 run tfsf_T${T}_yz --use-tfsf --time-block $T || exit 1
done
for hb in 4 5; do
  run cpml_tfsf_hb$hb --use-pml --pml-type cpml --use-tfsf --hybrid-block $hb || exit 1
  run upml_tfsf_hb$hb --use-pml --use-tfsf --hybrid-block $hb || exit 1
done
run cpml_tfsf_shell --use-pml --pml-type cpml --use-tfsf --hybrid-tfsf shell || exit 1
run upml_tfsf_shell --use-pml --use-tfsf --hybrid-tfsf shell || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_cpml_tfsf -o run -- python3 -m fdtd3d_amd $C --use-pml --pml-type cpml --use-tfsf --hybrid-block 4 > $O/prof_cpml_tfsf.log 2>&1 || echo "prof failed"
echo done
