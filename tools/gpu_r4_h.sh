#!/bin/bash
# Round 4: TF/SF faces inside the blocked core (hybrid_tfsf=core) vs in the
# stepped shell, 512^3 physics configs; rocprof of the core mode
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hybrid_gpu.py tests/test_hip_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]), round(d.get("max_mem_gb",0),1))')"
}
for cfg in "cpml_tfsf:--scene vacuum --use-pml --pml-type cpml --use-tfsf" "upml_tfsf:--scene vacuum --use-pml --use-tfsf"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  run ${lab}_core5 $args --hybrid-tfsf core || exit 1
  run ${lab}_core4 $args --hybrid-tfsf core --hybrid-block 4 || exit 1
  run ${lab}_shell5 $args --hybrid-tfsf shell || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cpml -o run -- python3 -m fdtd3d_amd $C512 \
  --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-tfsf core > $O/prof_cpml.log 2>&1 || { echo "prof failed"; tail -5 $O/prof_cpml.log; exit 1; }
echo done
