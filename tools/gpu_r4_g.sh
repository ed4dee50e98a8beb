#!/bin/bash
# Round 4: loads-first CPML split kernels -- correctness, A/B shell windows
# against the previous build (exp_old/), 512^3 CPML configs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_gpu.py tests/test_hybrid_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u tools/cpml_window_bench.py > $O/shell_new.log 2>&1 || { echo "new bench failed"; tail -5 $O/shell_new.log; exit 1; }
FDTD3D_HIP_LIB=$PWD/exp_old/libfdtd3d_hip.so timeout -k 10 200 python -u tools/cpml_window_bench.py > $O/shell_old.log 2>&1 || { echo "old bench failed"; tail -5 $O/shell_old.log; exit 1; }
echo "== new"; cat $O/shell_new.log; echo "== old"; cat $O/shell_old.log
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]), round(d.get("max_mem_gb",0),1))')"
}
run cpml_tfsf --scene vacuum --use-pml --pml-type cpml --use-tfsf || exit 1
run cpml_point --scene vacuum --use-pml --pml-type cpml || exit 1
echo done
