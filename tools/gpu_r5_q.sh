#!/bin/bash
# Round 5: 2D hybrid shell with one launch per half step for the windows and per disjoint slab group for the
# CPML corrections -- tests and 8192^2 rates (Python vs native)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hybrid_gpu.py tests/test_hip_gpu.py tests/test_graph_gpu.py tests/test_tb2d_gpu.py -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; }
tail -1 $O/tests.log
declare -A CF
B="--2d --sizex 8192 --sizey 8192 --dtype f32 --scene vacuum --use-pml --use-tfsf --warmup-steps 10 --time-steps 160 --json"
CF[tmz_cpml]="$B --pml-type cpml"
CF[tez_cpml]="$B --pml-type cpml --2d-mode tez"
CF[tmz_upml]="$B"
for k in tmz_cpml tez_cpml tmz_upml; do
  timeout -k 10 300 python -m fdtd3d_amd ${CF[$k]} > $O/py_$k.log 2>&1 || { echo "py $k failed"; tail -3 $O/py_$k.log; }
  timeout -k 10 300 ./fdtd3d_amd/fdtd3d ${CF[$k]} > $O/nat_$k.log 2>&1 || { echo "nat $k failed"; tail -3 $O/nat_$k.log; }
  echo "$k py $(grep -o '"mcells_per_s": [0-9.]*' $O/py_$k.log) nat $(grep -o '"mcells_per_s": [0-9.]*' $O/nat_$k.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p2 -o run -- python3 -m fdtd3d_amd ${CF[tmz_cpml]} > $O/prof.log 2>&1 && cp /tmp/p2/run_kernel_stats.csv $O/py_tmz_cpml_stats.csv
echo done
