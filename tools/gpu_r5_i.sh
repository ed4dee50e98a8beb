#!/bin/bash
# Round 5: Python vs native driver on the same configs (rates + per-kernel stats) -- where the plans differ
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
declare -A CF
CF[tmz_cpml]="--2d --sizex 8192 --sizey 8192 --dtype f32 --scene vacuum --use-pml --pml-type cpml --use-tfsf --warmup-steps 10 --time-steps 160"
CF[cpml_tfsf]="--3d --sizex 512 --same-size --dtype f32 --scene vacuum --use-pml --pml-type cpml --use-tfsf --warmup-steps 45 --time-steps 75"
CF[drude_upml]="--3d --sizex 512 --same-size --dtype f32 --scene drude-sphere --use-metamaterials --use-pml $S --warmup-steps 45 --time-steps 75"
for k in tmz_cpml cpml_tfsf drude_upml; do
  timeout -k 10 300 python -m fdtd3d_amd ${CF[$k]} --json > $O/py_$k.log 2>&1 || { echo "py $k failed"; tail -3 $O/py_$k.log; }
  timeout -k 10 300 ./fdtd3d_amd/fdtd3d ${CF[$k]} --json > $O/nat_$k.log 2>&1 || { echo "nat $k failed"; tail -3 $O/nat_$k.log; }
  echo "$k py $(grep -o '"mcells_per_s": [0-9.]*' $O/py_$k.log) nat $(grep -o '"mcells_per_s": [0-9.]*' $O/nat_$k.log)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pp_$k -o run -- python3 -m fdtd3d_amd ${CF[$k]} > $O/prof_py_$k.log 2>&1 && cp /tmp/pp_$k/run_kernel_stats.csv $O/py_${k}_stats.csv
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pn_$k -o run -- ./fdtd3d_amd/fdtd3d ${CF[$k]} > $O/prof_nat_$k.log 2>&1 && cp /tmp/pn_$k/run_kernel_stats.csv $O/nat_${k}_stats.csv
done
echo done
