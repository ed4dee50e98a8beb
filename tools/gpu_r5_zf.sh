#!/bin/bash
# Round 5: native vs Python on the physics companions after the Python shell-stream fork fix, plus kernel
# statistics of both drivers on Drude + UPML
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zf
mkdir -p $O
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
D="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json"
declare -A CF
CF[drude]="$D --scene drude-sphere --use-metamaterials $S"
CF[drude_upml]="$D --scene drude-sphere --use-metamaterials --use-pml $S"
CF[cpml_tfsf]="$D --scene vacuum --use-pml --pml-type cpml --use-tfsf"
CF[upml_tfsf]="$D --scene vacuum --use-pml --use-tfsf"
for k in drude drude_upml cpml_tfsf upml_tfsf; do
  timeout -k 10 300 ./fdtd3d_amd/fdtd3d ${CF[$k]} > $O/nat_$k.log 2>&1 || { echo "nat $k failed"; tail -3 $O/nat_$k.log; }
  timeout -k 10 300 python -m fdtd3d_amd ${CF[$k]} > $O/py_$k.log 2>&1 || { echo "py $k failed"; tail -3 $O/py_$k.log; }
  echo "$k nat $(grep -o '"mcells_per_s": [0-9.]*' $O/nat_$k.log) py $(grep -o '"mcells_per_s": [0-9.]*' $O/py_$k.log)"
done
for drv in nat py; do
  if [ $drv = nat ]; then P="./fdtd3d_amd/fdtd3d"; else P="python3 -m fdtd3d_amd"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pz_$drv -o run -- $P ${CF[drude_upml]} > $O/prof_$drv.log 2>&1 || { echo "prof $drv failed"; tail -3 $O/prof_$drv.log; continue; }
  f=$(find /tmp/pz_$drv -name 'run_kernel_stats.csv' | head -1); cp "$f" $O/stats_du_$drv.csv
done
echo done
