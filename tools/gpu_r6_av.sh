#!/bin/bash
# Round 6 (av): native driver shell streams 2 vs 3 (512^3 fp32 CPML + TF/SF, UPML + TF/SF; alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6av
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
U="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 8 --time-steps 64 --json --scene drude-sphere --use-metamaterials --use-pml --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
for cfg in C U; do
  for r in 1 2; do
    for n in 3 2; do
      timeout -k 10 200 fdtd3d_amd/fdtd3d ${!cfg} --shell-streams $n > $O/${cfg}_${n}_$r.log 2>&1 || { echo "$cfg $n failed"; tail -5 $O/${cfg}_${n}_$r.log; exit 1; }
      echo "$cfg streams=$n $(grep Throughput $O/${cfg}_${n}_$r.log)"
    done
  done
done
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -q -k "hybrid" --timeout 120 --timeout-method thread > $O/t.log 2>&1; grep -E "passed|failed" $O/t.log | tail -1
