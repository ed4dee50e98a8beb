#!/bin/bash
# Round 6 (as): shell streams 2 / 3 / 4 on the other hybrid configs (alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6as
mkdir -p $O
D="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 8 --time-steps 64 --json --scene drude-sphere --use-metamaterials --use-pml --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
C64="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 8 --time-steps 64 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
U="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json --scene vacuum --use-pml --use-tfsf"
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for cfg in D C64 U C; do
  for r in 1 2; do
    for n in 3 2 4; do
      timeout -k 10 200 python3 -m fdtd3d_amd ${!cfg} --shell-streams $n > $O/${cfg}_${n}_$r.log 2>&1 || { echo "$cfg $n failed"; tail -5 $O/${cfg}_${n}_$r.log; exit 1; }
      echo "$cfg streams=$n $(grep -o '"mcells_per_s[^,]*' $O/${cfg}_${n}_$r.log)"
    done
  done
done
