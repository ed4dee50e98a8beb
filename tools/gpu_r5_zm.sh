#!/bin/bash
# Round 5: fp32 multi-row kernel patch order on the Drude, CPML + TF/SF and amplitude configs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zm
mkdir -p $O
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
D="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json"
declare -A CF
CF[drude]="$D --scene drude-sphere --use-metamaterials $S"
CF[cpml_tfsf]="$D --scene vacuum --use-pml --pml-type cpml --use-tfsf"
run() {
  local lab=$1 k=$2; shift 2
  env "$@" timeout -k 10 300 python -m fdtd3d_amd ${CF[$k]} > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(grep -o '"mcells_per_s": [0-9.]*' $O/$lab.log)"
}
for r in 1 2; do
  for k in drude cpml_tfsf; do
    run ${k}_base_$r $k A=1
    for p in 4x4 2x8; do run ${k}_p${p}_$r $k FDTD3D_TB_PATCH=$p; done
  done
  for p in 0 4x4 2x8; do
    if [ $p = 0 ]; then E=A=1; else E=FDTD3D_TB_PATCH=$p; fi
    env $E timeout -k 10 300 python tools/amp_bench.py 512 64 f32 > $O/amp_${p}_$r.log 2>&1 || { echo amp failed; tail -3 $O/amp_${p}_$r.log; }
    echo "amp_${p}_$r $(grep "blocked T = 3, check every 8" $O/amp_${p}_$r.log)"
  done
done
