#!/bin/bash
# Round 4: exchange / interior overlap of the decomposed blocked step on ONE
# GPU (tools/decomp_cost.py loopback transport: real pack, device copy, unpack
# on the side stream, plus an optional spin for the xGMI wire time)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
run() {
  local lab=$1; shift
  timeout -k 10 240 python -u tools/decomp_cost.py "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "== $lab"; tail -3 $O/$lab.log
}
for t in "1024_421:--size 1024 1024 1024 --topology 4 2 1" "2048_222:--size 2048 1024 1024 --topology 2 2 2 --axes xyz"; do
  lab=${t%%:*}; args=${t#*:}
  run ${lab}_null $args --world 8 --time-block 4 --transport null || exit 1
  run ${lab}_loop $args --world 8 --time-block 4 --transport loopback || exit 1
  run ${lab}_loop50 $args --world 8 --time-block 4 --transport loopback --link-gbs 50 || exit 1
done
echo done1
# 1024^3 Drude + UPML on one GPU: peak memory with region-local D / D1
timeout -k 10 400 python -m fdtd3d_amd --3d --sizex 1024 --same-size --dtype f32 --warmup-steps 5 --time-steps 20 --json \
  --scene drude-sphere --use-metamaterials --use-pml --sphere-center-x 512 --sphere-center-y 512 --sphere-center-z 512 \
  --sphere-radius 256 > $O/drude_1024.log 2>&1 || { echo "drude 1024 failed"; tail -5 $O/drude_1024.log; exit 1; }
grep '^{' $O/drude_1024.log
timeout -k 10 400 python -m fdtd3d_amd --3d --sizex 1024 --same-size --dtype f32 --warmup-steps 5 --time-steps 20 --json \
  --scene vacuum --use-pml --use-tfsf > $O/upml_tfsf_1024.log 2>&1 || { echo "upml 1024 failed"; tail -5 $O/upml_tfsf_1024.log; exit 1; }
grep '^{' $O/upml_tfsf_1024.log
echo done2
