#!/bin/bash
# per-kind null coefficient arrays (fused + blocked kernels): GPU tests + sphere configs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pc.log 2>&1 || { tail -30 gpurun_out/pytest_pc.log; exit 1; }
tail -2 gpurun_out/pytest_pc.log
S="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --scene sphere --sphere-eps 4 --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128 --json"
for tb in "--time-steps 200" "--time-steps 200 --time-block 1" "--time-steps 210 --time-block 2"; do
  echo "== $tb"
  timeout -k 10 120 python -m fdtd3d_amd $S $tb > gpurun_out/pc.log 2>&1 || { tail -20 gpurun_out/pc.log; exit 1; }
  grep -o '"mcells_per_s[^,]*' gpurun_out/pc.log || tail -3 gpurun_out/pc.log
done
for mr in 1 2; do
  echo "== T=4 mrows=$mr"
  timeout -k 10 120 python -c "
import sys
from fdtd3d_amd.ops.hip_ops import HipOps
HipOps.tb_mrows = $mr
sys.argv = ['fdtd3d_amd'] + '$S --time-steps 210 --time-block 4'.split()
from fdtd3d_amd.runner import main
main()" > gpurun_out/pc.log 2>&1 || { tail -20 gpurun_out/pc.log; exit 1; }
  grep -o '"mcells_per_s[^,]*' gpurun_out/pc.log || tail -3 gpurun_out/pc.log
done
