#!/bin/bash
# per-kind null coefficient arrays in the blocked kernels: tests + sphere configs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tb_gpu.py tests/test_parallel_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pc.log 2>&1 || { tail -30 gpurun_out/pytest_pc.log; exit 1; }
tail -2 gpurun_out/pytest_pc.log
S="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --scene sphere --sphere-eps 4 --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128 --json"
for tb in "--time-steps 200" "--time-steps 210 --time-block 4" "--time-steps 210 --time-block 5" "--time-steps 210 --time-block 3"; do
  echo "== $tb"
  timeout -k 10 120 python -m fdtd3d_amd $S $tb > gpurun_out/pc.log 2>&1 || { tail -20 gpurun_out/pc.log; exit 1; }
  grep -o '"mcells_per_s[^,]*' gpurun_out/pc.log || tail -3 gpurun_out/pc.log
done
