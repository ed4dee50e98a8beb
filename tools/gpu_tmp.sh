#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parallel_gpu.py tests/test_tb_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_vec.log 2>&1 || { tail -30 gpurun_out/pytest_vec.log; exit 1; }
tail -2 gpurun_out/pytest_vec.log
: > gpurun_out/decomp_vec.log
for args in "--world 8 --axes xy --time-block 5" "--world 8 --axes xy --time-block 4" "--world 2 --axes xy --time-block 5"; do
  echo "== $args" >> gpurun_out/decomp_vec.log
  timeout -k 10 200 python tools/decomp_cost.py $args >> gpurun_out/decomp_vec.log 2>&1 || { tail -5 gpurun_out/decomp_vec.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/decomp_vec.log
