#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_hip_gpu.py -q -x -k "amplitude" --timeout 120 --timeout-method thread > gpurun_out/amp_t.log 2>&1 &&
timeout -k 10 300 python -u tools/amp_bench.py 256 100 f32 > gpurun_out/amp_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/amp_bench.py 256 100 f64 >> gpurun_out/amp_bench.log 2>&1
rc=$?
tail -3 gpurun_out/amp_t.log; grep -v amdgpu gpurun_out/amp_bench.log
exit $rc
