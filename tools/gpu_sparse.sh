#!/bin/bash
# GPU tests of the blocked kernels (incl. sparse per-cell coefficients), then
# the 512^3 sphere at T = 2 / 4 / 5 under rocprof.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tb_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tbtest.log 2>&1 || { tail -30 gpurun_out/tbtest.log; exit 1; }
tail -2 gpurun_out/tbtest.log
CONFIGS="sphere3 sphere4 sphere5" bash tools/gpu_prof_configs.sh
