#!/bin/bash
# Drude / 2D tests, then the Drude config (stepped and hybrid) with steady-state profiles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tb2d_gpu.py tests/test_hip_gpu.py \
  > gpurun_out/drude_tests.log 2>&1 || { tail -30 gpurun_out/drude_tests.log; exit 1; }
tail -2 gpurun_out/drude_tests.log
CONFIGS="drude" MARKER=k_update_h3d_v4 PASSES=20 bash tools/gpu_prof_configs.sh || exit 1
CONFIGS="drudeh" MARKER=k_tb3d_mr PASSES=8 bash tools/gpu_prof_configs.sh || exit 1
