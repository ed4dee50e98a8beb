#!/bin/bash
# hybrid-pass GPU tests, then the PML / TF-SF / Drude 512^3 configs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hybrid_gpu.py tests/test_parallel_gpu.py \
  > gpurun_out/hyb_tests.log 2>&1 || { tail -30 gpurun_out/hyb_tests.log; exit 1; }
tail -2 gpurun_out/hyb_tests.log
timeout -k 10 600 python tools/bench_configs.py --only ${ONLY:-3d-512-cpml-tfsf 3d-512-upml-tfsf 3d-512-drude 3d-512-cpml-point} \
  --out gpurun_out/cfg.md > gpurun_out/cfg.log 2>&1 || { tail -20 gpurun_out/cfg.log; exit 1; }
cat gpurun_out/cfg.md
