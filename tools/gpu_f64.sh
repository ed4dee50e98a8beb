#!/bin/bash
# fp64 blocked kernel: oracle tests, then 1024^3 throughput per tile shape and T
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tb_gpu.py -k f64 \
  > gpurun_out/f64_tests.log 2>&1 || { tail -30 gpurun_out/f64_tests.log; exit 1; }
tail -3 gpurun_out/f64_tests.log
for half in 1 0; do
  for T in 4 5; do
    FDTD3D_TB64_HALF=$half timeout -k 10 200 python bench.py --dtype f64 --steps 20 --warmup 5 --time-block $T \
      > gpurun_out/f64_h${half}_T$T.json 2> gpurun_out/f64_err.log || { tail gpurun_out/f64_err.log; exit 1; }
    echo "half=$half T=$T $(cat gpurun_out/f64_h${half}_T$T.json)"
  done
done
