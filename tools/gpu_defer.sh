#!/bin/bash
# fp32 multi-row kernel: tests, then headline throughput per store variant
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tb_gpu.py tests/test_tfsf_tb_gpu.py \
  > gpurun_out/defer_tests.log 2>&1 || { tail -30 gpurun_out/defer_tests.log; exit 1; }
tail -3 gpurun_out/defer_tests.log
for v in 4 5 6 7; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --tb-variant $v > gpurun_out/defer_v$v.json 2> gpurun_out/defer_err.log \
    || { tail gpurun_out/defer_err.log; exit 1; }
  echo "variant=$v $(grep -o '"value": [0-9.]*' gpurun_out/defer_v$v.json)"
done
