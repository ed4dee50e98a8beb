#!/bin/bash
# fp64 (the reference's default value type): blocked-kernel + hybrid tests, then runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tb_gpu.py tests/test_hybrid_gpu.py -x -q -k "f64" --timeout 120 --timeout-method thread > gpurun_out/pytest_f64.log 2>&1
rc=$?; grep -E "FAIL|Error|assert" gpurun_out/pytest_f64.log | head; tail -2 gpurun_out/pytest_f64.log; [ $rc -ne 0 ] && exit $rc
C512="--3d --sizex 512 --same-size --warmup-steps 8 --json"
for args in "--time-steps 64 --scene vacuum" "--time-steps 40 --scene vacuum --use-pml --pml-type cpml --use-tfsf" \
            "--time-steps 40 --scene vacuum --use-pml --use-tfsf" "--time-steps 40 --scene vacuum --use-pml --use-tfsf --hybrid-block 1"; do
  timeout -k 10 200 python -m fdtd3d_amd $C512 $args > gpurun_out/f64.log 2>&1 || { tail -5 gpurun_out/f64.log; exit 1; }
  echo "[f64 $args] $(grep -o '"mcells_per_s": [0-9.]*' gpurun_out/f64.log)"
done
timeout -k 10 300 python bench.py --dtype f64 --steps 16 --warmup 4 > gpurun_out/bench_f64.log 2>&1 && cut -c1-200 gpurun_out/bench_f64.log
