#!/bin/bash
# Temporal-blocking session: TB tests, then bench sweep over T and x chunk.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m fdtd3d_amd.ops.build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests/test_tb_gpu.py -x -q > gpurun_out/pytest_tb.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_tb.log
[ $rc -ne 0 ] && exit $rc
while read -r args; do
  [ -z "$args" ] && continue
  timeout -k 10 200 python bench.py --steps 24 --warmup 4 $args > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
  echo "[$args] $(grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/bench.log)"
done < "${TB_SWEEP_FILE:-tools/tb_sweep.txt}"
