#!/bin/bash
# Multi-row blocked kernel: correctness vs the torch oracle, then a bench sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tb_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tb.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_tb.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
while read -r extra; do
  [ -z "$extra" ] && continue
  timeout -k 10 200 python bench.py --steps 60 --warmup 6 $extra > gpurun_out/bench_mr.log 2>&1 || { tail -5 gpurun_out/bench_mr.log; exit 1; }
  echo "[$extra] $(python -c 'import json,sys; d=json.loads(open("gpurun_out/bench_mr.log").read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])')"
done < "${SWEEP:-tools/tb_sweep.txt}"
