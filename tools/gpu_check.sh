#!/bin/bash
# Re-entry GPU check: GPU tests, smoke(), headline bench (prebuilt in-tree .so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -8 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo "== bench"
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log | cut -c1-400
