#!/bin/bash
# GPU session: build, GPU tests, benches (split vs fused kernels).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python -m fdtd3d_amd.ops.build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
for extra in "" "--split" ${BENCH_EXTRA}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $extra > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 1; }
  echo "[$extra] $(grep metric gpurun_out/bench.log | cut -c1-200)"
done
