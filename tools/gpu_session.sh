#!/bin/bash
# One GPU session: build, GPU tests, headline bench (fused + split), native
# driver run, rocprofv3 kernel stats of both bench variants.
# Usage (from the container): gpurun --timeout 1100 -- bash tools/gpu_session.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
python -m fdtd3d_amd.ops.build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
echo "== pytest -m gpu"
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -6 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
echo "== bench"
for extra in "" "--split"; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 $extra > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 1; }
  echo "[$extra] $(grep metric gpurun_out/bench.log | cut -c1-220)"
done
echo "== native driver"
timeout -k 10 300 ./fdtd3d_amd/fdtd3d --3d --sizex 1024 --same-size --time-steps 50 --scene vacuum --dtype f32 \
  > gpurun_out/native.log 2>&1 || { cat gpurun_out/native.log; exit 1; }
grep -E "Total time|Throughput|Backend" gpurun_out/native.log
echo "== rocprofv3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/fused -o run -- python3 bench.py --steps 10 --warmup 3 \
  > gpurun_out/prof_fused.log 2>&1 || { tail -20 gpurun_out/prof_fused.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/split -o run -- python3 bench.py --steps 10 --warmup 3 --split \
  > gpurun_out/prof_split.log 2>&1 || { tail -20 gpurun_out/prof_split.log; exit 1; }
find gpurun_out/prof -name "*kernel_stats*"
