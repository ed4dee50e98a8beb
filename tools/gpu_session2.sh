#!/bin/bash
# Full GPU session: build, all GPU tests, headline bench (blocked T=2 and
# single-pass), rocprofv3 kernel stats and HBM counters of the blocked bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
python -m fdtd3d_amd.ops.build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
echo "== pytest -m gpu"
timeout -k 10 480 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -6 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
echo "== bench"
for extra in "" "--time-block 1"; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 4 $extra > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 1; }
  echo "[$extra] $(cut -c1-200 gpurun_out/bench.log)"
done
echo "== rocprofv3 stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/tb -o run -- python3 bench.py --steps 10 --warmup 2 \
  > gpurun_out/prof_tb.log 2>&1 || { tail -20 gpurun_out/prof_tb.log; exit 1; }
echo "== rocprofv3 pmc"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-trace -d gpurun_out/prof2/pmc -o run -- python3 bench.py --steps 4 --warmup 2 \
  > gpurun_out/prof_pmc.log 2>&1 || { tail -20 gpurun_out/prof_pmc.log; exit 1; }
find gpurun_out/prof2 -type f | head -20
