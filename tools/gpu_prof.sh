#!/bin/bash
# Profile the headline bench with rocprofv3 (kernel trace + stats) and sweep xchunk.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
python -m fdtd3d_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
for xc in 8 16 32 64 128; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --xchunk $xc > gpurun_out/bench_xc$xc.log 2>&1 || exit 1
  echo "xchunk=$xc $(cut -c1-160 gpurun_out/bench_xc$xc.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof.log 2>&1 || exit 1
find gpurun_out/prof -name "*stats*" | head
