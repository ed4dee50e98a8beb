#!/bin/bash
# Measure every BASELINE config on one MI355X; rocprof the non-vacuum ones.
# Usage: gpurun --timeout 1100 -- bash tools/gpu_configs.sh [config names...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
python -m fdtd3d_amd.ops.build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
ONLY=""
[ $# -gt 0 ] && ONLY="--only $*"
timeout -k 10 900 python tools/bench_configs.py $ONLY --out gpurun_out/configs.md > gpurun_out/configs.log 2>&1
rc=$?
cut -c1-260 gpurun_out/configs.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROF" ]; then
  for c in $PROF; do
    args=$(python -c "import sys; sys.path.insert(0,'tools'); import bench_configs as b; print(' '.join([x for n,d,x in b.CONFIGS if n=='$c'][0]))")
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/$c -o run -- python3 -m fdtd3d_amd $args \
      > gpurun_out/prof_$c.log 2>&1 || { tail -20 gpurun_out/prof_$c.log; exit 1; }
  done
fi
exit 0
