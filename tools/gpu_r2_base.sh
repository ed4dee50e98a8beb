#!/bin/bash
# Round-2 baseline on one MI355X: GPU tests, bench.py (fp32 headline + fp64
# companion), and the per-GPU decomposition cost of the 8-rank grids
# (4x2x1 vs 2x2x2, 1024^3 and 2048x1024x1024) with a null transport.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -30 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 200 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
: > gpurun_out/decomp.log
while read -r args; do
  [ -z "$args" ] && continue
  echo "== $args" >> gpurun_out/decomp.log
  timeout -k 10 200 python tools/decomp_cost.py $args >> gpurun_out/decomp.log 2>&1 || { tail -5 gpurun_out/decomp.log; exit 1; }
done <<'LIST'
--world 8 --topology 4 2 1 --time-block 4
--world 8 --topology 2 2 2 --time-block 4
--world 8 --topology 2 2 2 --time-block 5
--world 8 --size 2048 1024 1024 --topology 4 2 1 --time-block 4
--world 8 --size 2048 1024 1024 --topology 2 2 2 --time-block 4
--world 8 --size 2048 1024 1024 --topology 8 1 1 --time-block 4
LIST
grep -v amdgpu.ids gpurun_out/decomp.log
