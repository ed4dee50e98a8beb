#!/bin/bash
# 8-wave x 4-row multi-row tiles: GPU tests, then bench.py 1024^3 at T = 4 / 5 / 6 for both shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tb_gpu.py -q -k shape8 --timeout 120 --timeout-method thread > gpurun_out/shape.log 2>&1 || { tail -20 gpurun_out/shape.log; exit 1; }
tail -1 gpurun_out/shape.log
for sh in 0 1; do for T in 4 5 6; do
  FDTD3D_TB_MR_SHAPE=$sh timeout -k 10 200 python bench.py --time-block $T --fp64-companion off --steps 30 > gpurun_out/bs.log 2>&1 || { tail -5 gpurun_out/bs.log; exit 1; }
  python -c 'import json,sys; d=json.loads(open("gpurun_out/bs.log").read().strip().splitlines()[-1]); print("shape", sys.argv[1], "T", sys.argv[2], d["value"], d["ms_per_step"])' $sh $T
done; done
