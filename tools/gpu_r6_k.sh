#!/bin/bash
# Round 6 (k): amplitude variant with one copy of its trip loop and component offsets in the lane offset
# (fewer SGPR spills) vs the previous build (ab/libfdtd3d_hip_base.so), alternating; amplitude GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_gpu.py -k amplitude -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u tools/amp_bench.py 512 96 f32 > $O/amp_new_$rep.log 2>&1 || { echo "amp new failed"; tail -3 $O/amp_new_$rep.log; exit 1; }
  echo "rep $rep new:"; grep "blocked T = 3" $O/amp_new_$rep.log
  FDTD3D_HIP_LIB=$PWD/ab/libfdtd3d_hip_base.so timeout -k 10 300 python -u tools/amp_bench.py 512 96 f32 > $O/amp_base_$rep.log 2>&1 || { echo "amp base failed"; tail -3 $O/amp_base_$rep.log; exit 1; }
  echo "rep $rep base:"; grep "blocked T = 3" $O/amp_base_$rep.log
done
