#!/bin/bash
# Round 4: amplitude mode on blocked passes -- GPU tests, 256^3 rates
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_gpu.py -x -q -k amplitude --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/amp_bench.py 256 120 f32 > $O/amp256.log 2>&1 || { echo "bench failed"; tail -5 $O/amp256.log; exit 1; }
timeout -k 10 300 python -u tools/amp_bench.py 512 60 f32 > $O/amp512.log 2>&1 || { echo "bench512 failed"; tail -5 $O/amp512.log; exit 1; }
cat $O/amp512.log
cat $O/amp256.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m fdtd3d_amd --3d --sizex 256 \
  --same-size --dtype f32 --time-steps 20 --use-amp-mode --amplitude-time-steps 96 --scene vacuum \
  > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo done
