#!/bin/bash
# Round 5: amplitude passes with the running maxima in registers (8 waves x 2 rows, T <= 5) vs the LDS form
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_gpu.py -k amplitude -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/amp_bench.py 512 60 f32 > $O/amp512.log 2>&1 || { echo "bench512 failed"; tail -5 $O/amp512.log; exit 1; }
cat $O/amp512.log
timeout -k 10 300 python -u tools/amp_bench.py 256 120 f32 > $O/amp256.log 2>&1 || { echo "bench failed"; tail -5 $O/amp256.log; exit 1; }
cat $O/amp256.log
echo done
