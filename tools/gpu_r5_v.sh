#!/bin/bash
# Round 5 (re-entry): full GPU suite, smoke and bench on the rebuilt libraries at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5v7
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  --deselect "tests/test_native_gpu.py::test_native_checkpoint_roundtrip" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; }
tail -2 $O/tests.log
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -k checkpoint_roundtrip -q --timeout 240 --timeout-method thread > $O/tests_ck.log 2>&1 \
  || { echo "ckpt tests failed"; tail -30 $O/tests_ck.log; }
tail -2 $O/tests_ck.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -1 $O/bench.log
