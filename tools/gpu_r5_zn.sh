#!/bin/bash
# Round 5: 16-row multi-row tiles (8 waves x 2 rows) for the thin y shells of decomposed passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zn
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_tb_gpu.py -k "shape8" -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
tail -1 $O/tests.log
FDTD3D_TB_THIN_MR16=1 timeout -k 10 400 python -u -m pytest tests/test_parallel_gpu.py -q --timeout 240 --timeout-method thread > $O/tests_par.log 2>&1 || { echo par tests failed; grep -E "FAILED|Error" $O/tests_par.log | head; exit 1; }
tail -1 $O/tests_par.log
for r in 1 2; do
  for m in 0 1; do
    FDTD3D_TB_THIN_MR16=$m timeout -k 10 240 python -u tools/decomp_cost.py --size 1024 1024 1024 --world 8 --topology 4 2 1 --time-block 4 --transport loopback --link-gbs 50 > $O/421_m${m}_$r.log 2>&1 || { echo decomp failed; tail -5 $O/421_m${m}_$r.log; exit 1; }
    echo "== 4x2x1 mr16=$m"; grep -h "per pass\|decomposed" $O/421_m${m}_$r.log
  done
done
