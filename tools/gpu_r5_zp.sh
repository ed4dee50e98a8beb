#!/bin/bash
# Round 5: multi-round x-chunk cap 192 (new default) vs 256 on the headline; blocked-kernel tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zp
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_tb_gpu.py -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
tail -1 $O/tests.log
B="--steps 20 --warmup 5 --fp64-companion off --physics-companion off"
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py $B > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*')"
}
for r in 1 2 3; do run cap192_$r A=1; run cap256_$r FDTD3D_TB_XCAP=256; done
B="--size 2048 1024 1024 --steps 10 --warmup 3 --fp64-companion off --physics-companion off"
for r in 1 2; do run big192_$r A=1; run big256_$r FDTD3D_TB_XCAP=256; done
