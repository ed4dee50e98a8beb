#!/bin/bash
# Round 5: native driver after moving the amplitude mode, 2D half steps and the option check out of main.cpp
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zh
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_native_gpu.py -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
