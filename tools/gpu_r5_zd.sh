#!/bin/bash
# Round 5: hybrid tests after hoisting the CPML kernel table out of the parallel window launches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zd
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hybrid_gpu.py tests/test_graph_gpu.py tests/test_drude_blk_gpu.py tests/test_hip_gpu.py -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
