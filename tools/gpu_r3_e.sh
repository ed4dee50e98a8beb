#!/bin/bash
# CPML in the blocked kernel: pass vs stepped (all cases), blocked-shell hybrid tests, 512^3 configs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cpml_tb_gpu.py -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|^E " $O/tests.log | cut -c1-400 | head -60
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_hybrid_gpu.py -x -v --timeout 120 --timeout-method thread -k "hybrid3 or at_scale" > $O/tests2.log 2>&1
rc=$?
grep -E "PASS|FAIL|^E " $O/tests2.log | cut -c1-400 | head -40
[ $rc -ne 0 ] && exit $rc
TS="5 4" bash tools/gpu_r3_d_cfg.sh
