#!/bin/bash
# Round 6 (ab): native --parallel-grid physics (CPML / TF/SF on the split half steps over ranks) against the
# Python fp64 oracle, the native GPU suite, and the per-GPU rate of a decomposed 512^3 config 3 (4 ranks on one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_native_gpu.py -k "parallel_grid" -v --timeout 240 --timeout-method thread > $O/multi.log 2>&1 || { echo multi failed; grep -E "FAILED|Error|assert" $O/multi.log | head -30; tail -5 $O/multi.log; exit 1; }
grep -E "passed|failed" $O/multi.log | tail -2
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -q --timeout 240 --timeout-method thread > $O/native.log 2>&1 || { echo native failed; grep -E "FAILED|Error" $O/native.log | head -30; tail -5 $O/native.log; exit 1; }
tail -1 $O/native.log
C="--3d --sizex 512 --same-size --time-steps 40 --warmup-steps 8 --scene vacuum --use-pml --pml-type cpml --use-tfsf --json"
timeout -k 10 200 fdtd3d_amd/fdtd3d $C --parallel-grid --topology-sizex 2 --topology-sizey 2 > $O/n_2x2.log 2>&1 || { echo n2x2 failed; tail -5 $O/n_2x2.log; exit 1; }
grep -E "Throughput|Backend" $O/n_2x2.log
timeout -k 10 200 fdtd3d_amd/fdtd3d $C > $O/n_1.log 2>&1 || { echo n1 failed; tail -5 $O/n_1.log; exit 1; }
grep -E "Throughput" $O/n_1.log
