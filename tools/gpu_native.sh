#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_native_gpu.py -q -x --timeout 200 --timeout-method thread -k "upml or drude or lorentz or ntff" > gpurun_out/native_t.log 2>&1
rc=$?
tail -25 gpurun_out/native_t.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_amp.sh
