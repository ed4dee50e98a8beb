#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/dbg_shell.py pass > gpurun_out/dbg_pass.log 2>&1 &&
timeout -k 10 200 python -u tools/dbg_shell.py hybrid > gpurun_out/dbg_hy.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_shell_gpu.py tests/test_hybrid_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_hy.log 2>&1
rc=$?
grep -v '^     piece' gpurun_out/dbg_pass.log | cut -c1-200 | tail -8
cat gpurun_out/dbg_hy.log 2>/dev/null | cut -c1-250
tail -15 gpurun_out/t_hy.log 2>/dev/null
exit $rc
