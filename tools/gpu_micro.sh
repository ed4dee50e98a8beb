#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/shell_micro.py 512 > gpurun_out/shell_micro.log 2>&1 &&
FDTD3D_SHELL_WAVES=8 timeout -k 10 300 python -u tools/shell_micro.py 512 > gpurun_out/shell_micro8.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/shell_micro.log
echo "--- 8 waves"
grep -v amdgpu.ids gpurun_out/shell_micro8.log
exit $rc
