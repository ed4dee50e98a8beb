#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python -m fdtd3d_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python tools/kbench.py --rounds 3 --steps 8 --xchunks ${XCHUNKS:-16,32,64} > gpurun_out/kbench.log 2>&1
rc=$?; cat gpurun_out/kbench.log; exit $rc
