#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg_shell.py hybrid 2>&1 | tee gpurun_out/dbg_hybrid.log
