#!/bin/bash
# Round 4: blocked-kernel variant micro-bench + ISA resource table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 180 python -u tools/mr_bench.py --T 5 --rounds 3 > $O/mr5.log 2>&1 || { tail -5 $O/mr5.log; exit 1; }
grep -v amdgpu.ids $O/mr5.log
