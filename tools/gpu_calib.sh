#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on kernels of known traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/calib
mkdir -p $O
timeout -k 10 120 python tools/bw_calib.py > $O/plain.log 2>&1 && cat $O/plain.log &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 tools/bw_calib.py > $O/f.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 tools/bw_calib.py > $O/w.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tbf -o run -- python3 bench.py --steps 10 --warmup 0 --time-block 5 > $O/tbf.log 2>&1
echo rc=$?
