#!/bin/bash
# HBM-counter calibration on kernels of known traffic (tools/bw_calib.py: a
# 4 GiB read, a 2+2 GiB copy, a 2 GiB fill), then the default bench: shows that
# on gfx950 FETCH_SIZE under-reports reads (1/2..1/4) while
# TCC_EA0_RDREQ_128B x 128 B matches the copy's read volume exactly.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/calib
mkdir -p $O
C="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
timeout -k 10 120 python tools/bw_calib.py > $O/plain.log 2>&1 && cat $O/plain.log &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 tools/bw_calib.py > $O/f.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 tools/bw_calib.py > $O/w.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/c -o run -- python3 tools/bw_calib.py > $O/c.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/tb -o run -- python3 bench.py --steps 10 --warmup 0 > $O/tb.log 2>&1
echo rc=$?
