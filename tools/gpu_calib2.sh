#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/calib2
mkdir -p $O
C="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/c -o run -- python3 tools/bw_calib.py > $O/c.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/t4 -o run -- python3 bench.py --steps 8 --warmup 0 --time-block 4 --tb-mrows 1 > $O/t4.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/t4m -o run -- python3 bench.py --steps 8 --warmup 0 --time-block 4 --tb-mrows 2 > $O/t4m.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/t1 -o run -- python3 bench.py --steps 4 --warmup 0 --time-block 1 > $O/t1.log 2>&1
echo rc=$?
