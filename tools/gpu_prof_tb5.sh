#!/bin/bash
# Profiles of the default bench (blocked multi-row kernel, T=5): kernel trace
# stats, then EA read / write request counters in their own passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/prof_tb5
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 bench.py --steps 20 --warmup 5 > $O/kt.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/rd -o run -- python3 bench.py --steps 10 --warmup 0 > $O/rd.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wr -o run -- python3 bench.py --steps 10 --warmup 0 > $O/wr.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU --output-format csv -d $O/sq -o run -- python3 bench.py --steps 10 --warmup 0 > $O/sq.log 2>&1
echo rc=$?
find $O -name "*.db" -o -name "*.csv" | head -20
