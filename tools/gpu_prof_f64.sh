#!/bin/bash
# Kernel trace + EA traffic of the fp64 blocked kernel (bench.py --dtype f64).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/prof_f64
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 bench.py --dtype f64 --steps 16 --warmup 4 > $O/kt.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/rd -o run -- python3 bench.py --dtype f64 --steps 8 --warmup 0 > $O/rd.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wr -o run -- python3 bench.py --dtype f64 --steps 8 --warmup 0 > $O/wr.log 2>&1
echo rc=$?
