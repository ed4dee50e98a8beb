#!/bin/bash
# Kernel trace + EA traffic of the 2D blocked kernel (TMz 16384^2, T=7) and
# the per-step 2D kernels for comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/prof_2d
mkdir -p $O
ARGS="-m fdtd3d_amd --2d --sizex 16384 --sizey 16384 --scene vacuum --dtype f32 --json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $ARGS --time-steps 70 --time-block 7 > $O/kt.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt1 -o run -- python3 $ARGS --time-steps 20 --time-block 1 > $O/kt1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/rd -o run -- python3 $ARGS --time-steps 14 --time-block 7 > $O/rd.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wr -o run -- python3 $ARGS --time-steps 14 --time-block 7 > $O/wr.log 2>&1
echo rc=$?
