#!/bin/bash
# Headline profile (bench.py default: multi-row blocked kernel, T=5, automatic x chunk), fp32 only:
# kernel trace stats, then EA read requests, WRITE_SIZE and SQ counters in their own passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/prof_tb5r2
mkdir -p $O
B="bench.py --fp64-companion off"
if [ ! -f $O/kt.md ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $B --steps 20 --warmup 5 > $O/kt.log 2>&1 || exit 1
python3 tools/prof_summary.py $(find $O/kt -name '*results.db' | head -1) --cells 1073741824 > $O/kt.md 2>&1
rm -rf $O/kt
fi
B="$B --init zero"  # counter passes: skip the thousands of small random-init kernels
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/rd -o run -- python3 $B --steps 10 --warmup 0 > $O/rd.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wr -o run -- python3 $B --steps 10 --warmup 0 > $O/wr.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU --output-format csv -d $O/sq -o run -- python3 $B --steps 10 --warmup 0 > $O/sq.log 2>&1 || exit 1
python3 tools/pmc_csv.py k_tb3d_mr $(find $O/rd $O/wr $O/sq -name '*counter_collection.csv') > $O/pmc.txt
cat $O/kt.md | head -12; cat $O/pmc.txt; grep '^{' $O/kt.log | cut -c1-200
