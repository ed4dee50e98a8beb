#!/bin/bash
# PMC of the multi-row kernel: plain core vs CPML variants (T = 4), issue profile + instruction counts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
SQ2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES SQ_CYCLES"
SQ3="SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_SENDMSG"
for q in 1 2 3; do
  eval ctr=\$SQ$q
  timeout -s KILL 200 rocprofv3 --pmc $ctr --output-format csv -d $O/p$q -o run -- python3 -u tools/mr_bench.py --n 512 --rounds 1 --only "T4 " > $O/p$q.log 2>&1 || { echo "pass $q failed"; tail -5 $O/p$q.log; exit 1; }
done
python3 tools/pmc_csv.py k_tb3d_mr $(find $O -name '*counter_collection.csv') > $O/pmc.txt
cat $O/pmc.txt
