#!/bin/bash
# PMC passes (one counter group per run) over the blocked-kernel bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_tb
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
P5="SQ_WAVES SQ_CYCLES SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU"
for cfg in "${CFGS[@]:-mr1:--time-block 4 --tb-mrows 1}" ; do :; done
run() {  # name, bench args
  local name=$1; shift
  local n=0
  for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    n=$((n+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/$name/p$n -o run -- python3 bench.py --steps 8 --warmup 0 "$@" > $OUT/$name.p$n.log 2>&1 || { echo "pass $n of $name failed"; tail -5 $OUT/$name.p$n.log; return 1; }
  done
  echo "$name done"
}
run mr1 --time-block 4 --tb-mrows 1 && run mr2 --time-block 4 --tb-mrows 2 && run t5 --time-block 5
