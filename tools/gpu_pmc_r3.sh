#!/bin/bash
# Round 3 PMC: headline fp32 (T=5) and fp64 (T=4) blocked kernels -- EA read requests, writes, issue profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export FDTD3D_BENCH_TRACE=1
O=gpurun_out/pmc_r3
mkdir -p $O
RD="TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_sum"
WR="WRITE_SIZE"
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
SQ2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_CYCLES"
pass() {  # name, counters, bench args
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 280 rocprofv3 --pmc $ctr --output-format csv -d $O/$name -o run -- python3 -u bench.py --steps 10 --warmup 0 --init zero --fp64-companion off "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; return 1; }
  echo "$name ok"
}
[ -n "$SKIP_KT" ] || { timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt32 -o run -- python3 bench.py --steps 20 --warmup 5 --fp64-companion off > $O/kt32.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt64 -o run -- python3 bench.py --dtype f64 --steps 16 --warmup 4 > $O/kt64.log 2>&1; } &&
pass f32_rd "$RD" && pass f32_wr "$WR" && pass f32_sq1 "$SQ1" && pass f32_sq2 "$SQ2" &&
pass f64_rd "$RD" --dtype f64 && pass f64_wr "$WR" --dtype f64 && pass f64_sq1 "$SQ1" --dtype f64 && pass f64_sq2 "$SQ2" --dtype f64
rc=$?
for f in $O/*.log; do echo "== $f"; grep -E '^\{|error|Error' $f | cut -c1-200 | head -3; done
exit $rc
