#!/bin/bash
# Round 5, step A of the TF/SF work: why the in-kernel TF/SF variant costs 2x the plain kernel.
# Counter availability, then instruction-fetch counters of whole-grid vacuum + TF/SF vs plain vacuum
# (512^3 fp32, T = 4, no PML), one counter group per rocprofv3 run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || echo "list failed"
grep -oE '\bSQC?_[A-Z_]*(ICACHE|IFETCH|INST_LEVEL|WAIT_INST)[A-Z_]*' $O/avail.txt | sort -u > $O/ic_counters.txt || true
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 0 --time-steps 20 --json --time-block 4"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_IFETCH"
P2="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
for lab in plain tfsf; do
  extra=""
  [ $lab = tfsf ] && extra="--use-tfsf"
  timeout -k 10 120 python -m fdtd3d_amd $C --scene vacuum $extra > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; exit 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
  n=0
  for P in "$P1" "$P2"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$lab/p$n -o run -- python3 -m fdtd3d_amd $C --scene vacuum $extra > $O/pmc_$lab.p$n.log 2>&1 || { echo "pmc $lab p$n failed"; tail -3 $O/pmc_$lab.p$n.log; }
  done
done
echo done
