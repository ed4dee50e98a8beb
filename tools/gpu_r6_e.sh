#!/bin/bash
# Round 6 (e): headline PMC refresh of k_tb3d_mr<5, ...> at 1024^3 (EA reads, writes, two SQ groups: one
# counter group per rocprofv3 run), and the 2D TMz 8192^2 CPML + TF/SF hybrid run through the Python driver
# vs the native driver (kernel traces: where the Python pass loses)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6e
mkdir -p $O
RD="TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_sum"
WR="WRITE_SIZE"
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
SQ2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_CYCLES"
pass() {  # name, counters, bench args
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/$name -o run -- python3 -u bench.py --steps 10 --warmup 0 --init zero --fp64-companion off --physics-companion off "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; return 1; }
  echo "$name ok"
}
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --fp64-companion off --physics-companion off > $O/bench.log 2>&1 || { echo bench failed; exit 1; }
tail -1 $O/bench.log | cut -c1-200
pass f32_rd "$RD" && pass f32_wr "$WR" && pass f32_sq1 "$SQ1" && pass f32_sq2 "$SQ2" || exit 1
P2="--2d --sizex 8192 --sizey 8192 --time-steps 154 --warmup-steps 14 --scene vacuum --use-pml --pml-type cpml --use-tfsf --dtype f32 --json"
timeout -k 10 200 python3 -m fdtd3d_amd $P2 > $O/py2d.log 2>&1 || { echo py2d failed; tail -5 $O/py2d.log; exit 1; }
timeout -k 10 200 ./fdtd3d_amd/fdtd3d $P2 > $O/nat2d.log 2>&1 || { echo nat2d failed; tail -5 $O/nat2d.log; exit 1; }
echo "2D python $(grep -o '"mcells_per_s": [0-9.]*' $O/py2d.log)  native $(grep -o '"mcells_per_s": [0-9.]*' $O/nat2d.log)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_py2d -o run -- python3 -m fdtd3d_amd $P2 > $O/kt_py2d.log 2>&1 && cp /tmp/t_py2d/run_kernel_stats.csv $O/kt_py2d.csv || { echo "kt py2d failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_nat2d -o run -- ./fdtd3d_amd/fdtd3d $P2 > $O/kt_nat2d.log 2>&1 && cp /tmp/t_nat2d/run_kernel_stats.csv $O/kt_nat2d.csv || { echo "kt nat2d failed"; exit 1; }
echo done
