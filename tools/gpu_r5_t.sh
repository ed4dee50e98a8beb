#!/bin/bash
# Round 5: HBM traffic per kernel of config 3 (512^3 CPML + TF/SF, hybrid passes): reads (EA 128B / 64B
# requests), writes, and a kernel trace for the durations -- where the stepped shell's bandwidth goes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5t
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 5 --time-steps 25 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_kt -o run -- python3 -m fdtd3d_amd $C > $O/kt.log 2>&1 && cp /tmp/t_kt/run_kernel_stats.csv $O/kt_stats.csv || { echo "kt failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum --output-format csv -d /tmp/t_rd -o run -- python3 -m fdtd3d_amd $C > $O/rd.log 2>&1 && cp /tmp/t_rd/run_counter_collection.csv $O/rd.csv || { echo "rd failed"; tail -3 $O/rd.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/t_wr -o run -- python3 -m fdtd3d_amd $C > $O/wr.log 2>&1 && cp /tmp/t_wr/run_counter_collection.csv $O/wr.csv || { echo "wr failed"; tail -3 $O/wr.log; exit 1; }
ls -la $O
echo done
