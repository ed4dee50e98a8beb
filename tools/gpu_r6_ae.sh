#!/bin/bash
# Round 6 (ae): fp64 config 3 (CPML + TF/SF, 512^3) -- hybrid T and TF/SF placement sweep, kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6ae
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 12 --time-steps 60 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for v in "4 core" "3 core" "5 core" "4 shell" "3 shell" "4 core" ; do
  set -- $v
  timeout -k 10 200 python3 -m fdtd3d_amd $C --hybrid-block $1 --hybrid-tfsf $2 > $O/r_$1_$2.log 2>&1 || { echo "T=$1 $2 failed"; tail -5 $O/r_$1_$2.log; exit 1; }
  echo "T=$1 $2 $(grep -o '"mcells_per_s[^,]*' $O/r_$1_$2.log)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_ae -o run -- python3 -m fdtd3d_amd $C > $O/kt.log 2>&1 && cp /tmp/t_ae/run_kernel_stats.csv $O/kt_stats.csv || { echo "kt failed"; exit 1; }
echo done
