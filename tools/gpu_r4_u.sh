#!/bin/bash
# Round 4: 2D physics (8192^2 TMz) -- Python hybrid driver vs the native driver, and the Python run's kernel time
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
A="--2d --sizex 8192 --sizey 8192 --dtype f32 --warmup-steps 10 --time-steps 110 --scene vacuum"
for cfg in "cpml_tfsf:--use-pml --pml-type cpml --use-tfsf" "upml_tfsf:--use-pml --use-tfsf" "vacuum:"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 python -m fdtd3d_amd $A $args --json > $O/py_$lab.log 2>&1 || { echo "py $lab failed"; tail -3 $O/py_$lab.log; exit 1; }
  echo "python $lab: $(grep Throughput $O/py_$lab.log)"
  timeout -k 10 200 ./fdtd3d_amd/fdtd3d $A $args > $O/nat_$lab.log 2>&1 || { echo "native $lab failed"; tail -3 $O/nat_$lab.log; exit 1; }
  echo "native $lab: $(grep Throughput $O/nat_$lab.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m fdtd3d_amd $A --use-pml --pml-type cpml --use-tfsf > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
db=$(ls $O/prof/*.db | head -1); python3 tools/rocpd_stats.py "$db" --top 15 > $O/stats.md 2>&1; head -20 $O/stats.md
