#!/bin/bash
# Round 6 (o): fp64 512^3 CPML + TF/SF and UPML + TF/SF: steps per hybrid pass and shell streams
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6o
mkdir -p $O
B="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 12 --time-steps 48 --json --scene vacuum --use-pml --use-tfsf"
for rep in 1 2; do
  for m in cpml upml; do
    for v in "4 3" "3 3" "5 3" "4 2" "4 4"; do
      set -- $v
      timeout -k 10 300 python3 -m fdtd3d_amd $B --pml-type $m --hybrid-block $1 --shell-streams $2 > $O/r.log 2>&1 || { echo "$m $v failed"; tail -5 $O/r.log; exit 1; }
      echo "rep $rep f64 $m T=$1 streams=$2: $(grep -o '"mcells_per_s": [0-9.]*' $O/r.log | cut -d' ' -f2)"
    done
  done
done
