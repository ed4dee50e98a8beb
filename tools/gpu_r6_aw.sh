#!/bin/bash
# Round 6 (aw): fp64 config 3 with two shell streams -- T and TF/SF placement (alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6aw
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 8 --time-steps 64 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for r in 1 2; do
  for v in "4 core" "5 core" "4 shell" "3 core"; do
    set -- $v
    timeout -k 10 200 python3 -m fdtd3d_amd $C --hybrid-block $1 --hybrid-tfsf $2 > $O/r_$1_$2_$r.log 2>&1 || { echo "T=$1 $2 failed"; tail -5 $O/r_$1_$2_$r.log; exit 1; }
    echo "T=$1 $2 $(grep -o '"mcells_per_s[^,]*' $O/r_$1_$2_$r.log)"
  done
done
