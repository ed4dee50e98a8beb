#!/bin/bash
# Round 6 (aq): config 3 shell streams 2 / 3 / 4 (alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6aq
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for r in 1 2; do
  for n in 3 2 4; do
    timeout -k 10 200 python3 -m fdtd3d_amd $C --shell-streams $n > $O/s_${n}_$r.log 2>&1 || { echo "$n failed"; tail -5 $O/s_${n}_$r.log; exit 1; }
    echo "streams=$n $(grep -o '"mcells_per_s[^,]*' $O/s_${n}_$r.log)"
  done
done
