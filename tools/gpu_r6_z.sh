#!/bin/bash
# Round 6 (z): the 1024^3 headline at T = 4 / 5 / 6 (alternating, bench.py without companions)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6z
mkdir -p $O
for rep in 1 2 3; do
  for T in 5 4 6; do
    timeout -k 10 200 python3 bench.py --steps 30 --warmup 6 --time-block $T --fp64-companion off --physics-companion off > $O/b_$T.log 2>&1 || { echo "T$T failed"; tail -5 $O/b_$T.log; exit 1; }
    echo "rep $rep T=$T: $(tail -1 $O/b_$T.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
