#!/bin/bash
# Round 6 (an): fp64 1024^3 headline, T = 4 vs 5 (alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6an
mkdir -p $O
for r in 1 2; do
  for T in 4 5; do
    timeout -k 10 200 python3 bench.py --dtype f64 --time-block $T --steps 20 --warmup 4 --fp64-companion off --physics-companion off > $O/f64_T${T}_$r.log 2>&1 || { echo "T=$T failed"; tail -5 $O/f64_T${T}_$r.log; exit 1; }
    echo "T=$T $(tail -1 $O/f64_T${T}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["time_block"])')"
  done
done
