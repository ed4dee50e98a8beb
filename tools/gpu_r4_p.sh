#!/bin/bash
# Round 4: headline steadiness on one fresh box -- bench.py three times back to back (companions off), then
# once with a longer warm-up
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
for n in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --fp64-companion off --physics-companion off > $O/b$n.log 2>&1 || { echo "bench $n failed"; tail -3 $O/b$n.log; exit 1; }
  echo "run $n: $(tail -1 $O/b$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 40 --fp64-companion off --physics-companion off > $O/bw.log 2>&1 || { echo "bench w failed"; exit 1; }
echo "warmup 40: $(tail -1 $O/bw.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
