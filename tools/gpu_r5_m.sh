#!/bin/bash
# Round 5: headline repeatability on one box (3 bench runs) + the kernel's resource use
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --physics-companion off --fp64-companion off > $O/bench$r.log 2>&1 || { echo bench failed; tail -3 $O/bench$r.log; exit 1; }
  echo "run $r $(tail -1 $O/bench$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done
timeout -k 10 300 python -m fdtd3d_amd --3d --sizex 1024 --same-size --dtype f32 --scene vacuum --warmup-steps 5 --time-steps 25 --json > $O/cli.log 2>&1
grep -o '"mcells_per_s": [0-9.]*' $O/cli.log
