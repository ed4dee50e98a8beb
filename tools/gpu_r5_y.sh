#!/bin/bash
# Round 5: the shell-stream fork fix (side streams no longer wait for the main stream's first launch):
# decomposed 4x2x1 pass (with / without any exchange) and the bench with its physics companions
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5y
mkdir -p $O
A="--size 1024 1024 1024 --world 8 --topology 4 2 1 --time-block 4"
for v in "skip:--skip-exchange" "loop:--transport loopback --link-gbs 50" "loop1:--transport loopback --link-gbs 50 --shell-streams 1"; do
  lab=${v%%:*}; args=${v#*:}
  timeout -k 10 240 python -u tools/decomp_cost.py $A $args > $O/$lab.log 2>&1 || { echo $lab failed; tail -5 $O/$lab.log; exit 1; }
  echo "== $lab"; grep -h "per pass\|decomposed" $O/$lab.log
done
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -1 $O/bench.log
