#!/bin/bash
# Round 6 (y): per-GPU cost of the 1024^3 decompositions at T = 4 vs 5 with the cached-plan exchange (loopback)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6y
mkdir -p $O
for rep in 1 2; do
  for t in "8_421:--world 8 --topology 4 2 1" "4_221:--world 4 --topology 2 2 1" "2_211:--world 2 --topology 2 1 1"; do
    lab=${t%%:*}; args=${t#*:}
    for T in 4 5; do
      timeout -k 10 240 python -u tools/decomp_cost.py --size 1024 1024 1024 $args --time-block $T --transport loopback --link-gbs 50 > $O/${lab}_T$T.log 2>&1 || { echo "$lab T$T failed"; tail -5 $O/${lab}_T$T.log; exit 1; }
      echo "rep $rep $lab T=$T: $(grep -h 'decomposed step' $O/${lab}_T$T.log)"
    done
  done
done
