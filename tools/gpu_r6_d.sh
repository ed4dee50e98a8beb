#!/bin/bash
# Round 6 (d): repeat the 1024^3 decomposition costs (loopback, 50 GB/s links) for the bench.py rank grid / T
# choice: 2, 4 and 8 ranks at T = 4 and 5, alternating, plus the whole-grid serial pass at T = 4 / 5
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 200 python -u tools/tb_shape_probe.py --T 5 --reps 10 --case 1024,1024,1024:0,0,0:1024,1024,1024 \
  --case 1024,1024,1024:0,0,0:1024,1024,1024 > $O/serial5.log 2>&1 || { echo probe failed; exit 1; }
timeout -k 10 200 python -u tools/tb_shape_probe.py --T 4 --reps 10 --case 1024,1024,1024:0,0,0:1024,1024,1024 \
  --case 1024,1024,1024:0,0,0:1024,1024,1024 > $O/serial4.log 2>&1 || { echo probe failed; exit 1; }
grep Mcells $O/serial5.log $O/serial4.log
for rep in 1 2; do
  for t in "2_211:--world 2 --topology 2 1 1" "4_221:--world 4 --topology 2 2 1" "4_411:--world 4 --topology 4 1 1" "8_421:--world 8 --topology 4 2 1" "8_241:--world 8 --topology 2 4 1"; do
    lab=${t%%:*}; args=${t#*:}
    for T in 4 5; do
      timeout -k 10 240 python -u tools/decomp_cost.py --size 1024 1024 1024 $args --time-block $T --transport loopback --link-gbs 50 > $O/${lab}_T${T}_$rep.log 2>&1 || { echo $lab failed; tail -5 $O/${lab}_T${T}_$rep.log; exit 1; }
      echo "== $lab T=$T rep $rep: $(grep -h 'decomposed' $O/${lab}_T${T}_$rep.log)"
    done
  done
done
