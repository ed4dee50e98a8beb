#!/bin/bash
# Round 5: decomposed passes with the shells on the exchange stream next to the interior pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parallel_gpu.py -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in "8_421:--world 8 --topology 4 2 1" "4_221:--world 4 --topology 2 2 1" "8_222:--world 8 --topology 2 2 2 --size 2048 1024 1024" "8_811:--world 8 --topology 8 1 1"; do
  lab=${t%%:*}; args=${t#*:}
  timeout -k 10 240 python -u tools/decomp_cost.py --size 1024 1024 1024 $args --time-block 4 --transport loopback --link-gbs 50 > $O/$lab.log 2>&1 || { echo $lab failed; tail -5 $O/$lab.log; exit 1; }
  echo "== $lab"; grep -h "per pass\|decomposed" $O/$lab.log
done
for sh in "256 512 1024" "248 504 1024"; do
  set -- $sh
  timeout -k 10 200 python -u -m fdtd3d_amd --3d --sizex $1 --sizey $2 --sizez $3 --dtype f32 --time-block 4 --time-steps 48 --warmup-steps 16 > $O/ser_$1.log 2>&1 || { echo ser failed; tail -5 $O/ser_$1.log; exit 1; }
  echo "== serial $sh"; grep -i "mcells" $O/ser_$1.log | tail -1
done
