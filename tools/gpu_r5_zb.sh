#!/bin/bash
# Round 5: native 3D rank grids; x-face halo messages without pack / unpack; kernel rate vs array shape; decomposed passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zb
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_parallel_gpu.py tests/test_native_gpu.py -k "parallel" -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/tb_shape_probe.py --T 4 \
  --case 256,512,1024:0,0,0:256,512,1024 \
  --case 256,512,1024:4,4,0:248,504,1024 \
  --case 264,516,1024:0,0,0:264,516,1024 \
  --case 264,516,1024:8,8,0:248,504,1024 \
  --case 264,516,1024:4,4,0:256,512,1024 \
  --case 248,504,1024:0,0,0:248,504,1024 \
  --case 264,520,1024:8,8,0:248,504,1024 \
  > $O/probe.log 2>&1 || { echo probe failed; tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
for t in "8_421:--world 8 --topology 4 2 1" "4_221:--world 4 --topology 2 2 1" "8_222:--world 8 --topology 2 2 2 --size 2048 1024 1024" "8_811:--world 8 --topology 8 1 1"; do
  lab=${t%%:*}; args=${t#*:}
  timeout -k 10 240 python -u tools/decomp_cost.py --size 1024 1024 1024 $args --time-block 4 --transport loopback --link-gbs 50 > $O/$lab.log 2>&1 || { echo $lab failed; tail -5 $O/$lab.log; exit 1; }
  echo "== $lab"; grep -h "per pass\|decomposed" $O/$lab.log
done
