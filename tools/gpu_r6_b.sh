#!/bin/bash
# Round 6 (b): does the arrays' plane / row stride (power-of-two extents) cost the headline blocked pass?
# 1024^3 output box inside arrays padded along y or z, T = 5, alternating with the unpadded baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 400 python -u tools/tb_shape_probe.py --T 5 --reps 10 \
  --case 1024,1024,1024:0,0,0:1024,1024,1024 \
  --case 1024,1028,1024:0,0,0:1024,1024,1024 \
  --case 1024,1024,1028:0,0,0:1024,1024,1024 \
  --case 1024,1024,1024:0,0,0:1024,1024,1024 \
  --case 1024,1032,1024:0,0,0:1024,1024,1024 \
  --case 1024,1040,1024:0,0,0:1024,1024,1024 \
  --case 1024,1024,1024:0,0,0:1024,1024,1024 \
  --case 1024,1028,1028:0,0,0:1024,1024,1024 \
  > $O/probe.log 2>&1 || { echo probe failed; tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
