#!/bin/bash
# Round 5: the decomposed interior's rate vs array shape / box offset / box size (tools/tb_shape_probe.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5za
mkdir -p $O
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
