#!/bin/bash
# Round 4: 1024^3 vacuum -- native single rank vs x-slab ranks of one process on one GPU (concurrent launches)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
A="--3d --sizex 1024 --same-size --dtype f32 --time-steps 45 --warmup-steps 5 --scene vacuum"
for r in 1 2 4 8; do
  if [ $r = 1 ]; then X=""; else X="--parallel-grid --topology-sizex $r"; fi
  timeout -k 10 120 ./fdtd3d_amd/fdtd3d $A $X > $O/n$r.log 2>&1 || { echo "native $r failed"; tail -3 $O/n$r.log; exit 1; }
  echo "ranks $r: $(grep Throughput $O/n$r.log)"
done
timeout -k 10 120 ./fdtd3d_amd/fdtd3d $A > $O/n1b.log 2>&1 && echo "ranks 1 again: $(grep Throughput $O/n1b.log)"
timeout -k 10 120 ./fdtd3d_amd/fdtd3d $A --parallel-grid --topology-sizex 4 > $O/n4b.log 2>&1 && echo "ranks 4 again: $(grep Throughput $O/n4b.log)"
