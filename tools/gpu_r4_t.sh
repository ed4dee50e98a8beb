#!/bin/bash
# Round 4: per-GPU cost of 1024^3 decompositions (x slabs vs x-y grids) on ONE GPU, loopback transport with
# a 50 GB/s emulated link, T = 4 / 5
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
run() {
  local lab=$1; shift
  timeout -k 10 240 python -u tools/decomp_cost.py "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "== $lab"; tail -2 $O/$lab.log
}
for t in "8_811:--world 8 --topology 8 1 1" "8_421:--world 8 --topology 4 2 1" "4_411:--world 4 --topology 4 1 1" "4_221:--world 4 --topology 2 2 1" "2_211:--world 2 --topology 2 1 1"; do
  lab=${t%%:*}; args=${t#*:}
  for T in 4 5; do
    run ${lab}_T$T --size 1024 1024 1024 $args --time-block $T --transport loopback --link-gbs 50 || exit 1
  done
done
echo done
