#!/bin/bash
# Round 5: decomposed 1024^3 passes, T-thick shell slabs in order vs side by side on 3 streams
# (loopback transport, 50 GB/s emulated link), plus a kernel trace of the 4x2x1 rank
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5w
mkdir -p $O
run() {
  local lab=$1; shift
  timeout -k 10 240 python -u tools/decomp_cost.py "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "== $lab"; tail -2 $O/$lab.log
}
for t in "8_421:--world 8 --topology 4 2 1" "4_221:--world 4 --topology 2 2 1" "8_222:--world 8 --topology 2 2 2 --size 2048 1024 1024"; do
  lab=${t%%:*}; args=${t#*:}
  for ss in 1 3; do
    run ${lab}_s$ss --size 1024 1024 1024 $args --time-block 4 --transport loopback --link-gbs 50 --shell-streams $ss || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u tools/decomp_cost.py --size 1024 1024 1024 --world 8 --topology 4 2 1 --time-block 4 --transport loopback --link-gbs 50 --shell-streams 3 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
f=$(ls $O/prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cp "$f" $O/kernel_stats_421.csv
rm -rf $O/prof
echo done
