#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/calib3
mkdir -p $O
C="TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"
for v in "4 --tb-mrows 2 --tb-variant 0" "4 --tb-mrows 2 --tb-variant 4" "5 --tb-variant 4" "5 --tb-variant 0"; do
  n=$(echo $v | tr -d ' -')
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$n -o run -- python3 bench.py --steps 10 --warmup 0 --time-block $v > $O/$n.log 2>&1 || exit 1
done
echo rc=$?
