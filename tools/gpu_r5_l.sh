#!/bin/bash
# Round 5: per-kernel stats of the Drude + UPML companion through both drivers
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5l
mkdir -p $O
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json --scene drude-sphere --use-metamaterials --use-pml $S"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pn -o run -- ./fdtd3d_amd/fdtd3d $C > $O/nat.log 2>&1 && cp /tmp/pn/run_kernel_stats.csv $O/nat_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pp -o run -- python3 -m fdtd3d_amd $C > $O/py.log 2>&1 && cp /tmp/pp/run_kernel_stats.csv $O/py_stats.csv
echo done
