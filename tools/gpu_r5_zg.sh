#!/bin/bash
# Round 5: one Drude + UPML pass, native vs Python, from kernel traces
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zg
mkdir -p $O
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 20 --time-steps 36 --scene drude-sphere --use-metamaterials --use-pml $S"
for drv in nat py; do
  if [ $drv = nat ]; then P="./fdtd3d_amd/fdtd3d"; else P="python3 -m fdtd3d_amd"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pt_$drv -o run -- $P $C > $O/prof_$drv.log 2>&1 || { echo "prof $drv failed"; tail -3 $O/prof_$drv.log; continue; }
  f=$(find /tmp/pt_$drv -name 'run_kernel_trace.csv' | head -1)
  python3 tools/trace_pass.py "$f" --list > $O/pass_$drv.txt
  echo "== $drv"; grep -A30 "^ *[0-9]* *[0-9.]* us" $O/pass_$drv.txt | head -0; python3 tools/trace_pass.py "$f"
done
