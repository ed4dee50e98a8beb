#!/bin/bash
# Round 4: steady-state kernel breakdown of 512^3 Drude sphere + UPML (300 steps so the set-up kernels are a
# small share)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4dprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m fdtd3d_amd --3d --sizex 512 \
  --same-size --dtype f32 --warmup-steps 10 --time-steps 300 --json --scene drude-sphere --use-metamaterials \
  --use-pml --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128 \
  > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
db=$(ls $O/prof/*.db | head -1)
python3 tools/rocpd_stats.py "$db" --top 30 > $O/stats.md 2>&1
grep -h '^{' $O/prof.log | tail -1
echo done
