#!/bin/bash
# Round 5: headline A/B on one box -- the session-start library (libfdtd3d_hip_base.so) vs HEAD, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
B="--steps 20 --warmup 5 --physics-companion off --fp64-companion off"
for r in 1 2; do
  FDTD3D_HIP_LIB=$PWD/fdtd3d_amd/libfdtd3d_hip_base.so timeout -k 10 300 python bench.py $B > $O/base$r.log 2>&1 || { echo base failed; tail -3 $O/base$r.log; exit 1; }
  echo "base $r $(tail -1 $O/base$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  timeout -k 10 300 python bench.py $B > $O/head$r.log 2>&1 || { echo head failed; tail -3 $O/head$r.log; exit 1; }
  echo "head $r $(tail -1 $O/head$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done
