#!/bin/bash
# Kernel traces of the hybrid-blocked 512^3 CPML + TF/SF and UPML + TF/SF runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/prof_hybrid
mkdir -p $O
C="-m fdtd3d_amd --3d --sizex 512 --same-size --dtype f32 --warmup-steps 8 --time-steps 48 --scene vacuum --use-pml --use-tfsf --json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/cpml -o run -- python3 $C --pml-type cpml > $O/cpml.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/upml -o run -- python3 $C > $O/upml.log 2>&1
echo rc=$?
