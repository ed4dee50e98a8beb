#!/bin/bash
# Round 6 (c): the whole GPU suite; non-dispersive UPML chain with one component per thread (k_chain3d_c, no SGPR spills) against
# the three-component kernel (FDTD3D_CHAIN_SPLIT=0), alternating on one box; the UPML / Drude GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
DU="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 12 --time-steps 40 --json --scene drude-sphere --use-metamaterials --use-pml --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
UT="--3d --sizex 512 --same-size --warmup-steps 10 --time-steps 30 --json --scene vacuum --use-pml --use-tfsf"
for rep in 1 2; do
  for sp in 1 0; do
    FDTD3D_CHAIN_SPLIT=$sp timeout -k 10 200 python3 -m fdtd3d_amd $DU > $O/du_$sp.log 2>&1 || { echo "du $sp failed"; tail -5 $O/du_$sp.log; exit 1; }
    FDTD3D_CHAIN_SPLIT=$sp timeout -k 10 200 python3 -m fdtd3d_amd $UT --dtype f32 > $O/ut32_$sp.log 2>&1 || { echo "ut32 $sp failed"; exit 1; }
    FDTD3D_CHAIN_SPLIT=$sp timeout -k 10 200 python3 -m fdtd3d_amd $UT --dtype f64 > $O/ut64_$sp.log 2>&1 || { echo "ut64 $sp failed"; exit 1; }
    echo "rep $rep split=$sp: drude+upml $(grep -o '"mcells_per_s": [0-9.]*' $O/du_$sp.log | cut -d' ' -f2)  upml+tfsf f32 $(grep -o '"mcells_per_s": [0-9.]*' $O/ut32_$sp.log | cut -d' ' -f2)  f64 $(grep -o '"mcells_per_s": [0-9.]*' $O/ut64_$sp.log | cut -d' ' -f2)"
  done
done
FDTD3D_CHAIN_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_du -o run -- python3 -m fdtd3d_amd $DU > $O/ktdu.log 2>&1 && cp /tmp/t_du/run_kernel_stats.csv $O/kt_du_split.csv || { echo "ktdu failed"; exit 1; }
# config 3 with the TF/SF faces in the core at T = 4 (the TF/SF variant spills VGPRs at T = 5) vs the shell form
C3="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 40 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for rep in 1 2; do
  for v in "core 4" "core 5" "shell 5" "shell 4"; do
    set -- $v
    timeout -k 10 200 python3 -m fdtd3d_amd $C3 --hybrid-tfsf $1 --hybrid-block $2 > $O/c3_$1_$2.log 2>&1 || { echo "c3 $v failed"; exit 1; }
    echo "rep $rep config 3 faces in $1, T=$2: $(grep -o '"mcells_per_s": [0-9.]*' $O/c3_$1_$2.log | cut -d' ' -f2)"
  done
done
