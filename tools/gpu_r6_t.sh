#!/bin/bash
# Round 6 (t): the 3D hybrid shell's CPML windows of a half step in one launch per row layout (yee3d_cpml.hip
# Win3) vs one launch per window (FDTD3D_MULTI_CPML=0): hybrid / decomposed GPU tests, config 3 fp32 / fp64
# on one GPU, and the decomposed config-3 per-GPU cost (loopback), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hybrid_gpu.py tests/test_parallel_gpu.py tests/test_hip_gpu.py -k "cpml" -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--3d --sizex 512 --same-size --warmup-steps 10 --time-steps 40 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for rep in 1 2; do
  for m in 1 0; do
    FDTD3D_MULTI_CPML=$m timeout -k 10 200 python3 -m fdtd3d_amd $B --dtype f32 > $O/c3_$m.log 2>&1 || { echo "c3 $m failed"; tail -5 $O/c3_$m.log; exit 1; }
    FDTD3D_MULTI_CPML=$m timeout -k 10 200 python3 -m fdtd3d_amd $B --dtype f64 > $O/c364_$m.log 2>&1 || { echo "c364 $m failed"; tail -5 $O/c364_$m.log; exit 1; }
    FDTD3D_MULTI_CPML=$m timeout -k 10 240 python -u tools/decomp_cost.py --size 512 512 512 --world 4 --topology 2 2 1 --time-block 4 --physics cpml-tfsf --transport loopback --link-gbs 50 > $O/dc_$m.log 2>&1 || { echo "dc $m failed"; tail -5 $O/dc_$m.log; exit 1; }
    echo "rep $rep multi=$m: config 3 f32 $(grep -o '"mcells_per_s": [0-9.]*' $O/c3_$m.log | cut -d' ' -f2)  f64 $(grep -o '"mcells_per_s": [0-9.]*' $O/c364_$m.log | cut -d' ' -f2)  4-rank per GPU $(grep -o '[0-9]* Mcells/s per GPU' $O/dc_$m.log)"
  done
done
