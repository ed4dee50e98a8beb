#!/bin/bash
# Round 6 (f): fp64 split updates on double4 lanes (FDTD3D_F64_V4=1) vs the scalar kernels, 512^3 UPML / CPML +
# TF/SF and the stepped vacuum; the vacuum GPU tests over nz % 4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_gpu.py tests/test_hybrid_gpu.py -k "vacuum_3d or f64 or drude_3d" -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
tail -1 $O/tests.log
U="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 8 --time-steps 24 --json --scene vacuum --use-pml --use-tfsf"
for rep in 1 2; do
  for v in 1 0; do
    FDTD3D_F64_V4=$v timeout -k 10 200 python3 -m fdtd3d_amd $U > $O/u_$v.log 2>&1 || { echo "u $v failed"; exit 1; }
    FDTD3D_F64_V4=$v timeout -k 10 200 python3 -m fdtd3d_amd $U --pml-type cpml > $O/c_$v.log 2>&1 || { echo "c $v failed"; exit 1; }
    FDTD3D_F64_V4=$v timeout -k 10 200 python3 -m fdtd3d_amd --3d --sizex 512 --same-size --dtype f64 --warmup-steps 4 --time-steps 20 --json --scene vacuum --split-kernels > $O/v_$v.log 2>&1 || { echo "v $v failed"; exit 1; }
    echo "rep $rep f64_v4=$v: upml+tfsf $(grep -o '"mcells_per_s": [0-9.]*' $O/u_$v.log | cut -d' ' -f2)  cpml+tfsf $(grep -o '"mcells_per_s": [0-9.]*' $O/c_$v.log | cut -d' ' -f2)  vacuum split $(grep -o '"mcells_per_s": [0-9.]*' $O/v_$v.log | cut -d' ' -f2)"
  done
done
FDTD3D_F64_V4=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_u64 -o run -- python3 -m fdtd3d_amd $U > $O/kt_u64.log 2>&1 && cp /tmp/t_u64/run_kernel_stats.csv $O/kt_u64.csv || { echo "kt failed"; exit 1; }
# amplitude mode: the AMP variant's 16 x 2 tiles (128-VGPR cap, spills) vs 8 x 2 tiles (FDTD3D_TB_AMP_SHAPE=2)
for sh in 0 2; do
  FDTD3D_TB_AMP_SHAPE=$sh timeout -k 10 300 python -u tools/amp_bench.py 512 96 f32 > $O/amp_$sh.log 2>&1 || { echo "amp $sh failed"; tail -3 $O/amp_$sh.log; exit 1; }
  echo "amp shape $sh:"; grep "blocked T = 3\|automatic" $O/amp_$sh.log
done
