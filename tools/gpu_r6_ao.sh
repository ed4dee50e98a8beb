#!/bin/bash
# Round 6 (ao): native --parallel-grid physics -- kernel trace of 512^3 fp32 CPML + TF/SF on 2x2x1 ranks of one GPU
# (split half steps, face exchanges) next to the single-rank hybrid run; Drude + UPML on 2x1x2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6ao
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f32 --time-steps 24 --warmup-steps 4 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
D="--3d --sizex 512 --same-size --dtype f32 --time-steps 24 --warmup-steps 4 --json --scene drude-sphere --use-metamaterials --use-pml --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
timeout -k 10 200 fdtd3d_amd/fdtd3d $C > $O/c3_one.log 2>&1 || { echo one failed; tail -3 $O/c3_one.log; exit 1; }
timeout -k 10 200 fdtd3d_amd/fdtd3d $C --parallel-grid --topology-sizex 2 --topology-sizey 2 > $O/c3_221.log 2>&1 || { echo 221 failed; tail -3 $O/c3_221.log; exit 1; }
timeout -k 10 200 fdtd3d_amd/fdtd3d $D --parallel-grid --topology-sizex 2 --topology-sizez 2 > $O/du_212.log 2>&1 || { echo du failed; tail -3 $O/du_212.log; exit 1; }
timeout -k 10 200 fdtd3d_amd/fdtd3d $D > $O/du_one.log 2>&1 || { echo du1 failed; tail -3 $O/du_one.log; exit 1; }
for f in c3_one c3_221 du_212 du_one; do echo "$f $(grep -E 'Throughput' $O/$f.log)"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_ao -o run -- fdtd3d_amd/fdtd3d $C --parallel-grid --topology-sizex 2 --topology-sizey 2 > $O/kt.log 2>&1 && cp /tmp/t_ao/run_kernel_stats.csv $O/kt_c3_221_stats.csv || { echo "kt failed"; exit 1; }
echo done
