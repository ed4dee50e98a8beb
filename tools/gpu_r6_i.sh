#!/bin/bash
# Round 6 (i): config 3 with the TF/SF faces in the blocked core: x chunk of the TF/SF variant's core pass
# (FDTD3D_TF_XCHUNK: more, shorter workgroups so the dearer face tiles stop setting a one-round pass's length)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 40 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for rep in 1 2; do
  timeout -k 10 200 python3 -m fdtd3d_amd $C --hybrid-tfsf shell > $O/shell.log 2>&1 || { echo "shell failed"; tail -5 $O/shell.log; exit 1; }
  echo "rep $rep shell: $(grep -o '"mcells_per_s": [0-9.]*' $O/shell.log | cut -d' ' -f2)"
  for xc in 0 240 160 120 96 64; do
    FDTD3D_TF_XCHUNK=$xc timeout -k 10 200 python3 -m fdtd3d_amd $C --hybrid-tfsf core > $O/core_$xc.log 2>&1 || { echo "core $xc failed"; tail -5 $O/core_$xc.log; exit 1; }
    echo "rep $rep core xchunk=$xc: $(grep -o '"mcells_per_s": [0-9.]*' $O/core_$xc.log | cut -d' ' -f2)"
  done
done
for xc in 0 120; do
  FDTD3D_TF_XCHUNK=$xc timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_$xc -o run -- python3 -m fdtd3d_amd $C --hybrid-tfsf core > $O/kt_$xc.log 2>&1 && cp /tmp/t_$xc/run_kernel_stats.csv $O/kt_core_$xc.csv || { echo "kt $xc failed"; exit 1; }
  grep -h "k_tb3d_mr" $O/kt_core_$xc.csv | cut -c1-200
done
