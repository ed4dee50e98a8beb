#!/bin/bash
# Round 6 (j): TF/SF corrections in the fp64 blocked kernel (yee3d_tb64.hip tf_fix): GPU tests, then fp64 512^3
# CPML / UPML + TF/SF with the faces in the blocked core vs in the stepped shell (alternating), kernel traces
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tfsf_tb_gpu.py tests/test_hybrid_gpu.py -k "f64 or test_tfsf" -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C64="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 8 --time-steps 32 --json --scene vacuum --use-pml --use-tfsf"
for rep in 1 2; do
  for m in cpml upml; do
    for f in core shell; do
      timeout -k 10 200 python3 -m fdtd3d_amd $C64 --pml-type $m --hybrid-tfsf $f > $O/r64_${m}_$f.log 2>&1 || { echo "r64 $m $f failed"; tail -5 $O/r64_${m}_$f.log; exit 1; }
      echo "rep $rep f64 $m + TF/SF faces in the $f: $(grep -o '"mcells_per_s": [0-9.]*' $O/r64_${m}_$f.log | cut -d' ' -f2)"
    done
  done
done
for m in cpml upml; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t64$m -o run -- python3 -m fdtd3d_amd $C64 --pml-type $m --hybrid-tfsf core > $O/kt_$m.log 2>&1 && cp /tmp/t64$m/run_kernel_stats.csv $O/kt64_${m}_core.csv || { echo "kt $m failed"; exit 1; }
done
V64="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 8 --time-steps 32 --json --scene vacuum --use-tfsf"
timeout -k 10 200 python3 -m fdtd3d_amd $V64 > $O/v64.log 2>&1 || { echo "v64 failed"; tail -5 $O/v64.log; exit 1; }
echo "f64 vacuum + TF/SF (blocked passes): $(grep -o '"mcells_per_s": [0-9.]*' $O/v64.log | cut -d' ' -f2)"
