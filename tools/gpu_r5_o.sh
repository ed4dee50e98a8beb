#!/bin/bash
# Round 5: TF/SF core split into a plain inner box + face bands -- tests and 512^3 CPML / UPML + TF/SF
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hybrid_gpu.py tests/test_tfsf_tb_gpu.py -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; }
tail -1 $O/tests.log
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json --scene vacuum --use-pml --use-tfsf"
run() {
  local lab=$1; shift
  timeout -k 10 300 python -m fdtd3d_amd $C "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "$lab $(grep -o '"mcells_per_s": [0-9.]*' $O/$lab.log)"
}
run cpml_core5 --pml-type cpml --hybrid-tfsf core --hybrid-block 5
run cpml_shell5 --pml-type cpml --hybrid-tfsf shell --hybrid-block 5
run cpml_core4 --pml-type cpml --hybrid-tfsf core --hybrid-block 4
run upml_core5 --hybrid-tfsf core --hybrid-block 5
run upml_core4 --hybrid-tfsf core --hybrid-block 4
run cpml_core5b --pml-type cpml --hybrid-tfsf core --hybrid-block 5
run cpml_shell5b --pml-type cpml --hybrid-tfsf shell --hybrid-block 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pc -o run -- python3 -m fdtd3d_amd $C --pml-type cpml --hybrid-tfsf core > $O/prof.log 2>&1 && cp /tmp/pc/run_kernel_stats.csv $O/prof_core_stats.csv
echo done
