#!/bin/bash
# Round 5: the Drude box inside the blocked passes (tb3d_mr.h DrDev) -- GPU tests, the two Drude
# companions (blocked vs the stepped dispersive box), a kernel trace of each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
true || timeout -k 10 600 python -u -m pytest tests -m gpu -k "drude or Drude" -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; }
tail -1 $O/tests.log
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json --scene drude-sphere --use-metamaterials $S"
run() {
  local lab=$1; shift
  timeout -k 10 300 python -m fdtd3d_amd $C "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["mcells_per_s"], d.get("time_steps"))')"
}
run drude_blk || exit 1
run drude_off --blocked-drude off || exit 1
run drude_upml_blk --use-pml || exit 1
run drude_upml_off --use-pml --blocked-drude off || exit 1
run drude_blk_T4 --time-block 4 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_drude -o run -- python3 -m fdtd3d_amd $C > $O/prof_drude.log 2>&1 || echo "prof failed"
cp /tmp/prof_drude/*/run_kernel_stats.csv $O/prof_drude_stats.csv 2>/dev/null || find /tmp/prof_drude -name "*stats*" | head
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_drude_upml -o run -- python3 -m fdtd3d_amd $C --use-pml > $O/prof_drude_upml.log 2>&1 || echo "prof failed"
cp /tmp/prof_drude_upml/*/run_kernel_stats.csv $O/prof_drude_upml_stats.csv 2>/dev/null || find /tmp/prof_drude_upml -name "*stats*" | head
echo done
