#!/bin/bash
# Round 5: blocked Drude pass -- T sweep of the two Drude companions and per-kernel traces
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
S="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 45 --time-steps 75 --json --scene drude-sphere --use-metamaterials $S"
run() {
  local lab=$1; shift
  timeout -k 10 300 python -m fdtd3d_amd $C "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
for T in 3 4 5; do
  run drude_T$T --time-block $T || exit 1
  run drude_upml_T$T --use-pml --hybrid-block $T || exit 1
done
prof() {
  local lab=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$lab -o run -- python3 -m fdtd3d_amd $C "$@" > $O/prof_$lab.log 2>&1 || { echo "prof $lab failed"; return 0; }
  cp /tmp/p_$lab/run_kernel_stats.csv $O/prof_${lab}_stats.csv
}
prof drude_T4 --time-block 4
prof drude_T5 --time-block 5
prof drude_upml_T5 --use-pml --hybrid-block 5
echo done
