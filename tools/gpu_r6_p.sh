#!/bin/bash
# Round 6 (p): 2D launch records with the shell-stream forks / joins recorded (windows and copies on 3 streams)
# vs one stream (--shell-streams 1, the previous record form); the hybrid GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hybrid_gpu.py -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "tmz_cpml:--2d --sizex 8192 --sizey 8192 --use-pml --pml-type cpml --use-tfsf" "tmz_upml:--2d --sizex 8192 --sizey 8192 --use-pml --use-tfsf" "tez_upml:--2d --2d-mode tez --sizex 8192 --sizey 8192 --use-pml --use-tfsf"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  for rep in 1 2; do
    for m in 0 1; do
      timeout -k 10 200 python3 -m fdtd3d_amd $args --time-steps 224 --warmup-steps 14 --scene vacuum --dtype f32 --json --shell-streams $m > $O/${lab}_$m.log 2>&1 || { echo "$lab $m failed"; tail -3 $O/${lab}_$m.log; exit 1; }
    done
    echo "$lab rep $rep: 3 streams $(grep -o '"mcells_per_s": [0-9.]*' $O/${lab}_0.log | cut -d' ' -f2)  one stream $(grep -o '"mcells_per_s": [0-9.]*' $O/${lab}_1.log | cut -d' ' -f2)"
  done
done
