#!/bin/bash
# Round 6 (l): the fp64 Drude pass (yee3d_tb64.hip DrDev64): GPU tests, then fp64 512^3 Drude sphere r = 128
# without / with UPML, blocked Drude pass vs the stepped dispersive box (alternating), kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_drude_blk_gpu.py -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
D="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 8 --time-steps 32 --json --scene drude-sphere --use-metamaterials --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
for rep in 1 2; do
  for pml in "" "--use-pml"; do
    for b in on off; do
      lab="${pml:+upml}_$b"
      timeout -k 10 300 python3 -m fdtd3d_amd $D $pml --blocked-drude $b > $O/d64_$lab.log 2>&1 || { echo "d64 $lab failed"; tail -5 $O/d64_$lab.log; exit 1; }
      echo "rep $rep f64 Drude ${pml:-nopml} blocked-drude=$b: $(grep -o '"mcells_per_s": [0-9.]*' $O/d64_$lab.log | cut -d' ' -f2)"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/td64 -o run -- python3 -m fdtd3d_amd $D --use-pml > $O/kt.log 2>&1 && cp /tmp/td64/run_kernel_stats.csv $O/kt_d64_upml.csv || { echo "kt failed"; exit 1; }
