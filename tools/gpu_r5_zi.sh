#!/bin/bash
# Round 5: decomposed hybrid passes with the deep-halo shell windows on the shell streams
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zi
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_parallel_gpu.py -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
tail -1 $O/tests.log
for ph in cpml-tfsf upml-tfsf; do
  for ss in 1 3; do
    timeout -k 10 300 python -u tools/decomp_cost.py --size 512 512 512 --world 4 --topology 2 2 1 --time-block 4 --physics $ph --transport loopback --link-gbs 50 --shell-streams $ss > $O/${ph}_$ss.log 2>&1 || { echo $ph $ss failed; tail -5 $O/${ph}_$ss.log; exit 1; }
    echo "== $ph streams $ss"; grep -h "Mcells" $O/${ph}_$ss.log
  done
done
