#!/bin/bash
# Round 5: native --parallel-grid with the ghost pulls overlapped with the interior pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zc
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_native_gpu.py -k "parallel" -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in "1:--topology-sizex 1" "4_x:--topology-sizex 4" "4_xy:--topology-sizex 2 --topology-sizey 2"; do
  lab=${t%%:*}; args=${t#*:}
  timeout -k 10 200 ./fdtd3d_amd/fdtd3d --3d --sizex 512 --same-size --dtype f32 --scene vacuum --time-steps 60 --warmup-steps 20 --time-block 4 --parallel-grid $args > $O/nat_$lab.log 2>&1 || { echo nat $lab failed; tail -5 $O/nat_$lab.log; exit 1; }
  echo "== native 512^3 $lab (ranks on one GPU)"; grep -h "Throughput" $O/nat_$lab.log
done
