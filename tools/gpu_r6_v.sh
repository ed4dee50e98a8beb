#!/bin/bash
# Round 6 (v): the direct exchange from a cached plan with one pack / unpack launch (parallel/halo.py
# _exchange_direct_listed) vs per message and array (FDTD3D_HALO_LISTED=0): decomposed GPU tests incl. the real
# RCCL self-exchange, decomposed config 3 per GPU and the 8-rank vacuum per GPU (loopback), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parallel_gpu.py tests/test_rccl_gpu.py -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for m in 1 0; do
    FDTD3D_HALO_LISTED=$m timeout -k 10 240 python -u tools/decomp_cost.py --size 512 512 512 --world 4 --topology 2 2 1 --time-block 4 --physics cpml-tfsf --transport loopback --link-gbs 50 > $O/c3_$m.log 2>&1 || { echo "c3 $m failed"; tail -5 $O/c3_$m.log; exit 1; }
    FDTD3D_HALO_LISTED=$m timeout -k 10 240 python -u tools/decomp_cost.py --size 512 512 512 --world 8 --topology 4 2 1 --time-block 4 --physics upml-tfsf --transport loopback --link-gbs 50 > $O/u8_$m.log 2>&1 || { echo "u8 $m failed"; tail -5 $O/u8_$m.log; exit 1; }
    FDTD3D_HALO_LISTED=$m timeout -k 10 240 python -u tools/decomp_cost.py --size 1024 1024 1024 --world 8 --topology 4 2 1 --time-block 4 --transport loopback --link-gbs 50 > $O/v8_$m.log 2>&1 || { echo "v8 $m failed"; tail -5 $O/v8_$m.log; exit 1; }
    echo "rep $rep listed=$m: c3 2x2x1 $(grep -o '[0-9]* Mcells/s per GPU' $O/c3_$m.log)  upml-tfsf 4x2x1 $(grep -o '[0-9]* Mcells/s per GPU' $O/u8_$m.log)  vacuum 1024^3 4x2x1 $(grep -o '([0-9]* Mcells/s per GPU' $O/v8_$m.log)"
  done
done
grep -h "per pass" $O/c3_1.log $O/c3_0.log
