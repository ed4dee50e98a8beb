#!/bin/bash
# Round 6 (aa): decomposed UPML + TF/SF per-GPU cost breakdown (2x2x1 and 4x2x1, loopback; no exchange) and a
# kernel trace of the 2x2x1 rank; the listed-exchange bitwise GPU test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_parallel_gpu.py -k "listed" -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in "4:--world 4 --topology 2 2 1" "8:--world 8 --topology 4 2 1"; do
  lab=${t%%:*}; args=${t#*:}
  for v in "loop:--transport loopback --link-gbs 50" "skip:--transport null --skip-exchange"; do
    vl=${v%%:*}; va=${v#*:}
    timeout -k 10 240 python -u tools/decomp_cost.py --size 512 512 512 $args --time-block 4 --physics upml-tfsf $va > $O/u_${lab}_$vl.log 2>&1 || { echo "$lab $vl failed"; tail -5 $O/u_${lab}_$vl.log; exit 1; }
    echo "== $lab ranks $vl"; grep -h "per pass\|Mcells" $O/u_${lab}_$vl.log
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tu -o run -- python3 -u tools/decomp_cost.py --size 512 512 512 --world 4 --topology 2 2 1 --time-block 4 --physics upml-tfsf --transport loopback --link-gbs 50 > $O/kt.log 2>&1 && cp /tmp/tu/run_kernel_stats.csv $O/kt_u4.csv || { echo kt failed; exit 1; }
