#!/bin/bash
# Round 6 (r): per-GPU cost of decomposed config 3 (512^3 CPML + TF/SF, hybrid passes) on 2 / 4 / 8 ranks,
# one rank's sub-domain on one GPU with the loopback transport; a kernel trace of the 4-rank case
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6r
mkdir -p $O
for t in "2:--world 2 --topology 2 1 1" "4:--world 4 --topology 2 2 1" "8:--world 8 --topology 4 2 1"; do
  lab=${t%%:*}; args=${t#*:}
  for T in 4 5; do
    timeout -k 10 240 python -u tools/decomp_cost.py --size 512 512 512 $args --time-block $T --physics cpml-tfsf --transport loopback --link-gbs 50 > $O/c3_${lab}_T$T.log 2>&1 || { echo "$lab T$T failed"; tail -5 $O/c3_${lab}_T$T.log; exit 1; }
    echo "== $lab ranks T=$T"; grep -h "per pass\|Mcells" $O/c3_${lab}_T$T.log
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tdc -o run -- python3 -u tools/decomp_cost.py --size 512 512 512 --world 4 --topology 2 2 1 --time-block 5 --physics cpml-tfsf --transport loopback --link-gbs 50 > $O/kt.log 2>&1 && cp /tmp/tdc/run_kernel_stats.csv $O/kt_c3_4.csv || { echo kt failed; exit 1; }
