#!/bin/bash
# Round 6 (s): Python-side cost of a decomposed config-3 pass (cProfile of one rank's sub-domain run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 300 python -u -m cProfile -o $O/c3_4.prof tools/decomp_cost.py --size 512 512 512 --world 4 --topology 2 2 1 --time-block 5 --physics cpml-tfsf --transport loopback --link-gbs 50 --steps 40 > $O/c3_4.log 2>&1 || { echo failed; tail -5 $O/c3_4.log; exit 1; }
grep Mcells $O/c3_4.log
python3 -c "
import pstats
p = pstats.Stats('$O/c3_4.prof')
p.sort_stats('tottime').print_stats(30)
" > $O/c3_4_stats.txt
head -60 $O/c3_4_stats.txt | tail -45
