#!/bin/bash
# Round 4 close: the driver's default bench command three times back to back on one box, plus
# rocm-smi clocks, to separate box-to-box spread from run-to-run spread
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4rep
mkdir -p $O
rocm-smi --showclocks > $O/clocks.txt 2>&1 || true
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --physics-companion off --fp64-companion off > $O/b$i.log 2>&1 || { echo "run $i failed"; tail $O/b$i.log; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d["value"], d["ms_per_step"])' $O/b$i.log
done
grep -iE "sclk|mclk" $O/clocks.txt | head -4 || true
