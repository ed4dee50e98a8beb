#!/bin/bash
# Round 5: where a decomposed 1024^3 4x2x1 pass goes -- null vs loopback transport, kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5x
mkdir -p $O
A="--size 1024 1024 1024 --world 8 --topology 4 2 1 --time-block 4"
timeout -k 10 240 python -u tools/decomp_cost.py $A --transport null > $O/null.log 2>&1 || { echo null failed; tail -5 $O/null.log; exit 1; }
grep -h "per pass\|decomposed" $O/null.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_x -o run -- python3 -u tools/decomp_cost.py $A --transport loopback --link-gbs 50 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
grep -h "per pass\|decomposed" $O/prof.log
f=$(find /tmp/p_x -name 'run_kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv
f=$(find /tmp/p_x -name 'run_kernel_trace.csv' | head -1); python3 - "$f" > $O/trace_summary.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print("%s|%s|%s|%s|%s" % (r["Kernel_Name"][:80], r.get("Grid_Size_X", r.get("Grid_Size", "")),
          int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", "")))
PY
rm -rf /tmp/p_x
echo done
