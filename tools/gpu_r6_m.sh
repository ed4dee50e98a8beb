#!/bin/bash
# Round 6 (m): bench.py with the whole-pass physics companions and the fp64 companions (timed end to end)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6m
mkdir -p $O
s=$(date +%s)
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
e=$(date +%s)
echo "bench wall $((e - s)) s"
tail -1 $O/bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('headline', d['value'], 'fp64', d['fp64']['value'])
for k, v in d['physics'].items(): print(k, v.get('value'), v.get('steps'), v.get('warmup'), v.get('error', ''))
"
