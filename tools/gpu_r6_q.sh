#!/bin/bash
# Round 6 (q): the whole GPU suite, smoke(), the 1-GPU bench (all companions)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6Q_OUT:-r6q}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('headline', d['value'], 'fp64', d['fp64']['value'])
for k, v in d['physics'].items(): print(k, v.get('value'), v.get('error', ''))
"
