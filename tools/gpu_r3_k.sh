#!/bin/bash
# bench.py steadiness: the driver's 20 / 5 setting three times back to back, then 100 / 10
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --fp64-companion off > $O/b$i.json 2> $O/b$i.err || { tail $O/b$i.err; exit 1; }
  echo "20/5 run $i: $(python3 -c "import json;d=json.load(open('$O/b$i.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --fp64-companion off > $O/b100.json 2> $O/b100.err || { tail $O/b100.err; exit 1; }
echo "100/10: $(python3 -c "import json;d=json.load(open('$O/b100.json'));print(d['value'], d['ms_per_step'])")"
