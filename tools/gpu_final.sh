#!/bin/bash
# Round-end measurement: bench.py (fp32 / fp64), every bench config, steady-state kernel tables.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/bench_f32_$i.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  cat $O/bench_f32_$i.json
done
timeout -k 10 200 python bench.py --dtype f64 > $O/bench_f64.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench_f64.json
timeout -k 10 900 python tools/bench_configs.py --out $O/configs.md > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
cat $O/configs.md
