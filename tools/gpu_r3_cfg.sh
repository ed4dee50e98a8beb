#!/bin/bash
# Round-3 end-of-session config table (every bench config, one process each) + bench.py f32 / f64.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/cfg_r3
mkdir -p $O
timeout -k 10 1000 python tools/bench_configs.py --out $O/configs.md > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
cat $O/configs.md
