#!/bin/bash
# fp64 blocked kernel: tile patch order A/B (FDTD3D_TB64_PATCH) on bench.py --dtype f64, and T 4 vs 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/f64
mkdir -p $O
b() {
  local lab=$1; shift
  timeout -k 10 200 env "$@" > $O/$lab.json 2> $O/$lab.err || { echo "$lab failed"; tail -3 $O/$lab.err; return 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["value"], d["ms_per_step"])' $O/$lab.json $lab
}
b base python3 bench.py --dtype f64 --steps 16 --warmup 4 || exit 1
for p in 4x4 2x8 8x2 4x8 1x8 2x4; do
  b p$p FDTD3D_TB64_PATCH=$p python3 bench.py --dtype f64 --steps 16 --warmup 4 || exit 1
done
b t5 python3 bench.py --dtype f64 --steps 20 --warmup 5 --time-block 5 || exit 1
b base2 python3 bench.py --dtype f64 --steps 16 --warmup 4 || exit 1
