#!/bin/bash
# Round 3, first GPU session: full GPU test suite, headline bench (+ tile-order A/B), physics configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/bench_$i.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print("default", d["value"], d["ms_per_step"], d.get("fp64"))' $O/bench_$i.json
done
for p in 4x8 2x16 8x4 1x32 4x4; do
  FDTD3D_TB_PATCH=$p timeout -k 10 200 python bench.py --fp64-companion off --steps 40 > $O/bench_p$p.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print("patch", sys.argv[2], d["value"], d["ms_per_step"])' $O/bench_p$p.json $p
done
timeout -k 10 200 python bench.py --fp64-companion off --steps 40 > $O/bench_d40.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print("default40", d["value"], d["ms_per_step"])' $O/bench_d40.json
timeout -k 10 600 python tools/bench_configs.py --only 3d-512-vacuum 3d-512-cpml-tfsf 3d-512-upml-tfsf 3d-512-drude 3d-512-cpml-point \
  --out $O/cfg.md > $O/cfg.log 2>&1 || { tail -5 $O/cfg.log; exit 1; }
cut -c1-150 $O/cfg.md
