#!/bin/bash
# Round 3 GPU session: GPU tests, headline bench (+ tile-order A/B), physics configs, CPML/UPML kernel profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
PHASE=${1:-all}
if [ "$PHASE" = all ] || [ "$PHASE" = tests ]; then
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && exit $rc
fi
bench() {  # label, env..., args
  local lab=$1; shift
  timeout -k 10 200 env "$@" > $O/b_$lab.json 2> $O/bench.err || { tail $O/bench.err; return 1; }
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["value"], d["ms_per_step"], d.get("fp64", {}).get("value"))' $O/b_$lab.json $lab
}
if [ "$PHASE" = all ] || [ "$PHASE" = bench ]; then
bench default python bench.py || exit 1
bench d40 python bench.py --fp64-companion off --steps 40 || exit 1
for p in 4x8 2x16 8x4 1x32; do
  bench p$p FDTD3D_TB_PATCH=$p python bench.py --fp64-companion off --steps 40 || exit 1
done
fi
[ "$PHASE" = tests ] || [ "$PHASE" = bench ] && exit 0
timeout -k 10 600 python tools/bench_configs.py --only 3d-512-vacuum 3d-512-cpml-tfsf 3d-512-upml-tfsf 3d-512-drude 3d-512-cpml-point \
  --out $O/cfg.md > $O/cfg.log 2>&1 || { tail -5 $O/cfg.log; exit 1; }
cut -c1-150 $O/cfg.md
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json"
prof() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run -- python3 -m fdtd3d_amd $C512 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; return 1; }
  grep '^{' $O/$name.log | cut -c1-200
  python3 tools/prof_summary.py $(find $O/$name -name '*results.db' | head -1) --marker k_tb3d --passes 8 > $O/${name}_steady.md 2>&1
  rm -rf $O/$name
}
prof cpml --scene vacuum --use-pml --pml-type cpml --use-tfsf || exit 1
prof upml --scene vacuum --use-pml --use-tfsf || exit 1
head -30 $O/cpml_steady.md
head -30 $O/upml_steady.md
