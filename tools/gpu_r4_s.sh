#!/bin/bash
# Round 4: TF/SF in the blocked core as ONE TfsfSets launch (--hybrid-tfsf core1) vs ring split (core) vs the
# stepped-shell default; whole-grid in-kernel TF/SF without PML for the variant's per-cell cost
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C512 "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
run vac_tfsf --scene vacuum --use-tfsf || exit 1
run vac_tfsf_T5 --scene vacuum --use-tfsf --time-block 5 || exit 1
run vac --scene vacuum || exit 1
for m in auto core core1; do
  run cpml_tfsf_$m --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-tfsf $m || exit 1
  run upml_tfsf_$m --scene vacuum --use-pml --use-tfsf --hybrid-tfsf $m || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_hybrid_gpu.py -x -q -k "core" --timeout 200 > $O/tests.log 2>&1; tail -1 $O/tests.log
echo done
timeout -k 10 400 python -u -m pytest tests/test_tb_gpu.py tests/test_native_gpu.py -x -q -k "f64 or 64" --timeout 200 > $O/tests64.log 2>&1 || { echo "fp64 tests failed"; tail -20 $O/tests64.log; exit 1; }
tail -1 $O/tests64.log
for a in 1 0 1; do
  FDTD3D_TB64_ALIGN=$a timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dtype f64 --fp64-companion off --physics-companion off > $O/b64_$a.log 2>&1 || { echo "bench64 failed"; tail -3 $O/b64_$a.log; exit 1; }
  echo "fp64 align=$a: $(tail -1 $O/b64_$a.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done
