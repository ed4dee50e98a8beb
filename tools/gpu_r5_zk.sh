#!/bin/bash
# Round 5: fp64 XCD patch order 2x8 as the default (A/B vs z fastest) + the GPU suite; fp32 headline patch sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5zk
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  --deselect "tests/test_native_gpu.py::test_native_checkpoint_roundtrip" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py $B > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 0; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*')"
}
B="--dtype f64 --steps 12 --warmup 4 --fp64-companion off --physics-companion off"
for r in 1 2; do run f64_def_$r A=1; run f64_z_$r FDTD3D_TB64_PATCH=0x0; done
B="--steps 20 --warmup 5 --fp64-companion off --physics-companion off"
for r in 1 2; do
  run f32_base_$r A=1
  for p in 2x8 2x4 4x4 1x8; do run f32_p${p}_$r FDTD3D_TB_PATCH=$p; done
done
