#!/bin/bash
# GPU tests of the split / chain / hybrid paths, then the 512^3 physics configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_gpu.py tests/test_hybrid_gpu.py tests/test_parallel_gpu.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
tail -3 gpurun_out/t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_configs.py --only ${CFGS:-3d-512-drude-nopml 3d-512-drude 3d-512-upml-tfsf 3d-512-cpml-tfsf} \
  --out gpurun_out/cfg.md > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
cut -c1-130 gpurun_out/cfg.md
