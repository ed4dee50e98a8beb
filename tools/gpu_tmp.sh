set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hybrid_gpu.py tests/test_hip_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_configs.py --only 3d-512-cpml-tfsf 3d-512-upml-tfsf 3d-512-drude --out gpurun_out/configs_hy.md > gpurun_out/configs_hy.log 2>&1; echo rc=$?; cut -c1-100 gpurun_out/configs_hy.md
