set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_decomp.sh 2>&1 | grep -v "^topology" | tail -14
