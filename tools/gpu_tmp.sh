set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_check.sh && bash tools/gpu_multirank.sh
