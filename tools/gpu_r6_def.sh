#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r6_f.sh && bash tools/gpu_r6_e.sh && bash tools/gpu_r6_d.sh
