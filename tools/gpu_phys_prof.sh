#!/bin/bash
# steady-state kernel tables + B/cell-step of the 512^3 physics configs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
CONFIGS="cpml upml" MARKER=k_tb3d_mr PASSES=8 bash tools/gpu_prof_configs.sh || exit 1
CONFIGS="drude" MARKER=k_tb3d_mr PASSES=48 bash tools/gpu_prof_configs.sh || exit 1
bash tools/gpu_cfg_bytes.sh || exit 1
