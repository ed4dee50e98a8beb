#!/bin/bash
# Round 6: decomposition repeats (r6d) then the headline PMC refresh and 2D Python / native traces (r6e)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r6_e.sh && bash tools/gpu_r6_d.sh
