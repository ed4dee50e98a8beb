#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/decomp.log
while read -r args; do
  [ -z "$args" ] && continue
  echo "== $args" >> gpurun_out/decomp.log
  timeout -k 10 200 python tools/decomp_cost.py $args >> gpurun_out/decomp.log 2>&1 || { tail -5 gpurun_out/decomp.log; exit 1; }
done <<'LIST'
--world 8 --axes xy --time-block 5
--world 8 --axes xy --time-block 4
--world 8 --axes xy --time-block 3
--world 4 --axes xy --time-block 5
--world 4 --axes xy --time-block 4
--world 2 --axes xy --time-block 5
--world 2 --axes xy --time-block 4
LIST
grep -v amdgpu.ids gpurun_out/decomp.log
