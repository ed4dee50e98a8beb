#!/bin/bash
# Round 6 (u): where a decomposed config-3 pass goes: loopback vs null transport vs no exchange at all
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6u
mkdir -p $O
A="--size 512 512 512 --world 4 --topology 2 2 1 --time-block 4 --physics cpml-tfsf"
for v in "loop:--transport loopback --link-gbs 50" "null:--transport null" "skip:--transport null --skip-exchange"; do
  lab=${v%%:*}; args=${v#*:}
  timeout -k 10 240 python -u tools/decomp_cost.py $A $args > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -5 $O/$lab.log; exit 1; }
  echo "== $lab"; grep -h "per pass\|Mcells" $O/$lab.log
done
A8="--size 1024 1024 1024 --world 8 --topology 4 2 1 --time-block 4"
for v in "loop:--transport loopback --link-gbs 50" "skip:--transport null --skip-exchange"; do
  lab=${v%%:*}; args=${v#*:}
  timeout -k 10 240 python -u tools/decomp_cost.py $A8 $args > $O/v8_$lab.log 2>&1 || { echo "v8 $lab failed"; tail -5 $O/v8_$lab.log; exit 1; }
  echo "== vacuum 8 ranks $lab"; grep -h "per pass\|decomposed" $O/v8_$lab.log
done
