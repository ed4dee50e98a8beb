#!/bin/bash
# B/cell-step of the 512^3 physics configs: FETCH_SIZE / WRITE_SIZE passes of a
# short (20) and a long (60 step) run each; tools/cfg_bytes.py takes the difference.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/cfg_bytes
mkdir -p $O
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 0 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local name=$1; shift
  for n in 20 60; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 180 rocprofv3 --pmc $ctr -d $O/$name/$ctr$n -o run -- python3 -m fdtd3d_amd $C512 --time-steps $n "$@" \
        > $O/$name.$ctr$n.log 2>&1 || { echo "$name $ctr $n failed"; tail -5 $O/$name.$ctr$n.log; return 1; }
    done
  done
  db() { find $O/$name/$1 -name '*results.db' | head -1; }
  python3 tools/cfg_bytes.py --cells 134217728 --steps 20 60 --title "$name" \
    --fetch $(db FETCH_SIZE20) $(db FETCH_SIZE60) --write $(db WRITE_SIZE20) $(db WRITE_SIZE60) > $O/$name.md
  cat $O/$name.md
  rm -rf $O/$name
}
for n in ${CONFIGS:-cpml upml drude}; do
  case $n in
    cpml) run cpml --scene vacuum --use-pml --pml-type cpml --use-tfsf ;;
    upml) run upml --scene vacuum --use-pml --use-tfsf ;;
    drude) run drude --scene drude-sphere --use-metamaterials --use-pml $SPH ;;
    drudenopml) run drudenopml --scene drude-sphere --use-metamaterials $SPH ;;
    sphere) run sphere --scene sphere --sphere-eps 4 $SPH ;;
    vac) run vac --scene vacuum ;;
  esac || exit 1
done
