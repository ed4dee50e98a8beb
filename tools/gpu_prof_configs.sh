#!/bin/bash
# Kernel-trace profiles of the non-vacuum 512^3 configs (python -m fdtd3d_amd):
# per-kernel tables (tools/prof_summary.py) land in gpurun_out/prof_cfg/*.md;
# the rocpd databases are deleted (too big to copy back).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/prof_cfg
mkdir -p $O
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run -- python3 -m fdtd3d_amd $C512 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; return 1; }
  grep '^{' $O/$name.log | cut -c1-300
  python3 tools/prof_summary.py $(find $O/$name -name '*results.db' | head -1) --cells 134217728 > $O/$name.md 2>&1
  python3 tools/prof_summary.py $(find $O/$name -name '*results.db' | head -1) --marker ${MARKER:-k_tb3d} --passes ${PASSES:-8} > $O/${name}_steady.md 2>&1
  rm -rf $O/$name
}
for n in ${CONFIGS:-cpml upml drude sphere}; do
  case $n in
    cpml) run cpml --scene vacuum --use-pml --pml-type cpml --use-tfsf ;;
    cpml3) run cpml3 --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-block 3 ;;
    cpml5) run cpml5 --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-block 5 ;;
    cpmlsph) run cpmlsph --scene sphere --sphere-eps 4 $SPH --use-pml --pml-type cpml --use-tfsf ;;
    upml) run upml --scene vacuum --use-pml --use-tfsf ;;
    drude) run drude --scene drude-sphere --use-metamaterials --use-pml $SPH ;;
    drudenopml) run drudenopml --scene drude-sphere --use-metamaterials $SPH ;;
    sphere) run sphere --scene sphere --sphere-eps 4 $SPH ;;
    sphere3) run sphere3 --scene sphere --sphere-eps 4 $SPH --time-block 3 ;;
    sphere4) run sphere4 --scene sphere --sphere-eps 4 $SPH --time-block 4 ;;
    sphere5) run sphere5 --scene sphere --sphere-eps 4 $SPH --time-block 5 ;;
    vac) run vac --scene vacuum ;;
    cpmlpt) run cpmlpt --scene vacuum --use-pml --pml-type cpml ;;
    drudecpml) run drudecpml --scene drude-sphere --use-metamaterials --use-pml --pml-type cpml $SPH ;;
    drudecpmlh) run drudecpmlh --scene drude-sphere --use-metamaterials --use-pml --pml-type cpml $SPH --hybrid-block 4 ;;
    drudeh) run drudeh --scene drude-sphere --use-metamaterials --use-pml $SPH --hybrid-block 4 ;;
    vac4) run vac4 --scene vacuum --time-block 4 ;;
    tfsf4) run tfsf4 --scene vacuum --use-tfsf --time-block 4 ;;
    tfsf5) run tfsf5 --scene vacuum --use-tfsf --time-block 5 ;;
  esac || exit 1
done
echo done
