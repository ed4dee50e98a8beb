#!/bin/bash
# kernel trace of the blocked-shell CPML + TF/SF run at 512^3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 40 --json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m fdtd3d_amd $C512 --scene vacuum --use-pml --pml-type cpml --use-tfsf ${EXTRA:---hybrid-shell mixed} > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | cut -c1-200
python3 tools/prof_summary.py $(find $O/prof -name "*results.db" | head -1) > $O/prof.md 2>&1; head -16 $O/prof.md | cut -c1-120

rm -rf $O/prof
true
