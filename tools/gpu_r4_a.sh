#!/bin/bash
# Round 4 baseline: bench.py (headline + fp64 + physics companions), then the
# phase breakdown of 512^3 CPML + TF/SF.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json"
timeout -k 10 240 python -m fdtd3d_amd $C512 --scene vacuum --use-pml --pml-type cpml --use-tfsf --profile-phases > $O/cpml_tfsf_phases.log 2>&1 || { tail -5 $O/cpml_tfsf_phases.log; exit 1; }
tail -30 $O/cpml_tfsf_phases.log
