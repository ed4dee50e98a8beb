#!/bin/bash
# CPML variants: correctness (pass vs stepped, blocked-shell hybrid), micro-benchmark, 512^3 config
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cpml_tb_gpu.py tests/test_hybrid_gpu.py -q --timeout 120 --timeout-method thread -k "hybrid3" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^E " $O/tests.log | cut -c1-300 | head -20
[ $rc -ne 0 ] && exit $rc


C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 40 --json"
for MODE in mixed blocked; do T=$MODE
timeout -k 10 240 python -m fdtd3d_amd $C512 --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-shell $MODE > $O/cfg$T.log 2>&1 || { tail -5 $O/cfg$T.log; exit 1; }
echo "cpml_tfsf T$T $(grep '^{' $O/cfg$T.log | cut -c1-100)"
done
timeout -k 10 240 python -m fdtd3d_amd $C512 --scene vacuum --use-pml --pml-type cpml --hybrid-shell mixed > $O/cfgpt.log 2>&1 || { tail -5 $O/cfgpt.log; exit 1; }
echo "cpml_point mixed $(grep '^{' $O/cfgpt.log | cut -c1-100)"
