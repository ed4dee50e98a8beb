#!/bin/bash
# CPML variants: correctness (pass vs stepped, blocked-shell hybrid), micro-benchmark, 512^3 config
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cpml_tb_gpu.py tests/test_hybrid_gpu.py -q --timeout 120 --timeout-method thread -k "cpml_pass or hybrid3" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^E " $O/tests.log | cut -c1-300 | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/mr_bench.py --n 512 --rounds 3 > $O/mr.log 2>&1 || { tail -5 $O/mr.log; exit 1; }
grep -v amdgpu.ids $O/mr.log
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 40 --json"
for T in 4; do
timeout -k 10 240 python -m fdtd3d_amd $C512 --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-shell blocked --hybrid-block $T > $O/cfg$T.log 2>&1 || { tail -5 $O/cfg$T.log; exit 1; }
echo "cpml_tfsf T$T $(grep '^{' $O/cfg$T.log | cut -c1-100)"
done
