#!/bin/bash
# Round 6 (al): config 3 with the TF/SF x faces in the shell and the y / z faces in the core (--hybrid-tfsf split)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6al
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hybrid_gpu.py -k "split or core" -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 60 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for r in 1 2; do
  for m in split shell; do
    for T in 5 4; do
      timeout -k 10 200 python3 -m fdtd3d_amd $C --hybrid-tfsf $m --hybrid-block $T > $O/r_${m}_${T}_$r.log 2>&1 || { echo "$m $T failed"; tail -5 $O/r_${m}_${T}_$r.log; exit 1; }
      echo "$m T=$T $(grep -o '"mcells_per_s[^,]*' $O/r_${m}_${T}_$r.log)"
    done
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_al -o run -- python3 -m fdtd3d_amd $C --hybrid-tfsf split --hybrid-block 5 > $O/kt.log 2>&1 && cp /tmp/t_al/run_kernel_stats.csv $O/kt_split_stats.csv || { echo "kt failed"; exit 1; }
echo done
