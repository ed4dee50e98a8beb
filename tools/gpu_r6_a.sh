#!/bin/bash
# Round 6 (a): real RCCL self-exchange test, decomposed UPML + TF/SF hybrid case, config 3 kernel traces with the
# TF/SF faces in the core vs in the shell, and the per-GPU cost of 1024^3 rank grids (loopback)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py tests/test_parallel_gpu.py -k "rccl or upml_tfsf or upml-tfsf" \
  -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
# fp64 CPML on the double4 fused kernels (Python hybrid / stepped, native stepped)
timeout -k 10 500 python -u -m pytest tests/test_hip_gpu.py tests/test_hybrid_gpu.py tests/test_native_gpu.py \
  -k "cpml and (f64 or fused)" -v --timeout 240 --timeout-method thread > $O/tests64.log 2>&1 || { echo tests64 failed; tail -40 $O/tests64.log; exit 1; }
grep -E "passed|failed" $O/tests64.log | tail -3
C64="--3d --sizex 512 --same-size --dtype f64 --warmup-steps 8 --time-steps 24 --json --scene vacuum --use-pml --use-tfsf"
for m in cpml upml; do
  timeout -k 10 200 python3 -m fdtd3d_amd $C64 --pml-type $m > $O/rate64_$m.log 2>&1 || { echo "rate64 $m failed"; tail -5 $O/rate64_$m.log; exit 1; }
  echo "== f64 $m + TF/SF"; grep -o '"mcells_per_s[^,]*' $O/rate64_$m.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_64 -o run -- python3 -m fdtd3d_amd $C64 --pml-type cpml > $O/kt64.log 2>&1 && cp /tmp/t_64/run_kernel_stats.csv $O/kt64_cpml_stats.csv || { echo "kt64 failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_64u -o run -- python3 -m fdtd3d_amd $C64 --pml-type upml > $O/kt64u.log 2>&1 && cp /tmp/t_64u/run_kernel_stats.csv $O/kt64_upml_stats.csv || { echo "kt64u failed"; exit 1; }
D="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 8 --time-steps 24 --json --scene drude-sphere --use-metamaterials --use-pml --sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_du -o run -- python3 -m fdtd3d_amd $D > $O/ktdu.log 2>&1 && cp /tmp/t_du/run_kernel_stats.csv $O/kt_drude_upml_stats.csv || { echo "ktdu failed"; exit 1; }
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 30 --json --scene vacuum --use-pml --pml-type cpml --use-tfsf"
for m in core shell; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_$m -o run -- python3 -m fdtd3d_amd $C --hybrid-tfsf $m > $O/kt_$m.log 2>&1 && cp /tmp/t_$m/run_kernel_stats.csv $O/kt_${m}_stats.csv || { echo "kt $m failed"; tail -5 $O/kt_$m.log; exit 1; }
  timeout -k 10 200 python3 -m fdtd3d_amd $C --hybrid-tfsf $m > $O/rate_$m.log 2>&1 || { echo "rate $m failed"; exit 1; }
  echo "== $m"; grep -o '"mcells_per_s[^,]*' $O/rate_$m.log
done
for t in "8_421:--world 8 --topology 4 2 1" "8_241:--world 8 --topology 2 4 1" "8_222:--world 8 --topology 2 2 2" "8_811:--world 8 --topology 8 1 1" "4_221:--world 4 --topology 2 2 1" "4_411:--world 4 --topology 4 1 1" "2_211:--world 2 --topology 2 1 1"; do
  lab=${t%%:*}; args=${t#*:}
  for T in 4 5; do
    timeout -k 10 240 python -u tools/decomp_cost.py --size 1024 1024 1024 $args --time-block $T --transport loopback --link-gbs 50 > $O/${lab}_T$T.log 2>&1 || { echo $lab failed; tail -5 $O/${lab}_T$T.log; exit 1; }
    echo "== $lab T=$T"; grep -h "per pass\|decomposed" $O/${lab}_T$T.log
  done
done
