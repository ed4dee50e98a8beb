#!/bin/bash
# Round 4: native driver 2D PML / TF/SF, amplitude mode and x-slab parallel grids (parity tests), then
# per-kernel rocprof stats of the two physics companions (512^3 CPML + TF/SF, Drude sphere + UPML)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 240 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C512="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 40 --json"
SPH="--sphere-center-x 256 --sphere-center-y 256 --sphere-center-z 256 --sphere-radius 128"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cpml -o run -- python3 -m fdtd3d_amd $C512 \
  --scene vacuum --use-pml --pml-type cpml --use-tfsf > $O/prof_cpml.log 2>&1 || { echo "prof cpml failed"; tail -5 $O/prof_cpml.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_drude -o run -- python3 -m fdtd3d_amd $C512 \
  --scene drude-sphere --use-metamaterials --use-pml $SPH > $O/prof_drude.log 2>&1 || { echo "prof drude failed"; tail -5 $O/prof_drude.log; exit 1; }
for p in cpml drude; do
  db=$(ls $O/prof_$p/*.db 2>/dev/null | head -1)
  [ -n "$db" ] && python3 tools/rocpd_stats.py "$db" --top 25 > $O/stats_$p.md 2>&1
  grep -h '^{' $O/prof_$p.log | tail -1
done
timeout -k 10 120 ./fdtd3d_amd/fdtd3d --3d --sizex 1024 --same-size --dtype f32 --time-steps 25 --warmup-steps 5 \
  --scene vacuum --parallel-grid --topology-sizex 4 > $O/native_multi.log 2>&1 || { echo "native multi failed"; tail -5 $O/native_multi.log; exit 1; }
grep -E "Throughput|processes" $O/native_multi.log
echo done
