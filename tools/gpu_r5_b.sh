#!/bin/bash
# Round 5: scalar TF/SF fix in the blocked kernel + TF/SF faces in the hybrid core.
# Tests first, then whole-grid vacuum + TF/SF (new kernel vs the round-4 library), the hybrid configs
# (faces in the core vs in the shell), and one PMC group per kernel form.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tfsf_tb_gpu.py tests/test_hybrid_gpu.py -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 10 --time-steps 50 --json"
run() {
  local lab=$1; shift
  timeout -k 10 200 python -m fdtd3d_amd $C "$@" > $O/$lab.log 2>&1 || { echo "$lab failed"; tail -3 $O/$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/$lab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mcells_per_s"]))')"
}
run vac --scene vacuum || exit 1
run vac_tfsf_T4 --scene vacuum --use-tfsf --time-block 4 || exit 1
run vac_tfsf_T5 --scene vacuum --use-tfsf --time-block 5 || exit 1
FDTD3D_HIP_LIB=$PWD/fdtd3d_amd/libfdtd3d_hip_r4.so run vac_tfsf_T4_r4lib --scene vacuum --use-tfsf --time-block 4 || exit 1
run cpml_tfsf --scene vacuum --use-pml --pml-type cpml --use-tfsf || exit 1
run cpml_tfsf_shell --scene vacuum --use-pml --pml-type cpml --use-tfsf --hybrid-tfsf shell || exit 1
run upml_tfsf --scene vacuum --use-pml --use-tfsf || exit 1
run upml_tfsf_shell --scene vacuum --use-pml --use-tfsf --hybrid-tfsf shell || exit 1
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES"
P2="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
CP="--3d --sizex 512 --same-size --dtype f32 --warmup-steps 0 --time-steps 20 --json --time-block 4 --scene vacuum"
pmc() {
  local lab=$1; shift
  local n=0
  for P in "$P1" "$P2"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$lab/p$n -o run -- python3 -m fdtd3d_amd $CP "$@" > $O/pmc_$lab.p$n.log 2>&1 || { echo "pmc $lab p$n failed"; tail -3 $O/pmc_$lab.p$n.log; }
  done
}
pmc plain
pmc tfsf --use-tfsf
FDTD3D_HIP_LIB=$PWD/fdtd3d_amd/libfdtd3d_hip_r4.so pmc tfsf_r4 --use-tfsf
echo done
