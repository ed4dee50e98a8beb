#!/bin/bash
# Multi-rank rehearsal on ONE GPU: torchrun with 2 / 4 ranks sharing the
# device, halos over gloo (staged through host).  Checks the decomposed
# blocked path of bench.py end to end (topology, T-deep ghosts, overlap,
# max-over-ranks timing); throughput is not meaningful here.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp FDTD_BENCH_COMM=gloo
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --size 256 256 256 --steps 10 --warmup 5 \
    > gpurun_out/multirank_$n.log 2>&1 || { echo "n=$n failed"; tail -20 gpurun_out/multirank_$n.log; exit 1; }
  echo "n=$n $(grep metric gpurun_out/multirank_$n.log | cut -c1-300)"
done
timeout -k 10 300 python -u -m pytest tests/test_parallel_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_par.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_par.log; exit $rc
