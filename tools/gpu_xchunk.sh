#!/bin/bash
# Blocked-kernel GPU tests, then bench.py at several grid sizes with the automatic x chunk.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tb_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tb.log 2>&1
rc=$?; tail -2 gpurun_out/tb.log; [ $rc -ne 0 ] && exit $rc
val() { python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'])"; }
for sz in "1024 1024 1024" "2048 1024 1024" "512 512 512" "512 512 1024"; do
  v=$(timeout -k 10 150 python bench.py --fp64-companion off --steps 40 --size $sz 2>/dev/null | val) || exit 1
  echo "[$sz] $v"
done
v=$(timeout -k 10 150 python bench.py --fp64-companion off --steps 40 --size 512 512 1024 --tb-xchunk 512 2>/dev/null | val) || exit 1
echo "[512 512 1024, 512-plane chunks] $v"
for args in "" "--tb-xchunk 256" "--tb-xchunk 128"; do
  v=$(timeout -k 10 150 python bench.py --dtype f64 --fp64-companion off --steps 24 $args 2>/dev/null | val) || exit 1
  echo "[f64 1024^3 $args] $v"
done
