set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python tools/bench_configs.py --out gpurun_out/configs_all.md > gpurun_out/configs_all.log 2>&1; echo rc=$?
timeout -k 10 300 python bench.py --size 2048 1024 1024 --steps 20 --warmup 5 > gpurun_out/bench_2048.log 2>&1; echo rc=$?
cut -c1-240 gpurun_out/bench_2048.log
cut -c1-110 gpurun_out/configs_all.md
