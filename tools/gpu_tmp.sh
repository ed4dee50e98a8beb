bash tools/gpu_check.sh && bash tools/gpu_multirank.sh && timeout -k 10 200 python bench.py --steps 23 --warmup 3 > gpurun_out/bench_odd.log 2>&1 && cut -c1-200 gpurun_out/bench_odd.log
