cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 200 python bench.py > gpurun_out/bv.log 2>&1 && python -c 'import json; d=json.loads(open("gpurun_out/bv.log").read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; done
timeout -k 10 200 python bench.py --steps 60 --warmup 10 > gpurun_out/bv.log 2>&1 && python -c 'import json; d=json.loads(open("gpurun_out/bv.log").read().strip().splitlines()[-1]); print("60 steps", d["value"], d["ms_per_step"])'
