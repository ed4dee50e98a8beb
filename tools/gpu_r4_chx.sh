#!/bin/bash
# Round 4: A/B of the chain kernel's x planes per thread (FDTD3D_CHAIN_CHX) and the split kernels'
# workgroup target (FDTD3D_SPLIT_WGS) on the UPML configs (Drude + UPML, UPML + TF/SF, 512^3 fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4chx
mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 tools/bench_configs.py --only 3d-512-drude 3d-512-upml-tfsf \
    --out $O/$tag.md > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  echo "== $tag"; cut -d"|" -f2,3 $O/$tag.md | tail -2
}
run base FDTD3D_CHAIN_CHX=8 &&
run chx4 FDTD3D_CHAIN_CHX=4 &&
run chx16 FDTD3D_CHAIN_CHX=16 &&
run chx2 FDTD3D_CHAIN_CHX=2 &&
run wgs4k FDTD3D_SPLIT_WGS=4096 &&
run wgs1k FDTD3D_SPLIT_WGS=1024 &&
run base2 FDTD3D_CHAIN_CHX=8 &&
run chx4b FDTD3D_CHAIN_CHX=4 &&
run chx16b FDTD3D_CHAIN_CHX=16
echo done
