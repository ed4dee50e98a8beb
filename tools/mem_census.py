#!/usr/bin/env python3
"""Device-memory census of a scheme: every tensor reachable from the scheme
object (deduplicated by storage), grouped by attribute path, in bytes per
grid cell -- what a capacity plan at 1024^3 has to fit into 288 GB.

  python tools/mem_census.py --3d --sizex 256 --same-size --dtype f32 --scene drude-sphere \
      --use-metamaterials --use-pml --sphere-radius 64 ...   (any runner flags)"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fdtd3d_amd.runner import build  # noqa: E402
from fdtd3d_amd.utils.settings import setup_from_cmd  # noqa: E402


def walk(obj, path, seen, out, depth=0):
    if depth > 8:
        return
    if isinstance(obj, torch.Tensor):
        st = obj.untyped_storage()
        key = st.data_ptr()
        if obj.device.type != "cpu" or os.environ.get("CENSUS_CPU"):
            if key not in seen and st.nbytes() > 0:
                seen.add(key)
                out[path] += st.nbytes()
        return
    oid = id(obj)
    if oid in seen:
        return
    seen.add(oid)
    if isinstance(obj, dict):
        for k, v in obj.items():
            walk(v, path, seen, out, depth + 1)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            walk(v, path, seen, out, depth + 1)
    elif hasattr(obj, "__dict__") and type(obj).__module__.startswith("fdtd3d_amd"):
        for k, v in vars(obj).items():
            walk(v, (path + "." + k) if depth < 2 else path, seen, out, depth + 1)


def main():
    rc, st = setup_from_cmd(sys.argv[1:])
    if rc:
        return rc
    scheme, halo, core = build(st)
    scheme.init_scheme()
    scheme.init_grids()
    scheme.advance(2)
    if scheme.device.type == "cuda":
        torch.cuda.synchronize()
    out = collections.Counter()
    walk(scheme, "scheme", set(), out)
    cells = scheme.cells()
    tot = sum(out.values())
    print("cells %d, tensors reachable: %.2f GB = %.1f B/cell" % (cells, tot / 1e9, tot / cells))
    if scheme.device.type == "cuda":
        print("allocated %.2f GB, peak %.2f GB = %.1f B/cell" % (torch.cuda.memory_allocated() / 1e9,
                                                                  torch.cuda.max_memory_allocated() / 1e9,
                                                                  torch.cuda.max_memory_allocated() / cells))
    for k, v in out.most_common(30):
        print("  %-40s %8.3f GB %7.1f B/cell" % (k, v / 1e9, v / cells))
    return 0


if __name__ == "__main__":
    sys.exit(main())
