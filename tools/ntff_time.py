#!/usr/bin/env python3
"""Time one NTFF diagram evaluation (models/ntff.py ntff_report) on a 512^3
fp32 grid, after a warm-up evaluation."""
import io
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fdtd3d_amd.models.ntff import ntff_report  # noqa: E402
from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme  # noqa: E402
from fdtd3d_amd.ops import make_ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
cfg = SchemeConfig(scheme="3d", size=(n, n, n), dtype="f32", scene="vacuum", use_fused=True, use_ntff=True,
                   ntff_size=(15, 15, 15))
s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32))
s.init_scheme()
s.init_grids()
s.randomize_fields(seed=1)
for k in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ntff_report(s, 100, out=io.StringIO())
    torch.cuda.synchronize()
    print("ntff_report %.2f ms" % ((time.perf_counter() - t0) * 1e3))
