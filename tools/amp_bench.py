#!/usr/bin/env python3
"""Amplitude (steady-state) mode against plain stepping at N^3 (GPU):
ms per step of ``perform_amplitude_steps`` (split E/H steps + the device-side
amplitude update, counts read once per K steps), of the same per-step
stepping without the amplitude work, and of the automatic (blocked) plain
run."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme  # noqa: E402
from fdtd3d_amd.ops import make_ops  # noqa: E402


def mk(cfg):
    s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32 if cfg.dtype == "f32" else torch.float64))
    s.init_scheme()
    s.init_grids()
    return s


def timed(fn, steps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    dt = sys.argv[3] if len(sys.argv) > 3 else "f32"
    base = dict(scheme="3d", size=(n, n, n), dtype=dt, scene="vacuum", time_steps=steps)
    import fdtd3d_amd.models.scheme as sch
    rows = []
    for T in (1, 2, 3):
        # T = 1: per-step stepping + the separate amplitude kernel; T > 1:
        # blocked passes with the amplitude update folded in (tb3d_mr.h AmpDev)
        sch.AMP_TB_STEPS = T
        for K in ((1, 8, 32) if T == 1 else (8, 32)):
            s = mk(SchemeConfig(use_amp_mode=True, amplitude_steps=steps, amplitude_check_steps=K, **base))
            s.cfg.amplitude_steps = 12
            s.perform_amplitude_steps()  # warm-up
            s.cfg.amplitude_steps = steps
            ms = timed(s.perform_amplitude_steps, steps)
            rows.append(("amplitude mode, %s, check every %d steps"
                         % ("per-step" if T == 1 else "blocked T = %d" % T, K), ms))
            del s
    sch.AMP_TB_STEPS = 3
    s = mk(SchemeConfig(use_amp_mode=True, **base))
    s.advance(5)
    ms = timed(lambda: s.advance(steps), steps)
    rows.append(("same per-step stepping, no amplitude work", ms))
    for tb, name in ((1, "plain per-step (fused E+H kernel)"), (0, "plain automatic (blocked passes)")):
        s = mk(SchemeConfig(use_fused=True, time_block=tb, **dict(base, time_steps=steps)))
        s.advance(10)
        ms = timed(lambda: s.advance(steps), steps)
        rows.append((name, ms))
    cells = n ** 3
    print("| %d^3 %s | ms / step | Mcells/s |" % (n, dt))
    print("|---|---:|---:|")
    for name, ms in rows:
        print("| %s | %.3f | %.0f |" % (name, ms, cells / ms / 1e3))


if __name__ == "__main__":
    main()
