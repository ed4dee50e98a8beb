#!/usr/bin/env python3
"""Per-class timing of the fused single-step shell kernel (yee3d_shell.hip)
on the windows of a 512^3 CPML + TF/SF hybrid plan (GPU; CUDA events)."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme  # noqa: E402
from fdtd3d_amd.ops import make_ops  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    cfg = SchemeConfig(scheme="3d", size=(n, n, n), dtype="f32", pml_size=(10, 10, 10), time_steps=10,
                       scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=True, hybrid_block=5,
                       hybrid_shell="single-pass")
    s = YeeScheme(cfg, make_ops("hip", None, "cuda:0", torch.float32))
    s.init_scheme()
    s.init_grids()
    s.randomize_fields(seed=1)
    hp = s.hybrid
    assert hp is not None and hp.get("v2")
    cur, out = s.F[0], s.F_alt[0]
    cp = s.cpml.host_table(0)
    tot = n ** 3
    pieces = hp["windows"][0]
    by = collections.defaultdict(list)
    for b, a in pieces:
        zl = b[1][2] - b[0][2]
        by[(a, 32 if zl <= 30 else 64)].append((b, a))
    rows = []
    for key in sorted(by):
        ps = by[key]
        cells = sum((b[1][0] - b[0][0]) * (b[1][1] - b[0][1]) * (b[1][2] - b[0][2]) for b, _ in ps)
        ms = timeit(lambda: s.ops.shell_step(cur, out, hp["upd"], [b for b, _ in ps], [a for _, a in ps], s.cb, None,
                                             cpml=cp))
        rows.append((key, len(ps), cells, ms))
        print("class %d lw %d: %2d boxes %9d cells (%.3f) %.4f ms  %.1f Gcells/s  e.g. %s" % (
            key[0], key[1], len(ps), cells, cells / tot, ms, cells / ms / 1e6, ps[0][0]), flush=True)
    ms = timeit(lambda: s.ops.shell_step(cur, out, hp["upd"], [b for b, _ in pieces], [a for _, a in pieces], s.cb,
                                         None, cpml=cp))
    cells = sum(r[2] for r in rows)
    print("all windows of step 1: %.4f ms, %.1f Gcells/s" % (ms, cells / ms / 1e6))
    whole = ((0, 0, 0), (n, n, n))
    for a in (0, 1, 2, 4, 7):
        ms = timeit(lambda: s.ops.shell_step(cur, out, hp["upd"], [whole], [a], s.cb, None, cpml=cp))
        print("whole grid class %d: %.4f ms, %.1f Gcells/s" % (a, ms, tot / ms / 1e6))
    core = hp["core"][0]
    ms = timeit(lambda: s.ops.tb_step(s.F[0], s.F_alt[0], hp["upd"], core, s.cb, 5, None))
    cc = (core[1][0] - core[0][0]) * (core[1][1] - core[0][1]) * (core[1][2] - core[0][2])
    print("core T=5: %.4f ms, %.1f Gcell-steps/s" % (ms, 5 * cc / ms / 1e6))


if __name__ == "__main__":
    main()
