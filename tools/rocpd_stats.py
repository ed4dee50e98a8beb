#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 ``--kernel-trace`` database (the rocpd
SQLite file rocprofv3 writes by default): calls, total / mean time, share,
grid and VGPRs, as a markdown table.

    python tools/rocpd_stats.py gpurun_out/r4e/prof_cpml/run_results.db [--top 20] [--last-ms 0]

``--since-ms``: only dispatches that start at least that many ms after the
first one (skips initialisation and warm-up when the timed loop comes last).
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--since-ms", type=float, default=0.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, duration, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z, "
                     "vgpr_count, accum_vgpr_count from kernels order by start").fetchall()
    if not rows:
        print("no kernel dispatches")
        return
    t0 = rows[0][1] + a.since_ms * 1e6
    agg = {}
    for name, start, dur, gx, gy, gz, wx, wy, wz, vg, ag in rows:
        if start < t0:
            continue
        k = short(name)
        e = agg.setdefault(k, [0, 0, 0, vg + ag])
        e[0] += 1
        e[1] += dur
        e[2] = max(e[2], gx * gy * gz // max(1, wx * wy * wz))
    total = sum(v[1] for v in agg.values())
    print("| kernel | calls | total ms | mean us | share | max workgroups | VGPRs |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for k, (n, t, wg, vg) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print("| `%s` | %d | %.3f | %.1f | %.1f%% | %d | %d |" % (k, n, t / 1e6, t / n / 1e3, 100.0 * t / total, wg, vg))
    print("\nall kernels: %.3f ms, %d dispatches" % (total / 1e6, sum(v[0] for v in agg.values())))


if __name__ == "__main__":
    main()
