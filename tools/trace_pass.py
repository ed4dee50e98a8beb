#!/usr/bin/env python3
"""Print the kernels of one hybrid pass from a rocprofv3 kernel trace (csv):
the window between the last two launches of the blocked core kernel
(``k_tb3d_mr<..., 0, ...>``), with start offset, duration and stream, plus a
per-kernel-name summary of that window.

    python tools/trace_pass.py run_kernel_trace.csv [--which -2]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--which", type=int, default=-2, help="pass index among the core launches (default: the last full one)")
    ap.add_argument("--core", default="k_tb3d_mr<4, 1, 2, 0,")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "?"))
                 for r in rows), key=lambda x: x[0])
    cores = [i for i, k in enumerate(ks) if a.core in k[2]]
    i0, i1 = cores[a.which - 1], cores[a.which]
    t0 = ks[i0][0]
    win = ks[i0:i1]
    print("pass: %.1f us (%d kernels)" % ((ks[i1][0] - t0) / 1e3, len(win)))
    busy = collections.defaultdict(float)
    cnt = collections.Counter()
    for s, e, n, st in win:
        short = n[5:] if n.startswith("void ") else n
        short = short.replace("(anonymous namespace)::", "")
        short = short[:short.find(">(") + 1 if ">(" in short else 70][:80]
        busy[short] += (e - s) / 1e3
        cnt[short] += 1
        if a.list:
            print("%9.1f %8.1f %s %s" % ((s - t0) / 1e3, (e - s) / 1e3, st, short))
    for n, v in sorted(busy.items(), key=lambda x: -x[1]):
        print("%5d %9.1f us %s" % (cnt[n], v, n))
    # union of busy intervals (any stream)
    iv = sorted((s, e) for s, e, _, _ in win)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    print("GPU busy (union): %.1f us" % (tot / 1e3))


if __name__ == "__main__":
    main()
