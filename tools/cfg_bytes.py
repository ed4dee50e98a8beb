#!/usr/bin/env python3
"""HBM bytes per cell-step of a whole driver run from rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE databases of a short and a long run of the same
config: the difference cancels initialisation and warmup, leaving
(long - short) steady-state steps.  Per kernel family and in total.

    python tools/cfg_bytes.py --cells N --steps S_SHORT S_LONG \\
        --fetch short_fetch.db long_fetch.db --write short_write.db long_write.db

FETCH_SIZE on gfx950 counts 128-byte streaming reads at 64 B
(MI355X_MICROARCH.md), so both the raw and the doubled read volume are shown.
"""
import argparse
import sqlite3
from collections import defaultdict


def totals(path, counter):
    c = sqlite3.connect(path)
    out = defaultdict(float)
    for name, val in c.execute("select kernel_name, value from counters_collection where counter_name=?", (counter,)):
        n = name.replace("(anonymous namespace)::", "")
        n = n[5:] if n.startswith("void ") else n
        out[n.split("<")[0].split("(")[0][:48]] += float(val) * 1024.0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=float, required=True)
    ap.add_argument("--steps", type=int, nargs=2, required=True)
    ap.add_argument("--fetch", nargs=2, required=True)
    ap.add_argument("--write", nargs=2, required=True)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    fs, fl = totals(a.fetch[0], "FETCH_SIZE"), totals(a.fetch[1], "FETCH_SIZE")
    ws, wl = totals(a.write[0], "WRITE_SIZE"), totals(a.write[1], "WRITE_SIZE")
    cs = a.cells * (a.steps[1] - a.steps[0])
    rows = []
    for k in sorted(set(fl) | set(wl)):
        r = (fl.get(k, 0.0) - fs.get(k, 0.0)) / cs
        w = (wl.get(k, 0.0) - ws.get(k, 0.0)) / cs
        if abs(r) + abs(w) > 0.005:
            rows.append((k, r, w))
    rows.sort(key=lambda x: -(2 * x[1] + x[2]))
    if a.title:
        print("### %s\n" % a.title)
    print("| kernel family | FETCH B/cell-step | 2xFETCH | WRITE B/cell-step | 2xFETCH + WRITE |")
    print("|---|---:|---:|---:|---:|")
    tr = tw = 0.0
    for k, r, w in rows:
        tr += r
        tw += w
        print("| `%s` | %.2f | %.2f | %.2f | %.2f |" % (k, r, 2 * r, w, 2 * r + w))
    print("| **total** | %.2f | %.2f | %.2f | **%.2f** |" % (tr, 2 * tr, tw, 2 * tr + tw))


if __name__ == "__main__":
    main()
