"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs
(rocpd SQLite ``counters_collection``).

    python tools/pmc_summary.py FETCH.db WRITE.db --cells N [--steps-per-call T]

Prints, per kernel: calls, mean duration, FETCH_SIZE and WRITE_SIZE per call,
bytes per cell (per leapfrog step when --steps-per-call is given) and the
implied bandwidth.  On gfx950 FETCH_SIZE counts 128-byte streaming reads at
64 B (MI355X_MICROARCH.md, HBM section), so the corrected read volume is
2 x FETCH_SIZE for wide (16 B/lane) streams; both columns are shown.
"""
import argparse
import sqlite3
from collections import defaultdict


def load(path, counter):
    c = sqlite3.connect(path)
    out = defaultdict(list)
    for name, val, dur in c.execute("select kernel_name, value, duration from counters_collection where counter_name=?",
                                    (counter,)):
        out[name].append((float(val) * 1024.0, float(dur)))
    return out


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--cells", type=float, required=True)
    ap.add_argument("--steps-per-call", type=float, default=1.0)
    ap.add_argument("--min-ms", type=float, default=0.5)
    a = ap.parse_args()
    f, w = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    print("| kernel | calls | mean ms | FETCH_SIZE MB | 2xFETCH MB | WRITE_SIZE MB | read B/cell-step (2xFETCH) "
          "| write B/cell-step | HBM TB/s (2xFETCH + WRITE) |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in f:
        if k not in w:
            continue
        fb = sum(v for v, _ in f[k]) / len(f[k])
        wb = sum(v for v, _ in w[k]) / len(w[k])
        ms = sum(d for _, d in f[k]) / len(f[k]) / 1e6
        if ms < a.min_ms:
            continue
        cs = a.cells * a.steps_per_call
        print("| `%s` | %d | %.3f | %.1f | %.1f | %.1f | %.2f | %.2f | %.2f |" % (
            short(k), len(f[k]), ms, fb / 1e6, 2 * fb / 1e6, wb / 1e6, 2 * fb / cs, wb / cs,
            (2 * fb + wb) / (ms * 1e-3) / 1e12))


if __name__ == "__main__":
    main()
