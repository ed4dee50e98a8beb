"""Summarise a rocprofv3 ``run_results.db`` (rocpd SQLite) into a Markdown
per-kernel table: calls, total / mean / min time, share, and the effective
HBM bandwidth implied by the algorithmic bytes of the FDTD kernels.

    python tools/prof_summary.py gpurun_out/prof/fused/run_results.db --cells 1073741824 > profiles/x.md
"""
import argparse
import sqlite3
import subprocess
import sys

# algorithmic bytes per cell of each kernel family (fp32): reads + writes
BYTES_PER_CELL = {
    "k_fused3d_v4": 48, "k_fused3d": 48,
    # temporally blocked: one read + one write of the 6 fields per T-step pass
    "k_tb3d_v4": 48,
    "k_update_e3d_v4": 36, "k_update_h3d_v4": 36,
    "k_update_e3d": 36, "k_update_h3d": 36,
}


def demangle(name: str) -> str:
    if name.endswith(".kd"):
        name = name[:-3]
    if not name.startswith("_Z"):
        return name
    try:
        return subprocess.run(["c++filt", name], capture_output=True, text=True, timeout=10).stdout.strip() or name
    except (OSError, subprocess.SubprocessError):
        return name


def short(name: str) -> str:
    n = name
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("(anonymous namespace)::", "")
    return n.split("(")[0][:90]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--cells", type=float, default=0.0, help="cells per launch, for GB/s")
    ap.add_argument("--title", default="")
    ap.add_argument("--marker", default="", help="kernel-name substring that starts each pass / step")
    ap.add_argument("--passes", type=int, default=0,
                    help="with --marker: only the kernels between the start of the (passes+1)-th last marker "
                         "launch and the start of the last one (steady-state, init excluded)")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    where = ""
    if a.marker and a.passes > 0:
        names = c.execute("select k.start, coalesce(nullif(k.name, ''), s.kernel_name) from kernels k left join "
                          "kernel_symbols s on s.kernel_id = k.kernel_id order by k.start").fetchall()
        starts = [t for t, n in names if a.marker in demangle(n or "")]
        if len(starts) > a.passes:
            t0, t1 = starts[-a.passes - 1], starts[-1]
            where = " where k.start >= %d and k.start < %d" % (t0, t1)
            sys.stdout.write("window: %d passes, %.3f ms wall, %.3f ms per pass\n\n" % (
                a.passes, (t1 - t0) / 1e6, (t1 - t0) / 1e6 / a.passes))
    rows = c.execute("select coalesce(nullif(k.name, ''), s.kernel_name), count(*), sum(k.duration), "
                     "avg(k.duration), min(k.duration), max(k.vgpr_count), max(k.sgpr_count), max(k.lds_size), "
                     "max(k.scratch_size) from kernels k left join kernel_symbols s on s.kernel_id = k.kernel_id"
                     + where + " group by k.kernel_id order by sum(k.duration) desc").fetchall()
    rows = [(demangle(r[0] or "?"),) + tuple(r[1:]) for r in rows]
    total = sum(r[2] for r in rows) or 1
    out = sys.stdout
    if a.title:
        out.write("## %s\n\n" % a.title)
    out.write("| kernel | calls | total ms | mean ms | min ms | share | VGPR | SGPR | LDS B | scratch B | eff. GB/s |\n")
    out.write("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|\n")
    for name, n, tot, avg, mn, vg, sg, lds, scr in rows:
        s = short(name)
        bw = ""
        for k, b in BYTES_PER_CELL.items():
            if a.cells and (s.startswith(k + "<") or s == k or s.startswith("void " + k)):
                bw = "%.0f" % (a.cells * b / (mn * 1e-9) / 1e9)
                break
        out.write("| `%s` | %d | %.3f | %.4f | %.4f | %.1f%% | %s | %s | %s | %s | %s |\n" % (
            s, n, tot / 1e6, avg / 1e6, mn / 1e6, 100.0 * tot / total, vg, sg, lds, scr, bw))
    return 0


if __name__ == "__main__":
    sys.exit(main())
