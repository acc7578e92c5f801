"""Summarise a rocprofv3 rocpd database (``-o run`` -> ``run_results.db``).

The default rocprofv3 output on this image is a SQLite (rocpd) file; this writes the
same per-kernel ``--stats`` table the CSV output has (name, calls, total/avg/min/max
ns, percent) plus the individual launches of one kernel (grid, duration), so the
kernel-trace average can be compared with ``bench.py``'s HIP-event ``avg_launch_us``.

    python tools/rocpd_summary.py run_results.db out_stats.csv \
        --launches sep_kernel out_launches.txt
"""
import argparse
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("stats_csv")
    ap.add_argument("--launches", nargs=2, metavar=("SUBSTR", "OUT"))
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(a.stats_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs",
                    "Percentage"])
        for n, k, s, av, mn, mx in rows:
            w.writerow([n, k, s, f"{av:.1f}", mn, mx, f"{100.0 * s / total:.3f}"])
    if a.launches:
        sub, out = a.launches
        ls = c.execute(
            "select name, grid_x, workgroup_x, lds_size, duration from kernels "
            "where name like ? order by start", (f"%{sub}%",)).fetchall()
        with open(out, "w") as f:
            for n, gx, wx, lds, d in ls:
                f.write(f"{d / 1000.0:9.2f} us  grid {gx:9d}  wg {wx:4d}  lds {lds:6d}  {n}\n")
            by_grid = {}
            for _, gx, _, _, d in ls:
                by_grid.setdefault(gx, []).append(d)
            for gx, ds in sorted(by_grid.items()):
                f.write(f"# grid {gx}: {len(ds)} launches, avg {sum(ds) / len(ds) / 1000.0:.2f} us\n")


if __name__ == "__main__":
    main()
