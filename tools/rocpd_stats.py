#!/usr/bin/env python3
"""Per-kernel summary (name, calls, total/avg us (top_kernels view units), %) from a rocprofv3 SQLite
results database (the default output format of `rocprofv3 --kernel-trace
--stats -o run`), written as the same CSV columns as --output-format csv's
kernel_stats.csv.  usage: tools/rocpd_stats.py run_results.db out.csv"""
import csv
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    rows = con.execute("select name, total_calls, total_duration, average, percentage "
                       "from top_kernels order by total_duration desc").fetchall()
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for r in rows:
            w.writerow([r[0], int(r[1]), int(r[2]), round(float(r[3]), 3), round(float(r[4]), 4)])


if __name__ == "__main__":
    main()
