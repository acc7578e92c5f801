#!/usr/bin/env python3
"""Per-(kernel, grid) launch statistics from a rocprofv3 --kernel-trace CSV, so
the launches of one kernel at one shape (e.g. bench.py's roofline loop) can be
compared with the HIP-event average bench.py reports.

usage: tools/kernel_breakdown.py run_kernel_trace.csv [name-substring]"""
import collections
import csv
import sys


def main():
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        if pat in r["Kernel_Name"]:
            key = (r["Kernel_Name"][:100], r.get("Grid_Size", r.get("Grid_Size_X", "?")),
                   r.get("Workgroup_Size", r.get("Workgroup_Size_X", "?")))
            g[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print("%-100s %10s %6s %6s %10s %10s %10s" % ("kernel", "grid", "wg", "calls", "avg_us",
                                                 "min_us", "max_us"))
    for (name, grid, wg), d in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        print("%-100s %10s %6s %6d %10.1f %10.1f %10.1f" % (name, grid, wg, len(d),
                                                           sum(d) / len(d) / 1e3, min(d) / 1e3,
                                                           max(d) / 1e3))


if __name__ == "__main__":
    main()
