#!/usr/bin/env python3
"""Steady-state per-step kernel breakdown from a rocprofv3 --kernel-trace CSV of
bench.py: the span between two consecutive launches of the step's first kernel
(image_to_blob) is one step -- the shortest such span among the last ones, so the
bench's own measurement launches after the timed loop stay out; kernels are
aggregated by name.

usage: tools/analyze_trace.py run_kernel_trace.csv [marker] [top]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "image_to_blob"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(idx) < 3:
        print("not enough steps in trace")
        return
    spans = [(int(rows[idx[k + 1]]["Start_Timestamp"]) - int(rows[idx[k]]["Start_Timestamp"]), k)
             for k in range(max(0, len(idx) - 6), len(idx) - 1)]
    k = min(spans)[1]
    a, b = idx[k], idx[k + 1]
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in step:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy += d
        name = r["Kernel_Name"]
        agg[name][0] += d
        agg[name][1] += 1
    print("step wall %.3f ms, kernel busy %.3f ms, %d kernels" % ((t1 - t0) / 1e6, busy / 1e6,
                                                                  len(step)))
    for name, (d, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print("%8.3f ms %5.1f%% n=%4d avg=%8.1fus  %s" % (d / 1e6, 100.0 * d / busy, n,
                                                         d / n / 1e3, name[:110]))


if __name__ == "__main__":
    main()
