#!/usr/bin/env python3
"""Average PMC counters per dispatch of one kernel over the passes written by
tools/prof_roialign.sh (one sub-directory per counter group).

usage: tools/pmc_summary.py OUTDIR [kernel-substring] [out.json]
FETCH_SIZE is doubled for gfx950 (MI355X guide, HBM section: it reports half the
bytes of 16 B/lane streaming reads); FETCH_SIZE/WRITE_SIZE are in KiB."""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "roi_align"
    vals = collections.defaultdict(list)
    durs = []
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for (d, name), v in per.items():
            vals[name].append(v)
    out = {}
    for name, v in sorted(vals.items()):
        out[name] = sum(v) / len(v)
        print("%-32s %16.1f  (n=%d)" % (name, out[name], len(v)))
    if "FETCH_SIZE" in out:
        print("HBM-side read bytes/dispatch (FETCH_SIZE x2, KiB->B): %.3e" % (out["FETCH_SIZE"] * 2048))
    if "WRITE_SIZE" in out:
        print("write bytes/dispatch: %.3e" % (out["WRITE_SIZE"] * 1024))
    if "TCC_HIT_sum" in out and "TCC_MISS_sum" in out:
        print("L2 hit rate: %.3f" % (out["TCC_HIT_sum"] / (out["TCC_HIT_sum"] + out["TCC_MISS_sum"])))
    if durs:
        print("avg dispatch duration under counters: %.1f us" % (sum(durs) / len(durs) / 1e3))
    if len(sys.argv) > 3:  # JSON record for bench.py's roofline "traffic"
        import json
        rec = {"kernel_filter": pat, "counters": out,
               "read_bytes": out.get("FETCH_SIZE", 0) * 2048,
               "write_bytes": out.get("WRITE_SIZE", 0) * 1024,
               "correction": "FETCH_SIZE x2 (gfx950 half-count of 16 B/lane reads), KiB -> B"}
        rec["traffic_bytes"] = rec["read_bytes"] + rec["write_bytes"]
        json.dump(rec, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
