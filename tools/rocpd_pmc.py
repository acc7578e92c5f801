#!/usr/bin/env python3
"""Per-dispatch counter averages from rocprofv3 --pmc rocpd databases (the image's
default output, ``-o run`` -> ``run_results.db``), one database per pass, for the
kernels whose name contains FILTER.  usage: tools/rocpd_pmc.py FILTER OUT.json DB..."""
import json
import sqlite3
import sys


def main():
    filt, out, dbs = sys.argv[1], sys.argv[2], sys.argv[3:]
    cnt = {}
    for db in dbs:
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
        kcol = "kernel_name" if "kernel_name" in cols else "name"
        per = {}
        for disp, name, val in c.execute(
                "select dispatch_id, counter_name, value from counters_collection "
                "where %s like ?" % kcol, ("%" + filt + "%",)):
            per[(disp, name)] = per.get((disp, name), 0.0) + float(val)
        byname = {}
        for (_, name), v in per.items():
            byname.setdefault(name, []).append(v)
        for name, vs in byname.items():
            cnt[name] = sum(vs) / len(vs)
    rec = {"kernel_filter": filt, "counters": cnt}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in cnt and "SQ_BUSY_CYCLES" in cnt and "GRBM_GUI_ACTIVE" in cnt:
        # GRBM_GUI_ACTIVE sums the 8 XCDs; MFMA busy counts SIMD-cycles (1024 SIMDs)
        rec["mfma_busy_frac"] = cnt["SQ_VALU_MFMA_BUSY_CYCLES"] / (cnt["GRBM_GUI_ACTIVE"] / 8 * 1024)
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
