#!/usr/bin/env python3
"""Per-kernel table from one rocprofv3 --pmc rocpd database: for every kernel name
(first 90 characters), dispatches, mean duration, LDS bank-conflict share of the
LDS-array cycles, MFMA busy share of the SIMD-cycles (GRBM_GUI_ACTIVE / 8 x 1024
SIMDs), wait share of the wave-cycles.  usage: tools/rocpd_pmc_table.py DB OUT.json"""
import json
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = {}
    for disp, kname, cname, val, dur in c.execute(
            "select dispatch_id, kernel_name, counter_name, value, duration "
            "from counters_collection"):
        k = rows.setdefault(kname[:90], {"dispatches": set(), "dur": {}, "c": {}})
        k["dispatches"].add(disp)
        k["dur"][disp] = dur
        k["c"][cname] = k["c"].get(cname, 0.0) + float(val)
    table = []
    for name, k in rows.items():
        n = len(k["dispatches"])
        cc = {a: b / n for a, b in k["c"].items()}
        rec = {"kernel": name, "dispatches": n,
               "mean_us": sum(k["dur"].values()) / n / 1e3}
        if cc.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_conflict_share"] = round(cc.get("SQ_LDS_BANK_CONFLICT", 0) /
                                              cc["SQ_LDS_IDX_ACTIVE"], 3)
        if cc.get("GRBM_GUI_ACTIVE"):
            rec["mfma_busy"] = round(cc.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) /
                                     (cc["GRBM_GUI_ACTIVE"] / 8 * 1024), 3)
        if cc.get("SQ_WAVE_CYCLES"):
            rec["wait_share"] = round(cc.get("SQ_WAIT_ANY", 0) / cc["SQ_WAVE_CYCLES"], 3)
        rec["counters"] = cc
        table.append(rec)
    table.sort(key=lambda r: -r["mean_us"] * r["dispatches"])
    json.dump(table, open(out, "w"), indent=1)
    for r in table[:40]:
        print("%9.1f us x%-4d conflict %-6s mfma %-6s wait %-6s %s" % (
            r["mean_us"], r["dispatches"], r.get("lds_conflict_share"), r.get("mfma_busy"),
            r.get("wait_share"), r["kernel"][:80]))


if __name__ == "__main__":
    main()
