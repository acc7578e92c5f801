#!/usr/bin/env python3
"""MFMA busy share of one steady-state bench step from a rocprofv3 --pmc
counter CSV (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE): the
dispatches from the last image_to_blob launch on, summed per counter and per
kernel family.  MFMA utilisation = MFMA busy cycles / (kernel time x clock x
1024 SIMDs).  usage: tools/pmc_step_mfma.py run_counter_collection.csv [clock_GHz]"""
import collections
import csv
import json
import sys


def family(name):
    n = name.lower()
    if "conv" in n or "igemm" in n or "cijk" in n or "gemm" in n:
        return "conv/gemm (MIOpen, CK, hipBLASLt)"
    if "vd::" in n:
        return "vd:: HIP kernels"
    return "other"


def main():
    path = sys.argv[1]
    ghz = float(sys.argv[2]) if len(sys.argv) > 2 else 2.4
    disp = {}
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        disp[d] = (r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        vals[(d, r["Counter_Name"])] += float(r["Counter_Value"])
    order = sorted(disp, key=lambda d: disp[d][1])
    marks = [i for i, d in enumerate(order) if "image_to_blob" in disp[order[i]][0]]
    step = order[marks[-1]:] if marks else order
    fam = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in step:
        name, t0, t1 = disp[d]
        f = fam[family(name)]
        f["kernel_us"] += (t1 - t0) / 1e3
        f["dispatches"] += 1
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            f[c] += vals.get((d, c), 0.)
    out = {}
    for k, f in fam.items():
        cyc = f["kernel_us"] * 1e-6 * ghz * 1e9 * 1024
        out[k] = dict(f, mfma_util=f["SQ_VALU_MFMA_BUSY_CYCLES"] / cyc if cyc else 0.)
    step_us = disp[step[-1]][2] / 1e3 - disp[step[0]][1] / 1e3
    print(json.dumps({"step_span_us": step_us, "clock_GHz": ghz, "families": out}, indent=1))


if __name__ == "__main__":
    main()
