#!/usr/bin/env python3
"""RoIAlign variant sweep on the §8(d) workload: parity of each variant against
the bit-exact row kernel (variant 3) at 1e-4, then timing.  One process."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from vosdetectron_amd import ops  # noqa: E402


def run(variant, deal, P=7, frames=8, R=1000):
    os.environ["VOSDET_ROIALIGN_VARIANT"] = variant
    r = bench.measure_roialign_roofline(torch.device("cuda"), frames=frames, R=R, P=P, deal=deal)
    return {"variant": variant, "deal": deal, "P": P, "us": r["avg_launch_us"],
            "GBs": r["achieved"], "frac": r["frac"]}


def parity(variant, P=7, R=300):
    dev = torch.device("cuda")
    sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    g = torch.Generator(device=dev).manual_seed(3)
    pyr = [torch.randn((2, h, w, 256), generator=g, device=dev) for h, w in sizes]
    rr = np.concatenate([bench.synthetic_rois(f, R, batch_idx=f) for f in range(2)])
    lv = torch.from_numpy(bench.fpn_levels_np(rr) - 2).to(dev)
    rt = torch.from_numpy(rr).to(dev)
    outs = {}
    for v in ("3", variant):
        os.environ["VOSDET_ROIALIGN_VARIANT"] = v
        order = ops.xcd_roi_order(rt, lv, n_xcd=1 if v == "16" else 8)
        outs[v] = ops.roi_align_fpn(pyr, [1 / 4, 1 / 8, 1 / 16, 1 / 32], rt, lv, P, 2,
                                    roi_order=order, out_layout="nhwc")
    return float((outs["3"] - outs[variant]).abs().max())


if __name__ == "__main__":
    cases = [a.split(":") for a in sys.argv[1:]] or [["8", "8"], ["16", "1"]]
    for v, d in cases:
        for P in (7, 14):
            err = parity(v, P)
            res = run(v, int(d), P=P, R=1000 if P == 7 else 100)
            res["maxerr_vs_v3"] = err
            print(json.dumps(res), flush=True)
