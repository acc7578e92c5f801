#!/usr/bin/env python3
"""Where the register-gather RoIAlign (variant 10) spends its time: the same
8-frame x 1000-RoI launch with (a) 8 distinct frames (HBM), (b) every RoI on
frame 0 (the frame's 91 MB pyramid stays in the Infinity Cache), (c) one RoI
of each level repeated (footprints L2-resident).  Same kernel, same number of
wave loads per RoI class; prints us per launch for each."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import fpn_levels_np, synthetic_rois  # noqa: E402
from vosdetectron_amd import ops  # noqa: E402


def run(rois_np, pyr, scales, P=7, iters=30):
    dev = pyr[0].device
    lv = fpn_levels_np(rois_np) - 2
    rt = torch.from_numpy(rois_np).to(dev)
    lt = torch.from_numpy(lv.astype(np.int32)).to(dev)
    order = ops.xcd_roi_order(rt, lt)
    out = torch.empty((len(rois_np), P, P, 256), device=dev)
    f = lambda: ops.roi_align_fpn(pyr, scales, rt, lt, P, 2, roi_order=order, out=out,
                                  out_layout="nhwc")
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


if __name__ == "__main__":
    dev = torch.device("cuda")
    sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]
    g = torch.Generator(device=dev).manual_seed(1)
    pyr = [torch.randn((8, h, w, 256), generator=g, device=dev) for h, w in sizes]
    base = np.concatenate([synthetic_rois(f, 1000, batch_idx=f) for f in range(8)])
    res = {"a_8_frames": run(base, pyr, scales)}
    b = base.copy()
    b[:, 0] = 0
    res["b_frame0_mall"] = run(b, pyr, scales)
    c = base.copy()  # keep each RoI's size, move it to one of 4 spots per level
    w, h = c[:, 3] - c[:, 1], c[:, 4] - c[:, 2]
    c[:, 1], c[:, 2] = 100.0, 100.0
    c[:, 3], c[:, 4] = 100.0 + w, 100.0 + h
    c[:, 0] = 0
    res["c_l2_resident"] = run(c, pyr, scales)
    print(json.dumps({k: round(v, 1) for k, v in res.items()}))
