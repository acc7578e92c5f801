#!/usr/bin/env python3
"""What the product RoIAlign's dependent prologue (roi_order[p] -> rois[r], level[r])
costs: the bench.py roofline launch with its XCD schedule (a) as shipped and (b) with
rois / levels pre-permuted into schedule order and roi_order = None (same work, same
locality, one dependent load fewer).  HIP-event us per launch, alternating."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import synthetic_rois, fpn_levels_np  # noqa: E402
from vosdetectron_amd import ops  # noqa: E402

dev = torch.device("cuda")
frames, R, C, P, sr = 8, 1000, 256, 7, 2
sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]
g = torch.Generator(device=dev).manual_seed(1)
pyr = [torch.randn((frames, h, w, C), generator=g, device=dev) for h, w in sizes]
rois = np.concatenate([synthetic_rois(f, R, batch_idx=f) for f in range(frames)])
lv = np.concatenate([fpn_levels_np(synthetic_rois(f, R, batch_idx=f)) - 2 for f in range(frames)])
rois_t, lv_t = torch.from_numpy(rois).to(dev), torch.from_numpy(lv).to(dev)
order = ops.xcd_roi_order(rois_t, lv_t, n_xcd=8)
rois_p, lv_p = rois_t[order.long()].contiguous(), lv_t[order.long()].contiguous()
out = torch.empty((frames * R, P, P, C), device=dev)
out_p = torch.empty_like(out)


def run(pre):
    if pre:
        ops.roi_align_fpn(pyr, scales, rois_p, lv_p, P, sr, out=out_p, roi_order=None, out_layout="nhwc")
    else:
        ops.roi_align_fpn(pyr, scales, rois_t, lv_t, P, sr, out=out, roi_order=order, out_layout="nhwc")


def timed(pre, iters=50):
    for _ in range(3):
        run(pre)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        run(pre)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


res = {"shipped_us": [], "prepermuted_us": []}
for _ in range(3):
    res["shipped_us"].append(round(timed(False), 1))
    res["prepermuted_us"].append(round(timed(True), 1))
run(False)
run(True)
torch.cuda.synchronize()
res["same_values"] = bool(torch.equal(out[order.long()], out_p))
print(json.dumps(res), flush=True)
