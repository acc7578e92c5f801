#!/usr/bin/env python3
"""Winograd layouts of a batch of maps on the step's shapes: per-map launch (False)
vs the row mosaic (maps stacked, True) vs the 2-D mosaic ("2d": 16 / gcd(W, 16) maps
per row, odd sides padded to even) -- HIP-event ms per call, alternating, beside the
implicit GEMM (conv3x3_bias_act) and MIOpen, and which layout modeling._pick_mosaic
routes.  Mask head: 1600 RoI maps of 14 x 14; P3 / P4 / res5 / P5 / P6: the 16-frame
batch; C4: the res5 head's 8000 x 7 x 7 RoI maps."""
import torch.nn.functional as F
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402
from vosdetectron_amd.modeling import _pick_mosaic  # noqa: E402

SHAPES = [(1600, 256, 256, 14, 14, True), (16, 256, 256, 100, 168, False),
          (16, 256, 256, 100, 168, True), (16, 128, 128, 100, 168, True),
          (16, 256, 256, 50, 84, True), (16, 256, 256, 50, 84, False),
          (16, 512, 512, 25, 42, True), (16, 256, 256, 25, 42, False),
          (16, 256, 256, 13, 21, False), (8000, 512, 512, 7, 7, True)]
if os.environ.get("ODD_ONLY"):
    SHAPES = SHAPES[6:]


def timed(f, iters=20):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


for N, C, Co, H, W, relu in SHAPES:
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (9 * C) ** .5
    b = torch.randn(Co, device="cuda", generator=g)
    u = ops.conv3x3_wino_weight(w)
    out = torch.empty((N, Co, H, W), device="cuda").contiguous(memory_format=torch.channels_last)
    pm = _pick_mosaic(N, H, W)
    res = {"shape": [N, C, Co, H, W], "relu": relu, "routed": str(pm[0]),
           "block_use": round(pm[1], 3), "per_map": [], "rows": [], "2d": []}
    ref = ops.conv3x3_wino_bias_act(x, u, b, relu=relu).clone()
    for _ in range(3):
        for k, m in (("per_map", False), ("rows", True), ("2d", "2d")):
            if m is True and H % 2:
                continue
            res[k].append(round(timed(lambda: ops.conv3x3_wino_bias_act(
                x, u, b, relu=relu, out=out, mosaic=m)), 4))
            res.setdefault("bit_identical_" + k, True)
            res["bit_identical_" + k] &= bool(torch.equal(out, ref))
    w2 = ops.conv3x3_weight(w)
    res["implicit_gemm"] = round(timed(lambda: ops.conv3x3_bias_act(x, w2, b, relu=relu)), 4)
    res["miopen"] = round(timed(lambda: F.conv2d(x, w, b, padding=1)), 4)
    print(json.dumps(res), flush=True)
    del x, out, ref
    torch.cuda.empty_cache()
