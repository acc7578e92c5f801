#!/usr/bin/env python3
"""Mask-head Winograd conv (1600 RoI maps of 14 x 14, 256 -> 256, bias + ReLU):
per-map launch vs the row mosaic (maps stacked, VOSDET_WINO_MOSAIC=1) vs the 2-D
mosaic (8 maps per 112-column row, the default); HIP-event ms per call, alternating."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402

N, C, H, W = int(os.environ.get("MAPS", "1600")), 256, 14, 14
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
w = torch.randn(C, C, 3, 3, device="cuda", generator=g) / (9 * C) ** .5
b = torch.randn(C, device="cuda", generator=g)
u = ops.conv3x3_wino_weight(w)
out = torch.empty_like(x)


def timed(mode, iters=20):
    f = lambda: ops.conv3x3_wino_bias_act(x, u, b, relu=True, out=out, mosaic=mode)  # noqa: E731
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


res = {"maps": N, "per_map": [], "rows": [], "2d": []}
for _ in range(3):
    for k, m in (("per_map", False), ("rows", True), ("2d", "2d")):
        res[k].append(round(timed(m), 4))
print(json.dumps(res), flush=True)
