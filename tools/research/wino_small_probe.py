#!/usr/bin/env python3
"""Winograd F(2x2,3x3) with either block shape (VOSDET_WINO_SQ 0: 4 x 32 pixels,
1: 8 x 16) vs MIOpen (F.conv2d, channels_last) on the small-map 3x3 shapes that
stay on MIOpen / CK in the step (res5 conv2, FPN P5); HIP-event ms per call."""
import json
import os
import sys

import torch
import torch.nn.functional as Fn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402

torch.backends.cudnn.benchmark = True


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


for N, C, H, W in [(16, 512, 25, 42), (16, 256, 25, 42), (16, 256, 50, 84), (16, 256, 13, 21),
                   (8, 512, 25, 42), (16, 256, 100, 168)]:
    x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** .5
    b = torch.randn(C, device="cuda")
    u = ops.conv3x3_wino_weight(w)
    rec = {"shape": [N, C, H, W], "miopen": round(timed(lambda: Fn.conv2d(x, w, b, padding=1)), 4)}
    for sq in ("0", "1"):
        os.environ["VOSDET_WINO_SQ"] = sq
        rec["wino_sq" + sq] = round(timed(lambda: ops.conv3x3_wino_bias_act(x, u, b)), 4)
    os.environ.pop("VOSDET_WINO_SQ")
    print(json.dumps(rec), flush=True)
