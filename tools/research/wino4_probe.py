#!/usr/bin/env python3
"""F(4x4,3x3) vs F(2x2,3x3) Winograd on the step's 3x3 shapes: HIP-event ms per
call (3 warm-up, 10 timed) and max error vs torch fp32 relative to max|y|; one
JSON line per shape."""
import json
import os
import sys

import torch
import torch.nn.functional as Fn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


SHAPES = [(16, 256, 200, 336, 256), (16, 256, 100, 168, 256), (16, 128, 100, 168, 128),
          (16, 64, 200, 336, 64), (16, 256, 50, 84, 256), (1600, 256, 14, 14, 256)]
for N, C, H, W, Co in SHAPES:
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (9 * C) ** .5
    b = torch.randn(Co, device="cuda", generator=g)
    ref = Fn.conv2d(x, w, b, padding=1)
    rec = {"shape": [N, C, H, W, Co]}
    for name, wf, cf in (("wino2", ops.conv3x3_wino_weight, ops.conv3x3_wino_bias_act),
                         ("wino4", ops.conv3x3_wino4_weight, ops.conv3x3_wino4_bias_act)):
        u = wf(w)
        y = cf(x, u, b)
        err = float((y - ref).abs().max() / ref.abs().max())
        rec[name] = [round(timed(lambda: cf(x, u, b)), 3), "%.1e" % err]
        del y
    print(json.dumps(rec), flush=True)
    del x, ref
    torch.cuda.empty_cache()
