#!/usr/bin/env python3
"""F(2x2,3x3) Winograd: block -> (channel block, spatial block) mapping A/B
(VOSDET_WINO_MAP 0: the Cout/64 channel blocks of a spatial block on one XCD;
1: XCD x computes channel block x % ncb) on the step's 3x3 shapes, HIP-event ms
per call, bit-identical outputs checked.  One JSON line per shape."""
import json
import os
import sys

import torch

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


for N, C, H, W, Co in [(16, 256, 200, 336, 256), (16, 256, 100, 168, 256),
                       (16, 128, 100, 168, 128), (16, 64, 200, 336, 64),
                       (16, 256, 50, 84, 256), (1600, 256, 14, 14, 256)]:
    x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    u = ops.conv3x3_wino_weight(torch.randn(Co, C, 3, 3, device="cuda") / (9 * C) ** .5)
    rec, outs = {"shape": [N, C, H, W, Co]}, {}
    for m in ("0", "1"):
        os.environ["VOSDET_WINO_MAP"] = m
        outs[m] = ops.conv3x3_wino_bias_act(x, u, None).clone()
        rec["map" + m] = round(timed(lambda: ops.conv3x3_wino_bias_act(x, u, None)), 3)
    rec["identical"] = bool(torch.equal(outs["0"], outs["1"]))
    print(json.dumps(rec), flush=True)
    del x, outs
    torch.cuda.empty_cache()
