#!/usr/bin/env python3
"""Mask-head 3x3 convs (R RoI maps of 14 x 14, 256 -> 256, bias + ReLU): F(2x2) on
its 2-D mosaic (the engine's route) vs F(4x4) with two maps per block
(vd_conv3x3_wino4_mosaic_bias_act); HIP-event us per call.  usage:
tools/bench_wino4_mosaic.py [R ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for R in [int(a) for a in sys.argv[1:]] or [3200, 1600]:
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(R, 256, 14, 14, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(256, 256, 3, 3, device="cuda", generator=g) / 48.
    b = torch.randn(256, device="cuda", generator=g)
    u2, u4 = ops.conv3x3_wino_weight(w), ops.conv3x3_wino4_weight(w)
    y = torch.empty_like(x)
    t2 = timed(lambda: ops.conv3x3_wino_bias_act(x, u2, b, relu=True, mosaic="2d", out=y))
    t4 = timed(lambda: ops.conv3x3_wino4_bias_act(x, u4, b, relu=True, mosaic=True, out=y))
    print(json.dumps({"R": R, "wino2_2d_us": round(t2, 1), "wino4_pair_us": round(t4, 1)}),
          flush=True)
