#!/usr/bin/env python3
"""Winograd F(2x2,3x3) workgroup form A/B: 32 tiles x 64 channels vs 64 tiles x 32
channels (VOSDET_WINO_T64=0/1), each with its best block shape, on the step's
Winograd shapes; HIP-event ms per call and bit-identity of the two outputs."""
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
    return e0.elapsed_time(e1) / iters


SHAPES = [  # (N, C, Cout, H, W, relu, mosaic): FPN posthoc / RPN / mask head / res convs
    (16, 256, 256, 200, 336, False, False), (16, 256, 256, 200, 336, True, False),
    (16, 256, 256, 100, 168, False, False), (16, 256, 256, 50, 84, True, False),
    (16, 512, 512, 25, 42, True, False), (16, 256, 256, 25, 42, False, False),
    (16, 64, 64, 200, 336, True, False), (16, 128, 128, 100, 168, True, False),
    (16, 256, 256, 50, 84, False, False), (1600, 256, 256, 14, 14, True, True),
]
for N, C, Co, H, W, relu, mosaic in SHAPES:
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (9 * C) ** .5
    b = torch.randn(Co, device="cuda", generator=g)
    u = ops.conv3x3_wino_weight(w)
    rec = {"shape": [N, C, Co, H, W], "relu": relu, "mosaic": mosaic}
    outs = {}
    for t in ("0", "1"):
        os.environ["VOSDET_WINO_T64"] = t
        outs[t] = ops.conv3x3_wino_bias_act(x, u, b, relu=relu, mosaic=mosaic).clone()
        rec["t64_" + t] = round(timed(lambda: ops.conv3x3_wino_bias_act(
            x, u, b, relu=relu, mosaic=mosaic)), 4)
    os.environ.pop("VOSDET_WINO_T64")
    rec["auto"] = round(timed(lambda: ops.conv3x3_wino_bias_act(x, u, b, relu=relu,
                                                               mosaic=mosaic)), 4)
    rec["bit_identical"] = bool(torch.equal(outs["0"], outs["1"]))
    ref = torch.nn.functional.conv2d(x, w, b, padding=1) if not mosaic else None
    if ref is not None:
        if relu:
            ref = ref.clamp_min(0)
        rec["max_abs_err_t64"] = float((outs["1"] - ref).abs().max())
    print(json.dumps(rec), flush=True)
    del x, outs, ref
    torch.cuda.empty_cache()
