#!/usr/bin/env python3
"""A/B of the Winograd kernel's U operand path (VOSDET_WINO_UREG): LDS-DMA of the
U slice one chunk ahead, read back from LDS (0, the product) vs U fragments loaded
straight into registers one chunk ahead in their own weight order (1); HIP events,
one process, outputs compared bit for bit."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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


for (N, C, H, W, mosaic, relu) in [(16, 256, 200, 336, False, False), (16, 256, 100, 168, True, True),
                                   (16, 128, 100, 168, True, True), (1600, 256, 14, 14, True, True),
                                   (16, 64, 200, 336, False, True), (16, 512, 25, 42, True, True),
                                   (3, 64, 37, 53, False, True)]:
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** 0.5
    b = torch.randn(C, device="cuda")
    row = {"shape": [N, C, H, W], "mosaic": mosaic}
    outs, us = {}, {}
    for v in ("0", "1"):
        os.environ["VOSDET_WINO_UREG"] = v
        us[v] = ops.conv3x3_wino_weight(w)
    for v in ("0", "1", "0", "1"):
        os.environ["VOSDET_WINO_UREG"] = v
        u = us[v]
        fn = (lambda: ops.conv3x3_wino_bias_act(x, u, b, relu=relu, mosaic="2d")) if mosaic else \
            (lambda: ops.conv3x3_wino_bias_act(x, u, b, relu=relu))
        row.setdefault("ms_ureg" + v, []).append(round(timed(fn), 4))
        outs[v] = fn()
    os.environ.pop("VOSDET_WINO_UREG")
    ref = torch.nn.functional.conv2d(x, w, b, padding=1)
    if relu:
        ref = ref.relu()
    row["bit_identical"] = bool(torch.equal(outs["0"], outs["1"]))
    row["max_err_ureg1"] = float((outs["1"] - ref).abs().max())
    print(json.dumps(row), flush=True)
