#!/usr/bin/env python3
"""A/B of a Winograd kernel variant switched by an environment variable (AB_ENV,
e.g. VOSDET_WINO_PF: 0 the product, 1 the variant) at the benched shapes; HIP
events, one process, outputs compared bit for bit and against torch's conv2d.
(Round 4 used it first for the U-in-registers form, profiles/r04/wino_ureg_ab.jsonl,
when the weight order also followed the switch.)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vosdetectron_amd import ops  # noqa: E402

ENV = os.environ["AB_ENV"]


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
                                   (3, 64, 37, 53, False, True), (64, 128, 14, 14, "1d", True),
                                   (40, 64, 7, 7, True, False)]:
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** 0.5
    b = torch.randn(C, device="cuda")
    row = {"shape": [N, C, H, W], "mosaic": mosaic}
    outs = {}
    u = ops.conv3x3_wino_weight(w)
    for v in ("0", "1", "0", "1"):
        os.environ[ENV] = v
        mode = True if mosaic == "1d" else ("2d" if mosaic else False)
        fn = (lambda: ops.conv3x3_wino_bias_act(x, u, b, relu=relu, mosaic=mode)) if mosaic else \
            (lambda: ops.conv3x3_wino_bias_act(x, u, b, relu=relu))
        row.setdefault("ms_" + v, []).append(round(timed(fn), 4))
        outs[v] = fn()
    os.environ.pop(ENV)
    ref = torch.nn.functional.conv2d(x, w, b, padding=1)
    if relu:
        ref = ref.relu()
    row["bit_identical"] = bool(torch.equal(outs["0"], outs["1"]))
    row["max_err_1"] = float((outs["1"] - ref).abs().max())
    print(json.dumps(row), flush=True)
