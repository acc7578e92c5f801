#!/usr/bin/env python3
"""A/B of the Winograd kernel's patch path (VOSDET_WINO_RPF): LDS-DMA one chunk
ahead (0, the product) vs global loads into registers two chunks ahead (1), at the
benched shapes; HIP events, one process, outputs compared bit for bit."""
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


rec = []
for (N, C, H, W, mosaic) in [(16, 256, 200, 336, False), (16, 256, 100, 168, True),
                             (16, 128, 100, 168, True), (1600, 256, 14, 14, True),
                             (16, 64, 200, 336, False), (16, 512, 25, 42, True)]:
    x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    u = ops.conv3x3_wino_weight(torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** 0.5)
    b = torch.randn(C, device="cuda")
    fn = (lambda: ops.conv3x3_wino_bias_act(x, u, b, mosaic="2d")) if mosaic else \
        (lambda: ops.conv3x3_wino_bias_act(x, u, b))
    row = {"shape": [N, C, H, W], "mosaic": mosaic}
    outs = {}
    for rpf in ("0", "1", "0", "1"):
        os.environ["VOSDET_WINO_RPF"] = rpf
        row.setdefault("ms_rpf" + rpf, []).append(round(timed(fn), 4))
        outs[rpf] = fn()
    row["bit_identical"] = bool(torch.equal(outs["0"], outs["1"]))
    rec.append(row)
    print(json.dumps(row), flush=True)
